// Fused DiffSVC residual layer for gfx950: dilated conv + gate + residual half of the output projection + the
// split-fp16 residual update in ONE launch, 128 rows per workgroup (modules/diffsvc.py:212-232).
//
// Per 128-row tile, one 512-thread workgroup (8 waves = 2 (M) x 4 (N)) per CU, 160 KiB of LDS:
//   GEMM1  y = x[t-d | t | t+d] (128 x 1152) . W_dil (1152 x 768): three passes of 256 packed columns (128 channels,
//          groups of [32 gate | 32 filter]); wave tile 64 x 64 as conv_gemm4 (the gate and filter column of a channel in
//          one lane, MFMA operands swapped), 16 v_mfma_f32_16x16x32_f16 per wave per 32-deep K-step, a 4-slot LDS ring
//          (A 128 x 64 B + B 256 x 64 B = 24 KiB per slot) filled by LDS-DMA three K-steps ahead and run as ONE 108-step
//          stream over the three passes (the next pass's first K-steps land under the previous pass's gate epilogue);
//   gate   g = sigmoid(y_gate + b + cp) * tanh(y_filter + b + cp) in registers after each pass (conv_gemm4's register
//          gate epilogue) into an LDS image of the tile's gate output (3 x 32 KiB, channel-chunk-major), GEMM2's A
//          operand; it reaches HBM (the skip-sum GEMM's layer block) only after GEMM2, in whole 16-B row chunks;
//   GEMM2  r = g (128 x 384, from LDS) . W_res (384 x 384): W_res streamed through two ring slots, 24 MFMAs per wave per
//          K-step (wave tile 64 x 96);
//   update x' = ((hi + lo) - dproj_i + r + b_res) / sqrt(2); hi' = f16(x' + dproj_{i+1}), lo' = f16(x' + dproj_{i+1} - hi')
//          from registers, conv_gemm4's register residual epilogue (same operation order).
// The gate GEMM of the unfused path re-reads the layer input rows t +- d of NEIGHBOURING tiles, so the fused kernel
// cannot update the residual stream's hi half in place: it reads hi from one buffer and writes the other (lo, read
// and written only by the row's own tile, stays in place).
// Both GEMMs keep the unfused path's K order (32-deep K-steps in ascending K) and MFMA operand order, and the epilogues
// are the same expressions, so the layer is bit-identical to conv_gemm4 (gate) + conv_gemm4 (register residual update).
// Opt-in (tuning diff_fused): 118-125 us per full-batch layer against 71 + 42 us for the two kernels, because with one
// workgroup per CU the per-tile epilogue traffic (cp 46 MB, residual 92 MB per layer) runs as an un-overlapped burst
// (DESIGN.md "Fused residual layer, round 2"; tuning diff_dbg splits the time).
#include <type_traits>
#include <utility>

#include "common.h"

namespace svc {

constexpr int DL_BM = 128, DL_NT = 512, DL_C = 384;
constexpr int DL_KS1 = 3 * DL_C / 32;  // 36 K-steps per GEMM1 pass (3 taps x 384 channels)
constexpr int DL_S1 = 3 * DL_KS1;      // 108 K-steps over the three passes
constexpr int DL_KS2 = DL_C / 32;      // 12 K-steps of GEMM2
constexpr int DL_GCHUNK = DL_BM * 256;           // one pass's gate output image: 128 rows x 128 channels f16
constexpr int DL_RING = 2 * DL_GCHUNK;           // ring slots start at 64 KiB ...
constexpr int DL_SLOT = 24 * 1024;               // ... 4 x 24 KiB; gate chunk 2 ([64, 96) KiB) overlays slots 0 / 1
constexpr int DL_LDS = DL_RING + 4 * DL_SLOT;    // 160 KiB
static_assert(DL_LDS == 160 * 1024, "diff_layer: LDS map");
static_assert(DL_RING + DL_GCHUNK <= DL_RING + 2 * DL_SLOT, "diff_layer: gate chunk 2 must stay off slots 2 / 3");

// 64-B image rows (one 32-deep K-step): a 16-B chunk q of row r sits at q ^ ((r >> 1) & 2); conflict-free for the
// ds_read_b128 lane groups of a 16-row MFMA fragment read (every 16 lanes of a group hit 16 distinct 16-B bank slots)
__device__ __forceinline__ int dl_sw64(int row, int q) { return q ^ ((row >> 1) & 2); }
// gate-output image rows of 256 B (128 channels): chunk q at q ^ (row & 15), conflict-free for the GEMM2 A fragments
__device__ __forceinline__ int dl_swg(int row, int q) { return q ^ (row & 15); }

__device__ __forceinline__ void dl_dma(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void dl_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void dl_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

struct DiffLayerArgs {
  ConvGemmArgs a;              // GEMM1: X = layer input hi [rows][384], W = packed dilated conv [768][1152], taps, tv
  const float* bias1;          // dilated conv bias (packed order)
  const f16* cp;               // conditioner projection of this layer [rows][768] (packed order)
  f16* g;                      // gate output [rows][384] (the layer's block of the skip-sum operand)
  const f16* W2;               // residual half of output_projection, packed [384][384] (N = K = Kpad = 384: the
                               // caller checks its PackedGemm)
  const float* bias2;
  f16* lo;                     // split residual low half [rows][384], updated in place
  f16* hi_out;                 // next layer input hi [rows][384] (NOT a.X)
  const float* sub;            // dproj_i: x = (hi + lo) - sub
  const float* add;            // dproj_{i+1}
  float acc_div;               // sqrt(2)
  int dbg;                     // diagnostics (tuning diff_dbg): 1 A from the zero page, 2 no GEMM1 MFMAs,
                               // 4 B from one fixed K-step of W_dil, 8 no epilogue HBM traffic (16 no cp loads,
                               // 32 no residual read-modify-write, 64 no gate-output stores, 128 no residual loads,
                               // 256 no residual stores)
};

template <typename F, int... K>
__device__ __forceinline__ void dl_unroll(F&& f, std::integer_sequence<int, K...>) {
  (f(std::integral_constant<int, K>{}), ...);
}

union DlH4 {
  uint2 u;
  f16 h[4];
};

__device__ __forceinline__ int dl_xcd_remap() {  // consecutive tiles (shared halo rows) on one XCD
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
}

__global__ __launch_bounds__(DL_NT, 1) void diff_layer_kernel(DiffLayerArgs p, const f16* zpage) {
  extern __shared__ __align__(16) unsigned char sm[];
  const ConvGemmArgs& a = p.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int M = a.B * a.T_out;
  const int m0 = dl_xcd_remap() * DL_BM;
  const int fr = lane & 15, fk = lane >> 4;
  const f16* zsrc = zpage + lane * 8;

  // ---- DMA slots. A: image row wave * 16 + (lane >> 2) (one wave-instruction per K-step); B: rows wave * 32 + v * 16
  // + (lane >> 2) of the pass's 256 packed columns; W2: rows wave * 48 + v * 16 + (lane >> 2)
  const int ar = wave * 16 + (lane >> 2);
  int a_t, a_tin;
  const f16* a_p;
  {
    const int m = m0 + ar;
    const int kv = dl_sw64(ar, lane & 3);
    if (m < M) {
      const int b = m / a.T_out, t = m - b * a.T_out;
      a_t = t * a.istride;
      a_tin = valid_in_rows(a, b);
      a_p = a.X + (int64_t)b * a.T_in * a.ldx + kv * 8;
    } else {
      a_t = -(1 << 29);
      a_tin = 0;
      a_p = a.X;
    }
  }
  const f16* b_p[2];
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int row = wave * 32 + v * 16 + (lane >> 2);
    b_p[v] = a.W + (int64_t)row * a.Kpad + dl_sw64(row, lane & 3) * 8;
  }
  auto issue = [&](int s_in) {
    // the step index through an opaque scalar move: the fully unrolled pass body would otherwise hoist all 36 steps'
    // DMA addresses into live registers
    int s;
    asm volatile("s_mov_b32 %0, %1" : "=s"(s) : "s"(s_in));
    unsigned char* st = sm + DL_RING + (s & 3) * DL_SLOT;
    const int pass = s / DL_KS1, ks = s - pass * DL_KS1;
    const int kg = ks * 32;
    const int tap = kg / DL_C;
    const int c0 = kg - tap * DL_C;
    const int sti = a_t + tap * a.tap_mul + a.tap_add;
    const bool ok = sti >= 0 && sti < a_tin && !(p.dbg & 1);
    dl_dma(ok ? (const void*)(a_p + (int64_t)sti * a.ldx + c0) : (const void*)zsrc, st + wave * 1024);
    const int64_t boff = (p.dbg & 4) ? 0 : (int64_t)pass * 256 * a.Kpad + kg;
#pragma unroll
    for (int v = 0; v < 2; ++v) dl_dma(b_p[v] + boff, st + 8192 + (wave * 2 + v) * 1024);
  };
  auto issue2 = [&](int k2) {
    unsigned char* st = sm + DL_RING + (2 + (k2 & 1)) * DL_SLOT;
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      const int row = wave * 48 + v * 16 + (lane >> 2);
      dl_dma(p.W2 + (int64_t)row * DL_C + k2 * 32 + dl_sw64(row, lane & 3) * 8, st + (wave * 3 + v) * 1024);
    }
  };

  floatx4 acc[4][4];
  DlH4 cpg[4][2], cpf[4][2];
  float4 bg[2], bfl[2];

  // one K-step s of GEMM1: wait for its slot, issue step s + 3 (and GEMM2's first step after the last). X: vector
  // memory operations issued after step s's DMAs that may stay in flight (the gate operands, see below)
  auto step = [&](int s, auto xc) {
    constexpr int X = decltype(xc)::value;
    // this wave's DMAs of step s have landed (those of s + 1, s + 2 may still be in flight) ... and everyone's
    if (s + 2 < DL_S1) dl_vmwait<6 + X>();
    else if (s + 1 < DL_S1) dl_vmwait<3 + X>();
    else dl_vmwait<X>();
    dl_barrier();  // also: every wave has finished step s - 1, so its slot (s + 3) & 3 is free
    if (s + 3 < DL_S1) issue(s + 3);
    if (s + 1 == DL_S1) issue2(0);  // slot 2 (step 106) is free: GEMM2's first W_res K-step under the last epilogue
  };
  auto mfmas = [&](int s) {
    const unsigned char* A = sm + DL_RING + (s & 3) * DL_SLOT;
    const unsigned char* Bm = A + 8192;
    half8 af[4], bf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + fr;
      af[i] = *reinterpret_cast<const half8*>(A + row * 64 + (dl_sw64(row, fk) << 4));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wn * 64 + j * 16 + fr;
      bf[j] = *reinterpret_cast<const half8*>(Bm + row * 64 + (dl_sw64(row, fk) << 4));
    }
    if (p.dbg & 2) return;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)  // C^T fragment: acc[i][j][r] = C[row fr of block i][col fk*4 + r of block j]
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  issue(0);
  issue(1);
  issue(2);
  for (int pass = 0; pass < 3; ++pass) {
    const int s0 = pass * DL_KS1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // The gate operands (4 bias + 16 conditioner-projection loads per lane) are spread over the pass, one load
    // right after the DMAs of K-steps KP0 .. KP0 + 19, so that the whole chip's 46 MB of cp per layer is not read
    // in one burst after the K-loop. A load issued at step t is younger than step t + 3's DMAs: the waits of steps
    // t + 1 .. t + 3 leave it in flight (their vmcnt counts it), step t + 4's wait retires it.
    const int nw = pass * 256 + wn * 64;  // the wave's packed columns: 32 gate + 32 filter channels
    const bool live_ops = !(p.dbg & 24);
    auto load_op = [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      if (!live_ops) return;
      if constexpr (q < 4) {
        const int col = nw + (q >> 1) * 32 + (q & 1) * 16 + fk * 4;
        const float4 v = *reinterpret_cast<const float4*>(p.bias1 + col);
        if constexpr (q >> 1) bfl[q & 1] = v; else bg[q & 1] = v;
      } else {
        constexpr int i = (q - 4) >> 2, j = ((q - 4) >> 1) & 1, flt = (q - 4) & 1;
        const int m = min(m0 + wm * 64 + i * 16 + fr, M - 1);  // clamped rows are loaded but never stored
        const uint2 v = *reinterpret_cast<const uint2*>(p.cp + (int64_t)m * (2 * DL_C) + nw + fk * 4 + flt * 32 + j * 16);
        if constexpr (flt) cpf[i][j].u = v; else cpg[i][j].u = v;
      }
    };
    if (!live_ops) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) cpg[i][j].u = cpf[i][j].u = make_uint2(0u, 0u);
      bg[0] = bg[1] = bfl[0] = bfl[1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    constexpr int KP0 = 4, NOP = 20;
    static_assert(KP0 >= 3 && KP0 + NOP + 4 <= DL_KS1, "diff_layer: gate operand schedule");
    auto kstep = [&](auto kc) {
      constexpr int ks = decltype(kc)::value;
      // operand loads issued at steps ks - 3 .. ks - 1 (each after its step's DMAs) are younger than step ks's DMAs
      constexpr int X = (ks - 3 >= KP0 && ks - 3 < KP0 + NOP) + (ks - 2 >= KP0 && ks - 2 < KP0 + NOP) +
                        (ks - 1 >= KP0 && ks - 1 < KP0 + NOP);
      step(s0 + ks, std::integral_constant<int, X>{});
      if constexpr (ks >= KP0 && ks < KP0 + NOP) {
        __builtin_amdgcn_sched_barrier(0);
        load_op(std::integral_constant<int, ks - KP0>{});
        __builtin_amdgcn_sched_barrier(0);
      }
      mfmas(s0 + ks);
    };
    dl_unroll(kstep, std::make_integer_sequence<int, DL_KS1>{});

    // gate epilogue of this pass into the LDS image (GEMM2's A; copied to HBM at the end)
    unsigned char* G = sm + pass * DL_GCHUNK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + fr;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float4 g = make_float4(acc[i][j][0] + bg[j].x, acc[i][j][1] + bg[j].y, acc[i][j][2] + bg[j].z,
                                     acc[i][j][3] + bg[j].w);
        const float4 f = make_float4(acc[i][j + 2][0] + bfl[j].x, acc[i][j + 2][1] + bfl[j].y,
                                     acc[i][j + 2][2] + bfl[j].z, acc[i][j + 2][3] + bfl[j].w);
        DlH4 pk;
        pk.h[0] = (f16)gate_act(g.x + (float)cpg[i][j].h[0], f.x + (float)cpf[i][j].h[0]);
        pk.h[1] = (f16)gate_act(g.y + (float)cpg[i][j].h[1], f.y + (float)cpf[i][j].h[1]);
        pk.h[2] = (f16)gate_act(g.z + (float)cpg[i][j].h[2], f.z + (float)cpf[i][j].h[2]);
        pk.h[3] = (f16)gate_act(g.w + (float)cpg[i][j].h[3], f.w + (float)cpf[i][j].h[3]);
        const int q = wn * 4 + j * 2 + (fk >> 1);  // 16-B chunk of the pass's 128 channels
        *reinterpret_cast<uint2*>(G + row * 256 + (dl_swg(row, q) << 4) + (fk & 1) * 8) = pk.u;
      }
    }
  }

  // ---- GEMM2: r = g . W_res, g from the LDS image, W_res K-steps through ring slots 2 / 3 (one step ahead)
  floatx4 acc2[4][6];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) acc2[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int k2 = 0; k2 < DL_KS2; ++k2) {
    dl_vmwait<0>();  // this wave's W_res DMAs of step k2 (nothing younger is outstanding)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // k2 == 0: this wave's gate-image writes are done
    dl_barrier();    // ... everyone's; slot 2 + ((k2 + 1) & 1) was last read in step k2 - 1 (or GEMM1's last step)
    if (k2 + 1 < DL_KS2) issue2(k2 + 1);
    const unsigned char* Bm = sm + DL_RING + (2 + (k2 & 1)) * DL_SLOT;
    const unsigned char* G = sm + (k2 >> 2) * DL_GCHUNK;
    half8 af[4], bf[6];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + fr;
      af[i] = *reinterpret_cast<const half8*>(G + row * 256 + (dl_swg(row, ((k2 & 3) << 2) + fk) << 4));
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int row = wn * 96 + j * 16 + fr;
      bf[j] = *reinterpret_cast<const half8*>(Bm + row * 64 + (dl_sw64(row, fk) << 4));
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc2[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }

  // ---- the gate output to HBM (the skip-sum GEMM's operand) from the LDS image: whole 16-B chunks, rows contiguous
  // across lanes; issued after GEMM2 so that no K-step's DMA wait also waits for these stores
#pragma unroll
  for (int k = 0; k < DL_BM * 48 / DL_NT; ++k) {
    const int idx = k * DL_NT + tid;
    const int row = idx / 48, c8 = idx - row * 48;
    const int m = m0 + row;
    if (m < M && !(p.dbg & 72))
      *reinterpret_cast<uint4*>(p.g + (int64_t)m * DL_C + c8 * 8) = *reinterpret_cast<const uint4*>(
          sm + (c8 >> 4) * DL_GCHUNK + row * 256 + (dl_swg(row, c8 & 15) << 4));
  }

  // ---- residual update from registers (conv_gemm4's split-fp16 read-modify-write, same operation order)
  const int nb = wn * 96 + fk * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + fr;
    if (m >= M || (p.dbg & 40)) continue;
    DlH4 hi[6], lo[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {  // the row's residual operands first: the stores below may alias later loads
      if (p.dbg & 128) {
        hi[j].u = lo[j].u = make_uint2(0u, 0u);
        continue;
      }
      hi[j].u = *reinterpret_cast<const uint2*>(a.X + (int64_t)m * DL_C + nb + j * 16);
      lo[j].u = *reinterpret_cast<const uint2*>(p.lo + (int64_t)m * DL_C + nb + j * 16);
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int n = nb + j * 16;
      const float4 bi = *reinterpret_cast<const float4*>(p.bias2 + n);
      const float4 ad = *reinterpret_cast<const float4*>(p.add + n);
      const float4 sb = *reinterpret_cast<const float4*>(p.sub + n);
      float4 v = make_float4(acc2[i][j][0] + bi.x, acc2[i][j][1] + bi.y, acc2[i][j][2] + bi.z, acc2[i][j][3] + bi.w);
      float4 ac;
      ac.x = ((float)hi[j].h[0] + (float)lo[j].h[0]) - sb.x;
      ac.y = ((float)hi[j].h[1] + (float)lo[j].h[1]) - sb.y;
      ac.z = ((float)hi[j].h[2] + (float)lo[j].h[2]) - sb.z;
      ac.w = ((float)hi[j].h[3] + (float)lo[j].h[3]) - sb.w;
      v.x = (ac.x + v.x) / p.acc_div;
      v.y = (ac.y + v.y) / p.acc_div;
      v.z = (ac.z + v.z) / p.acc_div;
      v.w = (ac.w + v.w) / p.acc_div;
      const float4 w = make_float4(v.x + ad.x, v.y + ad.y, v.z + ad.z, v.w + ad.w);
      DlH4 pk, lw;
      pk.h[0] = f16_sat(w.x); pk.h[1] = f16_sat(w.y); pk.h[2] = f16_sat(w.z); pk.h[3] = f16_sat(w.w);
      lw.h[0] = (f16)(w.x - (float)pk.h[0]); lw.h[1] = (f16)(w.y - (float)pk.h[1]);
      lw.h[2] = (f16)(w.z - (float)pk.h[2]); lw.h[3] = (f16)(w.w - (float)pk.h[3]);
      if (p.dbg & 256) {
        if (pk.u.x == 0x12345u && lw.u.y == 0x54321u) p.hi_out[0] = (f16)1.f;  // keep the arithmetic
        continue;
      }
      *reinterpret_cast<uint2*>(p.hi_out + (int64_t)m * DL_C + n) = pk.u;
      *reinterpret_cast<uint2*>(p.lo + (int64_t)m * DL_C + n) = lw.u;
    }
  }
}

// ================================================================================================ fused head
// DiffSVC head (modules/diffsvc.py:311-321) after the skip sum, one launch per 128-row tile:
//   GEMM A  u = relu(s . W_sp + b_sp): s = the split-fp16 skip sum [hi | lo | hi] (K = 1152), N = 384, through a
//           4-slot ring of 32-deep K-steps (A 128 x 64 B + B 384 x 64 B = 32 KiB per slot, three steps ahead: one
//           tile per CU, so the step time is the DMA latency over the steps in flight);
//   GEMM B  eps = [u_hi | u_lo | u_hi] . W_out + b_out, N = 100 (packed rows to 128): u_hi as an f16 image in LDS
//           (over GEMM A's ring), u_lo packed in registers and written over the image for the last third, so the
//           138 MB split-fp16 intermediate of a full-batch call never reaches HBM; W_out K-steps through a 4-slot ring
//           whose first three steps load at kernel start.
//           K runs hi . W_hi, hi . W_lo, lo . W_hi (the unfused GEMM: hi, lo, hi), so the f32 sum differs from the
//           unfused path's in rounding order only (tests/test_gpu_stages.py::test_fused_head).
// Same epilogue expressions as conv_gemm3's LDS epilogue for these two calls (relu(acc + bias), hi = f16(v),
// lo = f16(v - hi); eps = acc + bias).
constexpr int DH_S1 = 3 * DL_C / 32;          // 36 K-steps of each GEMM
constexpr int DH_SLOT_A = 32 * 1024;          // GEMM A ring slot (4 slots)
constexpr int DH_IMG = 0;                     // u image [3 chunks][128 rows][256 B] = 96 KiB, over GEMM A's ring
constexpr int DH_RING_B = 128 * 1024;         // GEMM B ring: 4 x 8 KiB
constexpr int DH_LDS = DH_RING_B + 4 * 8192;  // 160 KiB

struct DiffHeadArgs {
  const f16* s16;    // [rows][1152] split-fp16 skip sum
  const f16* Wsp;    // skip_projection packed [>= 384][1152]
  const float* bsp;
  const f16* Wout;   // output_projection packed [>= 128][1152] (rows >= 100 zero)
  const float* bout;
  float* eps;        // [rows][ld_eps]
  int ld_eps, n_out, M;
  int plms;          // apply pl in the epilogue (the PLMS update that follows this eps, elementwise.hip plms4_kernel)
  PlmsArgs pl;
  int mel;           // then the next denoise's input projection from the updated x (GEMM C)
  MelNext mn;
};

// plms4_kernel's update of 4 channels (flat index i, row r = m, column c = n) with the freshly computed eps in
// registers: the same expressions in the same order, so x / x16 are those plms_update would write
__device__ __forceinline__ float4 head_plms(const PlmsArgs& p, const float* self, float4 e0v, int64_t i, int64_t r,
                                            int c) {
  auto ld = [&](const float* q) { return q == self ? e0v : *reinterpret_cast<const float4*>(q + i); };
  const float4 v0 = ld(p.e[0]);
  float e[4] = {p.c[0] * v0.x, p.c[0] * v0.y, p.c[0] * v0.z, p.c[0] * v0.w};
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    if (p.ne > k) {
      const float4 v = ld(p.e[k]);
      e[0] = e[0] + p.c[k] * v.x;
      e[1] = e[1] + p.c[k] * v.y;
      e[2] = e[2] + p.c[k] * v.z;
      e[3] = e[3] + p.c[k] * v.w;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) e[k] = e[k] / p.div;
  if (p.e_avg_out) *reinterpret_cast<float4*>(p.e_avg_out + i) = make_float4(e[0], e[1], e[2], e[3]);
  const float4 x = *reinterpret_cast<const float4*>(p.xin + i);
  const float4 xn = make_float4(x.x + p.d * (p.A * x.x - p.Bc * e[0]), x.y + p.d * (p.A * x.y - p.Bc * e[1]),
                                x.z + p.d * (p.A * x.z - p.Bc * e[2]), x.w + p.d * (p.A * x.w - p.Bc * e[3]));
  *reinterpret_cast<float4*>(p.xout + i) = xn;
  if (p.x16) {
    union { uint2 u; f16 h[4]; } pk;
    pk.h[0] = f16_sat(xn.x); pk.h[1] = f16_sat(xn.y); pk.h[2] = f16_sat(xn.z); pk.h[3] = f16_sat(xn.w);
    *reinterpret_cast<uint2*>(p.x16 + r * p.ld16 + c) = pk.u;
  }
  return xn;
}

__global__ __launch_bounds__(DL_NT, 1) void diff_head_kernel(DiffHeadArgs p, const f16* zpage) {
  extern __shared__ __align__(16) unsigned char sm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int M = p.M;
  const int m0 = dl_xcd_remap() * DL_BM;
  const int fr = lane & 15, fk = lane >> 4;
  const f16* zsrc = zpage + lane * 8;
  constexpr int LDS_ = 3 * DL_C;  // 1152 halves per s16 row / packed weight row

  // GEMM A DMA slots: A row wave * 16 + (lane >> 2); B rows wave * 48 + v * 16 + (lane >> 2), v < 3
  const int ar = wave * 16 + (lane >> 2);
  const f16* a_p = (m0 + ar < M) ? p.s16 + (int64_t)(m0 + ar) * LDS_ + dl_sw64(ar, lane & 3) * 8 : nullptr;
  const f16* b_p[3];
#pragma unroll
  for (int v = 0; v < 3; ++v) {
    const int row = wave * 48 + v * 16 + (lane >> 2);
    b_p[v] = p.Wsp + (int64_t)row * LDS_ + dl_sw64(row, lane & 3) * 8;
  }
  const int orow = wave * 16 + (lane >> 2);  // GEMM B weight rows (128)
  const f16* o_p = p.Wout + (int64_t)orow * LDS_ + dl_sw64(orow, lane & 3) * 8;
  auto issueA = [&](int s_in) {
    int s;
    asm volatile("s_mov_b32 %0, %1" : "=s"(s) : "s"(s_in));
    unsigned char* st = sm + (s & 3) * DH_SLOT_A;
    dl_dma(a_p ? (const void*)(a_p + s * 32) : (const void*)zsrc, st + wave * 1024);
#pragma unroll
    for (int v = 0; v < 3; ++v) dl_dma(b_p[v] + s * 32, st + 8192 + (wave * 3 + v) * 1024);
  };
  auto issueB = [&](int s_in) {  // GEMM B step s reads weight K-step 0-11, 24-35, 12-23 (see GEMM B)
    int s;
    asm volatile("s_mov_b32 %0, %1" : "=s"(s) : "s"(s_in));
    const int ws = s < DL_KS2 ? s : (s < 2 * DL_KS2 ? s + DL_KS2 : s - DL_KS2);
    dl_dma(o_p + ws * 32, sm + DH_RING_B + (s & 3) * 8192 + wave * 1024);
  };

  // ---- GEMM A
  floatx4 acc[4][6];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  issueB(0);  // GEMM B's first weight steps: their own ring, older than every GEMM A DMA (in-order vmcnt)
  issueB(1);
  issueB(2);
  issueA(0);
  issueA(1);
  issueA(2);
  for (int s = 0; s < DH_S1; ++s) {
    // step s landed (s + 1, s + 2 may be in flight: 4 DMAs each)
    if (s + 2 < DH_S1) dl_vmwait<8>(); else if (s + 1 < DH_S1) dl_vmwait<4>(); else dl_vmwait<0>();
    dl_barrier();  // every wave finished step s - 1: its slot (s + 3) & 3 is free
    if (s + 3 < DH_S1) issueA(s + 3);
    const unsigned char* A = sm + (s & 3) * DH_SLOT_A;
    const unsigned char* Bm = A + 8192;
    half8 af[4], bf[6];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + fr;
      af[i] = *reinterpret_cast<const half8*>(A + row * 64 + (dl_sw64(row, fk) << 4));
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int row = wn * 96 + j * 16 + fr;
      bf[j] = *reinterpret_cast<const half8*>(Bm + row * 64 + (dl_sw64(row, fk) << 4));
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }
  // u = relu(acc + b_sp); hi = f16(u) goes to the LDS image, lo = f16(u - hi) stays in registers (packed, half the
  // registers of u), so GEMM A's f32 accumulators die here
  const int nb = wn * 96 + fk * 4;
  uint2 ulo[4][6];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  dl_barrier();  // every wave finished GEMM A's last step: the ring under the image is free
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int n = nb + j * 16;
    const float4 bi = *reinterpret_cast<const float4*>(p.bsp + n);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + fr;
      const float u[4] = {fmaxf(acc[i][j][0] + bi.x, 0.f), fmaxf(acc[i][j][1] + bi.y, 0.f),
                          fmaxf(acc[i][j][2] + bi.z, 0.f), fmaxf(acc[i][j][3] + bi.w, 0.f)};
      DlH4 hi, lo;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hi.h[r] = f16_sat(u[r]);
        lo.h[r] = (f16)(u[r] - (float)hi.h[r]);
      }
      ulo[i][j] = lo.u;
      *reinterpret_cast<uint2*>(sm + DH_IMG + (n >> 7) * DL_GCHUNK + row * 256 + (dl_swg(row, (n & 127) >> 3) << 4) +
                                ((n >> 2) & 1) * 8) = hi.u;
    }
  }

  // ---- GEMM B: K steps in the order u_hi . W_hi (weight K-steps 0-11), u_hi . W_lo (24-35), u_lo . W_hi (12-23)
  floatx4 acc2[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc2[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int s = 0; s < DH_S1; ++s) {
    if (s == 2 * DL_KS2) {  // the lo image replaces the hi image once every wave has finished reading it
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      dl_barrier();
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int n = nb + j * 16;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wm * 64 + i * 16 + fr;
          *reinterpret_cast<uint2*>(sm + DH_IMG + (n >> 7) * DL_GCHUNK + row * 256 +
                                    (dl_swg(row, (n & 127) >> 3) << 4) + ((n >> 2) & 1) * 8) = ulo[i][j];
        }
      }
    }
    if (s + 2 < DH_S1) dl_vmwait<2>(); else if (s + 1 < DH_S1) dl_vmwait<1>(); else dl_vmwait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's image writes
    dl_barrier();
    if (s + 3 < DH_S1) issueB(s + 3);
    const int k2 = s % DL_KS2;  // K-step within the 384-channel image
    const unsigned char* Bm = sm + DH_RING_B + (s & 3) * 8192;
    half8 af[4], bf[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + fr;
      af[i] = *reinterpret_cast<const half8*>(sm + DH_IMG + (k2 >> 2) * DL_GCHUNK + row * 256 +
                                              (dl_swg(row, ((k2 & 3) << 2) + fk) << 4));
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wn * 32 + j * 16 + fr;
      bf[j] = *reinterpret_cast<const half8*>(Bm + row * 64 + (dl_sw64(row, fk) << 4));
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc2[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }
  // ---- eps = acc + b_out, columns < n_out (+ the PLMS update; + the next input projection's A image of f16(x'))
  constexpr int DH_XIMG = 0, DH_WMEL = 32 * 1024;  // GEMM C: x' image [128 rows][256 B], W_mel [384 rows][256 B]
  if (p.mel) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    dl_barrier();  // every wave finished GEMM B: the u image and ring B are free
#pragma unroll
    for (int v = 0; v < 12; ++v) {  // W_mel, 1 KiB = 4 rows per DMA, granules swizzled at the source
      const int row = (wave * 12 + v) * 4 + (lane >> 4);
      dl_dma(p.mn.W + (int64_t)row * 128 + dl_swg(row, lane & 15) * 8, sm + DH_WMEL + (wave * 12 + v) * 1024);
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = wn * 32 + j * 16 + fk * 4;
    const bool col = n < p.n_out;
    const float4 bi = col ? *reinterpret_cast<const float4*>(p.bout + n) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + fr;
      const int m = m0 + row;
      float4 xn = make_float4(0.f, 0.f, 0.f, 0.f);
      if (col && m < M) {
        const float4 ev =
            make_float4(acc2[i][j][0] + bi.x, acc2[i][j][1] + bi.y, acc2[i][j][2] + bi.z, acc2[i][j][3] + bi.w);
        const int64_t idx = (int64_t)m * p.ld_eps + n;
        *reinterpret_cast<float4*>(p.eps + idx) = ev;
        if (p.plms) xn = head_plms(p.pl, p.eps, ev, idx, m, n);
      }
      if (p.mel) {
        DlH4 pk;
        pk.h[0] = f16_sat(xn.x); pk.h[1] = f16_sat(xn.y); pk.h[2] = f16_sat(xn.z); pk.h[3] = f16_sat(xn.w);
        *reinterpret_cast<uint2*>(sm + DH_XIMG + row * 256 + (dl_swg(row, n >> 3) << 4) + ((n >> 2) & 1) * 8) = pk.u;
      }
    }
  }
  if (!p.mel) return;
  // ---- GEMM C: h = relu(x' . W_mel + b_mel) + dproj_0(t_next) as split-fp16, 4 K-steps of 32 (Kpad 128)
  dl_vmwait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  dl_barrier();
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    half8 af[4], bf[6];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + fr;
      af[i] = *reinterpret_cast<const half8*>(sm + DH_XIMG + row * 256 + (dl_swg(row, ks * 4 + fk) << 4));
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int row = wn * 96 + j * 16 + fr;
      bf[j] = *reinterpret_cast<const half8*>(sm + DH_WMEL + row * 256 + (dl_swg(row, ks * 4 + fk) << 4));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int n = nb + j * 16;
    const float4 bi = *reinterpret_cast<const float4*>(p.mn.bias + n);
    const float4 ad = *reinterpret_cast<const float4*>(p.mn.dp + n);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + i * 16 + fr;
      if (m >= M) continue;
      // conv_gemm3's epilogue expressions: v = relu(acc + b); w = v + add16; hi = f16_sat(w); lo = f16(w - hi)
      const float w[4] = {fmaxf(acc[i][j][0] + bi.x, 0.f) + ad.x, fmaxf(acc[i][j][1] + bi.y, 0.f) + ad.y,
                          fmaxf(acc[i][j][2] + bi.z, 0.f) + ad.z, fmaxf(acc[i][j][3] + bi.w, 0.f) + ad.w};
      DlH4 hi, lo;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hi.h[r] = f16_sat(w[r]);
        lo.h[r] = (f16)(w[r] - (float)hi.h[r]);
      }
      *reinterpret_cast<uint2*>(p.mn.y16 + (int64_t)m * p.mn.N + n) = hi.u;
      *reinterpret_cast<uint2*>(p.mn.lo16 + (int64_t)m * p.mn.N + n) = lo.u;
    }
  }
}

int diff_head(const f16* s16, const f16* Wsp, const float* bsp, int Nsp, int Ksp, const f16* Wout, const float* bout,
              int Nout, int Kout, int Npad_out, float* eps, int ld_eps, int M, const f16* zpage, hipStream_t s,
              const PlmsArgs* plms, const MelNext* mel) {
  SVC_REQUIRE(Nsp == DL_C && Ksp == 3 * DL_C && Kout == 3 * DL_C && Nout >= 1 && Nout <= 128 && Nout % 4 == 0 &&
                  Npad_out >= 128 && ld_eps % 4 == 0,
              "diff_head: shape (Nsp %d Ksp %d Nout %d Kout %d)", Nsp, Ksp, Nout, Kout);
  const void* ptrs[] = {s16, Wsp, bsp, Wout, bout, eps};
  for (const void* q : ptrs) SVC_REQUIRE(q && ((uintptr_t)q & 15) == 0, "diff_head: operand not 16-B aligned");
  const int64_t grid = cdiv64(M, DL_BM);
  SVC_REQUIRE(grid > 0 && grid < (1ll << 31), "diff_head: bad grid");
  DiffHeadArgs p{s16, Wsp, bsp, Wout, bout, eps, ld_eps, Nout, M, 0, PlmsArgs{}, 0, MelNext{}};
  if (plms) {  // the update's flat index is the eps index: rows of ld_eps == Nout channels, 16-B aligned operands
    SVC_REQUIRE(ld_eps == Nout && plms->ne >= 1 && plms->ne <= 4 && (!plms->x16 || plms->ld16 % 4 == 0),
                "diff_head: PLMS update shape (ld_eps %d Nout %d ne %d)", ld_eps, Nout, plms->ne);
    auto al = [](const void* q, uintptr_t a) { return ((uintptr_t)q & (a - 1)) == 0; };  // null passes
    bool ok = plms->xin && plms->xout && al(plms->xin, 16) && al(plms->xout, 16) && al(plms->x16, 8) &&
              al(plms->e_avg_out, 16);
    for (int k = 0; k < plms->ne; ++k) ok = ok && plms->e[k] && al(plms->e[k], 16);
    SVC_REQUIRE(ok, "diff_head: PLMS operand missing or misaligned");
    p.plms = 1;
    p.pl = *plms;
  }
  if (mel) {
    SVC_REQUIRE(plms && mel->N == DL_C && mel->Kpad == 128 && mel->K <= 128 && Nout <= mel->K,
                "diff_head: next input projection shape (N %d K %d Kpad %d)", mel->N, mel->K, mel->Kpad);
    const void* mp[] = {mel->W, mel->bias, mel->dp, mel->y16, mel->lo16};
    for (const void* q : mp) SVC_REQUIRE(q && ((uintptr_t)q & 15) == 0, "diff_head: input-projection operand");
    p.mel = 1;
    p.mn = *mel;
  }
  static bool attr = false;
  if (!attr) {
    SVC_HIP_CHECK(hipFuncSetAttribute((const void*)diff_head_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      DH_LDS));
    attr = true;
  }
  const double flops = 2.0 * M * (double)DL_C * 3 * DL_C + 2.0 * M * (double)Nout * 3 * DL_C;
  const int tok = prof_begin("diff_head<128>", flops, 0.0, s);
  void* args[] = {&p, const_cast<const f16**>(&zpage)};
  SVC_HIP_CHECK(hipLaunchKernel((const void*)diff_head_kernel, dim3((unsigned)grid), dim3(DL_NT), args, DH_LDS, s));
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// The fused layer's shape: 384 channels, a 3-tap dilated conv, 1:1 rows (the DiffSVC residual layer)
bool diff_layer_form(const ConvGemmArgs& a) {
  return a.Cp == DL_C && a.K == 3 * DL_C && a.Kpad == 3 * DL_C && a.N == 2 * DL_C && a.ldx == DL_C &&
         a.T_in == a.T_out && a.istride == 1 && a.Cvalid == DL_C;
}

int diff_layer(const ConvGemmArgs& a, const float* bias1, const f16* cp, f16* g, const f16* W2, const float* bias2,
               f16* lo, f16* hi_out, const float* sub, const float* add, float acc_div, const f16* zpage,
               hipStream_t s, int dbg) {
  SVC_REQUIRE(diff_layer_form(a), "diff_layer: shape (Cp %d K %d Kpad %d N %d ldx %d)", a.Cp, a.K, a.Kpad, a.N, a.ldx);
  SVC_REQUIRE(hi_out != a.X, "diff_layer: the layer input cannot be updated in place");
  const void* ptrs[] = {a.X, a.W, cp, g, W2, lo, hi_out, bias1, bias2, sub, add};
  for (const void* q : ptrs) SVC_REQUIRE(q && ((uintptr_t)q & 15) == 0, "diff_layer: operand not 16-B aligned");
  const int64_t M = (int64_t)a.B * a.T_out;
  const int64_t grid = cdiv64(M, DL_BM);
  SVC_REQUIRE(grid > 0 && grid < (1ll << 31), "diff_layer: bad grid");
  DiffLayerArgs p{};
  p.a = a;
  p.bias1 = bias1;
  p.cp = cp;
  p.g = g;
  p.W2 = W2;
  p.bias2 = bias2;
  p.lo = lo;
  p.hi_out = hi_out;
  p.sub = sub;
  p.add = add;
  p.acc_div = acc_div;
  p.dbg = dbg;
  static bool attr = false;
  if (!attr) {
    SVC_HIP_CHECK(hipFuncSetAttribute((const void*)diff_layer_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      DL_LDS));
    attr = true;
  }
  const double flops = 2.0 * M * (2.0 * DL_C * 3 * DL_C + (double)DL_C * DL_C);
  const int tok = prof_begin("diff_layer<128>", flops, 0.0, s);
  void* args[] = {&p, const_cast<const f16**>(&zpage)};
  SVC_HIP_CHECK(hipLaunchKernel((const void*)diff_layer_kernel, dim3((unsigned)grid), dim3(DL_NT), args, DL_LDS, s));
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
