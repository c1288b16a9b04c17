// Second-generation implicit-GEMM Conv1d / Linear for gfx950 (v_mfma_f32_32x32x16_f16).
//
// Differences from gemm.hip (kept for N <= 64):
//   * 32x32x16 fragments: half the LDS fragment bytes per FLOP of 16x16x32.
//   * global -> LDS by LDS-DMA (global_load_lds_dwordx4): no staging registers, no ds_write. The LDS
//     image stays lane-linear (1 KiB per wave instruction = 8 rows x 128 B); the XOR swizzle that makes
//     the fragment reads conflict-free is applied to the per-lane SOURCE address instead
//     (chunk p of row r holds logical k-chunk p ^ ((r>>1)&7)).
//   * conv zero padding / K tail / M tail: those lanes load from a zero page instead of masking.
//     A-operand buffers must therefore have zero (or finite, zero-weighted) pad channels.
//   * two LDS buffers: the DMA of K-tile k+1 is in flight while tile k is multiplied; one
//     __syncthreads per K-tile (it waits vmcnt(0), i.e. the DMA, and orders the buffer reuse).
// Paired epilogues (DiffSVC) use 64-column groups: 32 first-half channels then their 32 partners, so a
// lane holds both halves of a pair in fragments j and j+1.
#include "common.h"
#include "epilogue.h"

namespace svc {

template <int BM, int BN, int WM, int WN, int ST>
struct G2 {
  static constexpr int NT = 64 * WM * WN;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int FM = TM / 32, FN = TN / 32;
  static constexpr int A_INSTR = BM / 8;  // 1 KiB wave instructions per A tile
  static constexpr int B_INSTR = BN / 8;
  static constexpr int NW = WM * WN;
  static constexpr int RING_BYTES = ST * (BM + BN) * 128;
  // epilogue staging of the f32 C tile: one pass if it fits 160 KiB, else two column halves
  static constexpr int EP = (BM * (BN + 4) * 4 <= 163840) ? 1 : 2;
  static constexpr int C_BYTES = BM * (BN / EP + 4) * 4;
  static constexpr int LDS_BYTES = RING_BYTES > C_BYTES ? RING_BYTES : C_BYTES;
  static_assert(LDS_BYTES <= 163840, "LDS budget");
  // LDS-DMA instructions each wave issues per K-tile (the vmcnt unit of the ring)
  static constexpr int I_PER_TILE = (A_INSTR + NW - 1) / NW + (B_INSTR + NW - 1) / NW;
  static_assert(A_INSTR % NW == 0 && B_INSTR % NW == 0, "uniform DMA count per wave");
};

// counted wait for this wave's LDS-DMA: all but the N youngest vector-memory ops complete
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  if constexpr (N >= 63) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int sw_chunk(int row, int kv) { return kv ^ ((row >> 1) & 7); }

template <int BM, int BN, int WM, int WN, int ST, bool PAIR>
__global__ __launch_bounds__(64 * WM * WN, 1) void conv_gemm2_kernel(ConvGemmArgs a, EpiArgs e, const f16* zpage,
                                                                     float inv_cp) {
  using CF = G2<BM, BN, WM, WN, ST>;
  extern __shared__ __align__(16) unsigned char smem2[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;

  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, rr8 = nwg & 7;
  const int wgid = (xcd < rr8 ? xcd * (q + 1) : rr8 * (q + 1) + (xcd - rr8) * q) + (orig >> 3);
  const int tile_n = wgid % a.ntiles_n, tile_m = wgid / a.ntiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int M = a.B * a.T_out;

  // ---- per-lane DMA source rows: this wave issues A instructions wave, wave+NW, ... (8 rows each)
  constexpr int AI = (CF::A_INSTR + CF::NW - 1) / CF::NW;
  constexpr int BI = (CF::B_INSTR + CF::NW - 1) / CF::NW;
  int a_base[AI], a_tt[AI], a_kv[AI];
#pragma unroll
  for (int u = 0; u < AI; ++u) {
    const int ins = wave + u * CF::NW;
    const int r = ins * 8 + (lane >> 3);
    const int m = m0 + r;
    a_kv[u] = sw_chunk(r, lane & 7);
    if (ins < CF::A_INSTR && m < M) {
      const int b = m / a.T_out, t = m - b * a.T_out;
      a_base[u] = b * a.T_in;
      a_tt[u] = t * a.istride;
    } else {
      a_base[u] = 0;
      a_tt[u] = -(1 << 29);
    }
  }
  int b_kv[BI];
#pragma unroll
  for (int u = 0; u < BI; ++u) b_kv[u] = sw_chunk((wave + u * CF::NW) * 8 + (lane >> 3), lane & 7);

  auto lds_a = [&](int buf) { return smem2 + buf * (BM + BN) * 128; };
  auto lds_b = [&](int buf) { return smem2 + buf * (BM + BN) * 128 + BM * 128; };

  auto issue = [&](int kt, int buf) {
#pragma unroll
    for (int u = 0; u < AI; ++u) {
      const int ins = wave + u * CF::NW;
      if (ins < CF::A_INSTR) {
        const int kg = kt * 64 + a_kv[u] * 8;
        int tap = (int)((float)kg * inv_cp);
        if ((tap + 1) * a.Cp <= kg) ++tap;
        if (tap * a.Cp > kg) --tap;
        const int c = kg - tap * a.Cp;
        const int st = a_tt[u] + tap * a.tap_mul + a.tap_add;
        const f16* src = zpage + lane * 8;
        if (kg < a.K && st >= 0 && st < a.T_in) src = a.X + (int64_t)(a_base[u] + st) * a.ldx + c;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(lds_a(buf) + ins * 1024), 16, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < BI; ++u) {
      const int ins = wave + u * CF::NW;
      if (ins < CF::B_INSTR) {
        const int r = ins * 8 + (lane >> 3);
        const f16* src = a.W + (int64_t)(n0 + r) * a.Kpad + kt * 64 + b_kv[u] * 8;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(lds_b(buf) + ins * 1024), 16, 0, 0);
      }
    }
  };

  floatx16 acc[CF::FM][CF::FN];
#pragma unroll
  for (int i = 0; i < CF::FM; ++i)
#pragma unroll
    for (int j = 0; j < CF::FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // ST-deep LDS ring: tiles kt+1 .. kt+ST-1 are in flight while tile kt is multiplied. Waits are
  // counted per wave (vmcnt), then a raw s_barrier publishes every wave's DMA for tile kt; the buffer
  // refilled at iteration kt was last read at iteration kt-1, i.e. before that barrier.
  const int nk = a.Kpad / 64;
#pragma unroll
  for (int p = 0; p < ST - 1; ++p)
    if (p < nk) issue(p, p);
  const int lr = lane & 31, lh = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % ST;
    if (kt + ST - 2 < nk) wait_vmcnt<(ST - 2) * CF::I_PER_TILE>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + ST - 1 < nk) issue(kt + ST - 1, (kt + ST - 1) % ST);
    const unsigned char* Ab = lds_a(cur);
    const unsigned char* Bb = lds_b(cur);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      half8 af[CF::FM], bf[CF::FN];
      const int kv = 2 * s + lh;
#pragma unroll
      for (int i = 0; i < CF::FM; ++i) {
        const int row = wm * CF::TM + i * 32 + lr;
        af[i] = *reinterpret_cast<const half8*>(Ab + row * 128 + (sw_chunk(row, kv) << 4));
      }
#pragma unroll
      for (int j = 0; j < CF::FN; ++j) {
        const int row = wn * CF::TN + j * 32 + lr;
        bf[j] = *reinterpret_cast<const half8*>(Bb + row * 128 + (sw_chunk(row, kv) << 4));
      }
#pragma unroll
      for (int i = 0; i < CF::FM; ++i)
#pragma unroll
        for (int j = 0; j < CF::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }

  // ---------------------------------------------------------------- epilogue
  // Stage the f32 tile through LDS (the ring is free once every wave left the K loop), then apply the
  // epilogue on 4-column chunks with 16-byte vector loads/stores (coalesced rows).
  // acc[i][j][r] = C[wm*TM + i*32 + (r&3) + 8(r>>2) + 4*lh][wn*TN + j*32 + lr]
  __syncthreads();
  // the staged C tile may exceed LDS: process it in EP column passes (each wave belongs to one pass)
  constexpr int EP = CF::EP;
  constexpr int BNP = BN / EP;
  constexpr int LDC = BNP + 4;
  static_assert(WN % EP == 0 && BM * LDC * 4 <= CF::LDS_BYTES, "C tile pass must fit the LDS ring");
  float* Cs = reinterpret_cast<float*>(smem2);
#pragma unroll
  for (int pass = 0; pass < EP; ++pass) {
  if (wn / (WN / EP) == pass) {
#pragma unroll
    for (int i = 0; i < CF::FM; ++i)
#pragma unroll
      for (int j = 0; j < CF::FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          Cs[(wm * CF::TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * LDC + wn * CF::TN - pass * BNP + j * 32 + lr] =
              acc[i][j][r];
  }
  __syncthreads();
  epilogue_pass<BM, BNP, LDC, CF::NT, PAIR>(Cs, m0, n0 + pass * BNP, M, a, e, tid);
  __syncthreads();
  }  // pass
}

template <int BM, int BN, int WM, int WN, int ST, bool PAIR>
static int launch2(const ConvGemmArgs& a0, const EpiArgs& e, const f16* zpage, hipStream_t s, const char* tag) {
  using CF = G2<BM, BN, WM, WN, ST>;
  ConvGemmArgs a = a0;
  const int M = a.B * a.T_out;
  a.ntiles_n = cdiv(a.N, BN);
  const int64_t grid = (int64_t)cdiv(M, BM) * a.ntiles_n;
  SVC_REQUIRE(grid > 0 && grid < (1ll << 31), "conv_gemm2: bad grid");
  SVC_REQUIRE((int64_t)a.ntiles_n * BN <= round_up(a.N, 256), "conv_gemm2: weights not padded for BN=%d", BN);
  static bool attr = false;
  if (!attr) {
    SVC_HIP_CHECK(hipFuncSetAttribute((const void*)conv_gemm2_kernel<BM, BN, WM, WN, ST, PAIR>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, CF::LDS_BYTES));
    attr = true;
  }
  const double kreal = (double)(a.K / a.Cp) * a.Cvalid;
  const int tok = prof_begin(tag, 2.0 * M * (double)a.N * kreal, 0.0, s);
  hipLaunchKernelGGL((conv_gemm2_kernel<BM, BN, WM, WN, ST, PAIR>), dim3((unsigned)grid), dim3(CF::NT), CF::LDS_BYTES, s,
                     a, e, zpage, 1.0f / (float)a.Cp);
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

int conv_gemm2(const ConvGemmArgs& a, const EpiArgs& e, const f16* zpage, int variant, hipStream_t s) {
  SVC_REQUIRE(a.Cp % 8 == 0 && a.ldx % 8 == 0 && a.Kpad % 64 == 0 && a.N % 4 == 0, "conv_gemm2: layout");
  SVC_REQUIRE(e.ld32 % 4 == 0 && e.ld16 % 4 == 0 && e.ld_add_row % 4 == 0 && e.ld_acc % 4 == 0 && e.ld_add_t % 4 == 0 &&
                  e.ld_cp % 4 == 0 && e.ldy16 % 4 == 0 && e.ld_emb % 4 == 0,
              "conv_gemm2: epilogue leading dimensions must be multiples of 4 (vector epilogue)");
  SVC_REQUIRE(((uintptr_t)a.X & 15) == 0 && ((uintptr_t)a.W & 15) == 0, "conv_gemm2: 16-B alignment");
  const bool pair = e.kind == EPI_GATE;
  if (pair) {
    SVC_REQUIRE(a.N % 64 == 0, "conv_gemm2: paired epilogue needs N %% 64 == 0");
    if (variant == 1) return launch2<256, 128, 4, 2, 3, true>(a, e, zpage, s, "conv_gemm2<256,128,pair>");
    if (variant == 2) return launch2<256, 256, 2, 4, 2, true>(a, e, zpage, s, "conv_gemm2<256,256,pair>");
    if (variant == 3) return launch2<192, 256, 2, 4, 2, true>(a, e, zpage, s, "conv_gemm2<192,256,pair>");
    if (variant == 4) return launch2<128, 128, 2, 2, 2, true>(a, e, zpage, s, "conv_gemm2<128,128,st2,pair>");
    return launch2<128, 128, 2, 2, 4, true>(a, e, zpage, s, "conv_gemm2<128,128,pair>");
  }
  if (variant == 1) return launch2<256, 128, 4, 2, 3, false>(a, e, zpage, s, "conv_gemm2<256,128>");
  if (variant == 2) return launch2<256, 256, 2, 4, 2, false>(a, e, zpage, s, "conv_gemm2<256,256>");
  if (variant == 3) return launch2<192, 256, 2, 4, 2, false>(a, e, zpage, s, "conv_gemm2<192,256>");
  // 2-deep ring: 68 KiB of LDS, two workgroups per CU overlap one's epilogue with the other's K loop
  if (variant == 4) return launch2<128, 128, 2, 2, 2, false>(a, e, zpage, s, "conv_gemm2<128,128,st2>");
  return launch2<128, 128, 2, 2, 4, false>(a, e, zpage, s, "conv_gemm2<128,128>");
}

}  // namespace svc
