// Fourth-generation implicit-GEMM Conv1d for gfx950: a 4-wave 128 x 128 tile built for 2 workgroups per CU.
//
// conv_gemm3 (8 waves, staggered ping-pong inside one workgroup) pays for its phase barriers with a small amount of
// MFMA work per phase on 128-wide tiles (4 MFMAs per wave per phase at 128 x 128) and cannot overlap its prologue
// and epilogue with anything. This kernel takes the other route on the short-K DiffSVC / BigVGAN shapes:
//   * 4 waves = 2 (M) x 2 (N), wave tile 64 x 64: 32 v_mfma_f32_16x16x32_f16 per wave per K-tile (BK = 64), fragments
//     read straight from LDS;
//   * 2 LDS K-tile stages (A 128 rows + B 128 rows of 128 B each, 32 KiB per stage) filled by LDS-DMA one K-tile ahead,
//     one barrier per K-tile;
//     with the C-staging epilogue the workgroup needs 66 KiB, so two workgroups share a CU and one's prologue /
//     epilogue runs beside the other's MFMAs (inter-workgroup overlap in place of intra-workgroup staggering);
//   * the same operand images (128-B rows, 16-B chunk swizzle kv ^ (row & 6)), A loader (per-tap row shifts, zero
//     rows outside the utterance) and LDS-staged vector epilogue (epilogue.h) as conv_gemm3.
#include <type_traits>

#include "common.h"
#include "epilogue.h"

namespace svc {

constexpr int G4_BM = 128, G4_BN = 128, G4_NT = 256;
constexpr int G4_STAGE = (G4_BM + G4_BN) * 128;  // 32 KiB
constexpr int G4_LDC = G4_BN + 4;
constexpr int G4_LDS = (2 * G4_STAGE > G4_BM * G4_LDC * 4) ? 2 * G4_STAGE : G4_BM * G4_LDC * 4;

__device__ __forceinline__ int sw4(int row, int kv) { return kv ^ (row & 6); }

__device__ __forceinline__ void g4_dma(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// CP64 form: LDS-DMA through buffer descriptors. A lane's 32-bit voffset is fixed per conv tap (per K-tile for W) and
// the K-tile's channel offset is the scalar soffset, so the K-loop issues its DMAs with no per-lane address arithmetic;
// a padding row (outside its utterance) gets a voffset past the descriptor's range, which the hardware bounds check
// turns into zeros.
constexpr uint32_t G4_OOR = 0x7ffffff0u;
__device__ __forceinline__ void g4_bdma(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, unsigned char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, (int)voff, (int)soff,
                                           0, 0);
}

template <int N>
__device__ __forceinline__ void g4_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void g4_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// DIRECT (gate epilogue only): the MFMAs run with the operands swapped, so a lane's accumulator holds 4 CONSECUTIVE
// packed columns of one output row, and the gate column block j (< 2) and its filter partner j + 2 (packed column + 32)
// sit in the same lane. The gate is then applied in registers: no 64 KiB f32 round trip through LDS, the conditioner
// projection and bias are prefetched into registers under the last K-tile's MFMAs, and each lane stores 4 channels
// (8 B) per row.
// (Round 2 also had a register read-modify-write epilogue for the DiffSVC output projection here; faster alone, slower
// beside the sampler's other stream, it was removed in round 3.)
// blockIdx -> a workgroup index whose consecutive values land on one XCD (tiles sharing A rows share that XCD's L2)
__device__ __forceinline__ int g4_xcd_remap() {
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
}

// One 128 x 128 output tile (index wgid, N-tiles fastest) of the implicit GEMM, by the calling 256-thread workgroup.
template <bool CP64, bool PAIR, bool DIRECT, bool BF>
__device__ __forceinline__ void conv_gemm4_tile(const ConvGemmArgs& a, const EpiArgs& e, const f16* zpage,
                                                float inv_cp, int wgid, unsigned char* sm4) {
  static_assert(!DIRECT || PAIR, "the register epilogue is the gate's");
  using O = Op16<BF>;  // operand format (binary16 or bfloat16)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tile_n = wgid % a.ntiles_n, tile_m = wgid / a.ntiles_n;
  const int m0 = tile_m * G4_BM, n0 = tile_n * G4_BN;
  const int M = a.B * a.T_out;
  const int nk = a.Kpad / 64;
  const f16* zsrc = zpage + lane * 8;

  // DMA slots: image rows (wave * 4 + v) * 8 + (lane >> 3), v < 4, for A and for B
  int a_t[4], a_kv[4], a_tin[4];
  const f16* a_p[4];
  const f16* b_p[4];
  uint32_t a_row[4], a_voff[4], b_voff[4];  // CP64: byte offsets of the lane's A row (tap shift 0) / W row
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int row = (wave * 4 + v) * 8 + (lane >> 3);
    const int kv = sw4(row, lane & 7);
    a_kv[v] = kv;
    const int m = m0 + row;
    if (m < M) {
      const int b = m / a.T_out, t = m - b * a.T_out;
      a_t[v] = t * a.istride;
      a_tin[v] = valid_in_rows(a, b);
      a_p[v] = a.X + (int64_t)b * a.T_in * a.ldx + kv * 8;
      a_row[v] = (uint32_t)(((b * a.T_in + a_t[v]) * a.ldx + kv * 8) * 2);
    } else {
      a_t[v] = -(1 << 29);
      a_tin[v] = 0;
      a_p[v] = a.X;
      a_row[v] = 0u;
    }
    a_voff[v] = G4_OOR;
    b_p[v] = a.W + (int64_t)(n0 + row) * a.Kpad + kv * 8;
    b_voff[v] = (uint32_t)(((n0 + row) * a.Kpad + kv * 8) * 2);
  }
  // CP64 descriptors (unused otherwise); extents checked on the host (< 1 GiB: no voffset + soffset wraps)
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(a.X), (short)0, a.B * a.T_in * a.ldx * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(a.W), (short)0, a.ntiles_n * G4_BN * a.Kpad * 2, 0x00020000);
  auto issue = [&](int kt) {
    unsigned char* A = sm4 + (kt & 1) * G4_STAGE;
    unsigned char* Bm = A + G4_BM * 128;
    if constexpr (CP64) {
      const int kg = kt * 64;
      const int tap = kg / a.Cp;
      const int c0 = kg - tap * a.Cp;
      if (c0 == 0) {  // a new tap (wave-uniform): the rows it reads, and which of them are padding
        const int shift = tap * a.tap_mul + a.tap_add;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int st = a_t[v] + shift;
          a_voff[v] = st >= 0 && st < a_tin[v] ? a_row[v] + (uint32_t)(shift * a.ldx * 2) : G4_OOR;
        }
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) g4_bdma(rx, a_voff[v], (uint32_t)(c0 * 2), A + (wave * 4 + v) * 1024);
#pragma unroll
      for (int v = 0; v < 4; ++v) g4_bdma(rw, b_voff[v], (uint32_t)(kt * 128), Bm + (wave * 4 + v) * 1024);
      return;
    } else {
      const bool live = kt < nk;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int kg = kt * 64 + a_kv[v] * 8;
        int tap = (int)((float)kg * inv_cp);
        if ((tap + 1) * a.Cp <= kg) ++tap;
        if (tap * a.Cp > kg) --tap;
        const int c = kg - tap * a.Cp;
        const int st = a_t[v] + tap * a.tap_mul + a.tap_add;
        const bool ok = live && kg < a.K && st >= 0 && st < a_tin[v];
        g4_dma(ok ? (const void*)(a_p[v] + (int64_t)st * a.ldx + (c - a_kv[v] * 8)) : (const void*)zsrc,
               A + (wave * 4 + v) * 1024);
      }
#pragma unroll
      for (int v = 0; v < 4; ++v)
        g4_dma(live ? (const void*)(b_p[v] + kt * 64) : (const void*)zsrc, Bm + (wave * 4 + v) * 1024);
    }
  };

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fk = lane >> 4;

  // DIRECT epilogue operands: rows m0 + wm*64 + i*16 + fr, packed columns nw + j*16 + fk*4 .. +3 (j < 2) and + 32
  const int nw = n0 + wn * 64;
  const bool wave_cols = nw < a.N;
  union H4 { uint2 u; f16 h[4]; };
  H4 cpg[4][2], cpf[4][2];
  float4 bg[2], bfl[2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) cpg[i][j].u = cpf[i][j].u = make_uint2(0u, 0u);  // diagnostics runs without cp
  bg[0] = bg[1] = bfl[0] = bfl[1] = make_float4(0.f, 0.f, 0.f, 0.f);
  // row group i of the epilogue operands; group 0 also loads the bias
  auto prefetch = [&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if (!wave_cols || e.cp == nullptr) return;
    if constexpr (i == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bg[j] = *reinterpret_cast<const float4*>(e.bias + nw + j * 16 + fk * 4);
        bfl[j] = *reinterpret_cast<const float4*>(e.bias + nw + 32 + j * 16 + fk * 4);
      }
    }
    const int m = min(m0 + wm * 64 + i * 16 + fr, M - 1);  // clamped rows are loaded but never stored
    const f16* c = e.cp + (int64_t)m * e.ld_cp + nw + fk * 4;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      cpg[i][j].u = *reinterpret_cast<const uint2*>(c + j * 16);
      cpf[i][j].u = *reinterpret_cast<const uint2*>(c + 32 + j * 16);
    }
  };

  // One barrier per K-tile: DMA(kt + 1) is issued right after the barrier of iteration kt (which also proves every wave
  // has finished reading that stage in iteration kt - 1) and lands under the MFMAs of iteration kt.
  issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    g4_vmwait<0>();  // this wave's DMAs of stage kt have landed (nothing younger is outstanding)
    g4_barrier();    // ... and everyone's; stage (kt + 1) & 1 is free
    if (kt + 1 < nk) issue(kt + 1);
    if constexpr (DIRECT) {
      if (kt + 1 == nk) {  // under the last K-tile's MFMAs (spreading these over earlier K-steps measured no better)
        prefetch(std::integral_constant<int, 0>{});
        prefetch(std::integral_constant<int, 1>{});
        prefetch(std::integral_constant<int, 2>{});
        prefetch(std::integral_constant<int, 3>{});
      }
    }
    const unsigned char* A = sm4 + (kt & 1) * G4_STAGE;
    const unsigned char* Bm = A + G4_BM * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      half8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + fr;
        af[i] = *reinterpret_cast<const half8*>(A + row * 128 + (sw4(row, s * 4 + fk) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wn * 64 + j * 16 + fr;
        bf[j] = *reinterpret_cast<const half8*>(Bm + row * 128 + (sw4(row, s * 4 + fk) << 4));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if constexpr (DIRECT)  // C^T fragment: acc[i][j][r] = C[row fr of block i][col fk*4 + r of block j]
            acc[i][j] = O::mfma(bf[j], af[i], acc[i][j]);
          else
            acc[i][j] = O::mfma(af[i], bf[j], acc[i][j]);
        }
      __builtin_amdgcn_s_setprio(0);
    }
  }
  if constexpr (DIRECT && PAIR) {
    if (!wave_cols) return;
    if (e.y16 == nullptr) {  // diagnostics sink (svc_gemm_bench epi 3 / 5): keep the MFMAs and cp reads, no stores
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) sum += (float)cpg[i][j].h[0] + (float)cpf[i][j].h[3];
      if (sum == 1.2345e-38f && e.out32) e.out32[0] = sum;
      return;
    }
    const int chb = (nw >> 6) * 32 + fk * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + i * 16 + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float4 g = make_float4(acc[i][j][0] + bg[j].x, acc[i][j][1] + bg[j].y, acc[i][j][2] + bg[j].z,
                                     acc[i][j][3] + bg[j].w);
        const float4 f = make_float4(acc[i][j + 2][0] + bfl[j].x, acc[i][j + 2][1] + bfl[j].y,
                                     acc[i][j + 2][2] + bfl[j].z, acc[i][j + 2][3] + bfl[j].w);
        H4 pk;
        pk.h[0] = O::enc_lo(gate_act(g.x + O::dec(cpg[i][j].h[0]), f.x + O::dec(cpf[i][j].h[0])));
        pk.h[1] = O::enc_lo(gate_act(g.y + O::dec(cpg[i][j].h[1]), f.y + O::dec(cpf[i][j].h[1])));
        pk.h[2] = O::enc_lo(gate_act(g.z + O::dec(cpg[i][j].h[2]), f.z + O::dec(cpf[i][j].h[2])));
        pk.h[3] = O::enc_lo(gate_act(g.w + O::dec(cpg[i][j].h[3]), f.w + O::dec(cpf[i][j].h[3])));
        // 4 channels (8 B) per lane and row; a 16-B form (quad exchange between lanes fk, fk ^ 1) measured 2-3 % slower
        *reinterpret_cast<uint2*>(e.y16 + (int64_t)m * e.ldy16 + chb + j * 16) = pk.u;
      }
    }
    return;
  }
  g4_vmwait<0>();
  __syncthreads();
  // acc[i][j][r] = C[wm*64 + i*16 + fk*4 + r][wn*64 + j*16 + fr]
  float* Cs = reinterpret_cast<float*>(sm4);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(wm * 64 + i * 16 + fk * 4 + r) * G4_LDC + wn * 64 + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  epilogue_pass<G4_BM, G4_BN, G4_LDC, G4_NT, PAIR, BF>(Cs, m0, n0, M, a, e, tid);
}

template <bool CP64, bool PAIR, bool DIRECT, bool BF>
__global__ __launch_bounds__(256, 2) void conv_gemm4_kernel(ConvGemmArgs a, EpiArgs e, const f16* zpage, float inv_cp) {
  extern __shared__ __align__(16) unsigned char sm4[];
  conv_gemm4_tile<CP64, PAIR, DIRECT, BF>(a, e, zpage, inv_cp, g4_xcd_remap(), sm4);
}

// direct: the register gate epilogue (paired epilogues only), otherwise the LDS-staged epilogue_pass
int conv_gemm4(const ConvGemmArgs& a0, const EpiArgs& e, const f16* zpage, hipStream_t s, bool direct_gate) {
  ConvGemmArgs a = a0;
  SVC_REQUIRE(a.Cp % 8 == 0 && a.ldx % 8 == 0 && a.Kpad % 64 == 0 && a.N % 4 == 0, "conv_gemm4: layout");
  SVC_REQUIRE(((uintptr_t)a.X & 15) == 0 && ((uintptr_t)a.W & 15) == 0, "conv_gemm4: 16-B alignment");
  const bool pair = e.kind == EPI_GATE;
  SVC_REQUIRE(!pair || a.N % 64 == 0, "conv_gemm4: paired epilogue needs N %% 64 == 0");
  const int M = a.B * a.T_out;
  a.ntiles_n = cdiv(a.N, G4_BN);
  const int64_t grid = (int64_t)cdiv(M, G4_BM) * a.ntiles_n;
  SVC_REQUIRE(grid > 0 && grid < (1ll << 31), "conv_gemm4: bad grid");
  // the buffer-descriptor (CP64) form: one tap per K-tile, and X / W extents addressable by 32-bit offsets
  const bool cp64 = a.Cp % 64 == 0 && a.K == a.Kpad && (int64_t)a.B * a.T_in * a.ldx * 2 < (1ll << 30) &&
                    (int64_t)a.ntiles_n * G4_BN * a.Kpad * 2 < (1ll << 30);
  const bool direct = direct_gate && pair;
  const int bf = a.bf16 ? 1 : 0;
#define G4_FORMS(BFV)                                                                                              \
  {{{(const void*)conv_gemm4_kernel<false, false, false, BFV>, nullptr},                                           \
    {(const void*)conv_gemm4_kernel<false, true, false, BFV>, (const void*)conv_gemm4_kernel<false, true, true, BFV>}}, \
   {{(const void*)conv_gemm4_kernel<true, false, false, BFV>, nullptr},                                            \
    {(const void*)conv_gemm4_kernel<true, true, false, BFV>, (const void*)conv_gemm4_kernel<true, true, true, BFV>}}}
  const void* fns[2][2][2][2] = {G4_FORMS(false), G4_FORMS(true)};
#undef G4_FORMS
  const void* fn = fns[bf][cp64][pair][direct];
  if (int st = ensure_dyn_lds(fn, G4_LDS)) return st;
  const double kreal = (double)(a.K / a.Cp) * a.Cvalid;
  const char* tag = direct ? "conv_gemm4<128,128,gate>" : pair ? "conv_gemm4<128,128,pair>" : "conv_gemm4<128,128>";
  const int tok = prof_begin(tag, 2.0 * M * (double)a.N * kreal, 0.0, s);
  const dim3 g((unsigned)grid), b(G4_NT);
  const float inv = 1.0f / (float)a.Cp;
  void* args[] = {&a, const_cast<EpiArgs*>(&e), const_cast<const f16**>(&zpage), const_cast<float*>(&inv)};
  SVC_HIP_CHECK(hipLaunchKernel(fn, g, b, args, G4_LDS, s));
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
