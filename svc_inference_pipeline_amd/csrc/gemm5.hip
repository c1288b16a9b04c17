// Fifth-generation implicit-GEMM Conv1d for gfx950: conv_gemm4's 4-wave 128 x 128 tile (2 workgroups per CU) with a
// DEEP LDS ring of half-depth K-steps.
//
// conv_gemm4 keeps one 64-deep K-tile in flight while it multiplies the other. Its counters on the DiffSVC gate GEMM
// (29 984 x 768 x 1152) put MFMA busy at 29 % with 32 % of wave time waiting, and the L2 -> CU stream at ≈ 21 B/clk per
// CU: Little's law with 32 KiB in flight per workgroup means an operand fetch under full-chip load takes ≈ 3 k cycles,
// far longer than the 512 MFMA cycles a wave has to hide it. This kernel keeps the bytes per K-step and the tile, and
// raises the bytes in flight:
//   * BK = 32 per ring slot (16 KiB: A 128 rows + B 128 rows of 64 B), NS slots, NS - 1 K-steps in flight;
//     NS = 4 -> 48 KiB in flight in 66 KiB of LDS, NS = 5 -> 64 KiB in flight in 80 KiB (still two workgroups per CU);
//   * one barrier per K-step: after it, the slot read in the previous step is refilled (every wave has passed it);
//   * slot image: 64 lines of 128 B, line = row & 63, 16-B chunk kv = (row >> 6) * 4 + c (c = the K chunk, 0..3),
//     stored at chunk position kv ^ (line & 6). A 16-lane ds_read_b128 group (rows r..r+15 of one 64-row half, chunks
//     fk and fk + 1) then covers 16 distinct 16-B bank slots, as conv_gemm4's 128-B rows do;
//   * LDS-DMA writes 1 KiB per wave instruction = 8 whole lines, so the swizzle is applied on the SOURCE side.
// Operand loader, zero rows outside the utterance and the LDS-staged epilogue are conv_gemm4's.
#include "common.h"
#include "epilogue.h"

namespace svc {

constexpr int G5_BM = 128, G5_BN = 128, G5_NT = 256;
constexpr int G5_SLOT = (G5_BM + G5_BN) * 64;  // 16 KiB
constexpr int G5_LDC = G5_BN + 4;
constexpr int g5_lds(int ns) { return (ns * G5_SLOT > G5_BM * G5_LDC * 4) ? ns * G5_SLOT : G5_BM * G5_LDC * 4; }

__device__ __forceinline__ int sw5(int line, int kv) { return kv ^ (line & 6); }

__device__ __forceinline__ void g5_dma(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void g5_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void g5_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int NS, bool CP32, bool PAIR>
__global__ __launch_bounds__(256, 2) void conv_gemm5_kernel(ConvGemmArgs a, EpiArgs e, const f16* zpage, float inv_cp) {
  extern __shared__ __align__(16) unsigned char sm5[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tile_n = wgid % a.ntiles_n, tile_m = wgid / a.ntiles_n;
  const int m0 = tile_m * G5_BM, n0 = tile_n * G5_BN;
  const int M = a.B * a.T_out;
  const int nk = a.Kpad / 32;
  const f16* zsrc = zpage + lane * 8;

  // DMA slots: instruction v (< 2) of this wave fills lines (wave * 2 + v) * 8 + (lane >> 3), chunk position lane & 7,
  // of the A and of the B image
  int a_t[2], a_c[2];
  const f16* a_p[2];
  const f16* b_p[2];
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int line = (wave * 2 + v) * 8 + (lane >> 3);
    const int kv = sw5(line, lane & 7);
    const int row = (kv >> 2) * 64 + line, c = kv & 3;
    a_c[v] = c;
    const int m = m0 + row;
    if (m < M) {
      const int b = m / a.T_out, t = m - b * a.T_out;
      a_t[v] = t * a.istride;
      a_p[v] = a.X + (int64_t)b * a.T_in * a.ldx + c * 8;
    } else {
      a_t[v] = -(1 << 29);
      a_p[v] = a.X;
    }
    b_p[v] = a.W + (int64_t)(n0 + row) * a.Kpad + c * 8;
  }
  auto issue = [&](int kt) {
    unsigned char* A = sm5 + (kt % NS) * G5_SLOT;
    unsigned char* Bm = A + G5_BM * 64;
    const bool live = kt < nk;
    if constexpr (CP32) {
      const int kg = kt * 32;
      const int tap = kg / a.Cp;
      const int c0 = kg - tap * a.Cp;
      const int shift = tap * a.tap_mul + a.tap_add;
      const int64_t off = (int64_t)shift * a.ldx + c0;
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int st = a_t[v] + shift;
        const bool ok = live && st >= 0 && st < a.T_in;
        g5_dma(ok ? (const void*)(a_p[v] + (int64_t)a_t[v] * a.ldx + off) : (const void*)zsrc,
               A + (wave * 2 + v) * 1024);
      }
    } else {
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int kg = kt * 32 + a_c[v] * 8;
        int tap = (int)((float)kg * inv_cp);
        if ((tap + 1) * a.Cp <= kg) ++tap;
        if (tap * a.Cp > kg) --tap;
        const int c = kg - tap * a.Cp;
        const int st = a_t[v] + tap * a.tap_mul + a.tap_add;
        const bool ok = live && kg < a.K && st >= 0 && st < a.T_in;
        g5_dma(ok ? (const void*)(a_p[v] + (int64_t)st * a.ldx + (c - a_c[v] * 8)) : (const void*)zsrc,
               A + (wave * 2 + v) * 1024);
      }
    }
#pragma unroll
    for (int v = 0; v < 2; ++v)
      g5_dma(live ? (const void*)(b_p[v] + kt * 32) : (const void*)zsrc, Bm + (wave * 2 + v) * 1024);
  };

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fk = lane >> 4;
  // fragment byte offsets inside a slot (A half = wm, B half = wn); line = i * 16 + fr, so line & 6 = fr & 6
  const int a_off = fr * 128 + (sw5(fr, wm * 4 + fk) << 4);
  const int b_off = G5_BM * 64 + fr * 128 + (sw5(fr, wn * 4 + fk) << 4);

#pragma unroll
  for (int p = 0; p < NS - 1; ++p) issue(p);
  for (int kt = 0; kt < nk; ++kt) {
    g5_vmwait<(NS - 2) * 4>();  // this wave's DMAs of step kt have landed (steps kt+1 .. kt+NS-2 may be in flight)
    g5_barrier();               // ... and everyone's; slot (kt - 1) % NS has been read by every wave
    issue(kt + NS - 1);         // past the end: zero-page loads into a slot nobody reads (keeps vmcnt counts static)
    const unsigned char* S = sm5 + (kt % NS) * G5_SLOT;
    half8 af[4], bf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const half8*>(S + a_off + i * 16 * 128);
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const half8*>(S + b_off + j * 16 * 128);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }
  g5_vmwait<0>();
  __syncthreads();
  float* Cs = reinterpret_cast<float*>(sm5);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(wm * 64 + i * 16 + fk * 4 + r) * G5_LDC + wn * 64 + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  epilogue_pass<G5_BM, G5_BN, G5_LDC, G5_NT, PAIR>(Cs, m0, n0, M, a, e, tid);
}

template <int NS>
static int launch_g5(const ConvGemmArgs& a, const EpiArgs& e, const f16* zpage, bool cp32, bool pair, int64_t grid,
                     float inv, hipStream_t s) {
  constexpr int lds = g5_lds(NS);
  static bool attr[2][2] = {};
  const void* fn = cp32 ? (pair ? (const void*)conv_gemm5_kernel<NS, true, true> : (const void*)conv_gemm5_kernel<NS, true, false>)
                        : (pair ? (const void*)conv_gemm5_kernel<NS, false, true> : (const void*)conv_gemm5_kernel<NS, false, false>);
  if (!attr[cp32][pair]) {
    SVC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr[cp32][pair] = true;
  }
  const dim3 g((unsigned)grid), b(G5_NT);
  if (cp32 && pair) hipLaunchKernelGGL((conv_gemm5_kernel<NS, true, true>), g, b, lds, s, a, e, zpage, inv);
  else if (cp32) hipLaunchKernelGGL((conv_gemm5_kernel<NS, true, false>), g, b, lds, s, a, e, zpage, inv);
  else if (pair) hipLaunchKernelGGL((conv_gemm5_kernel<NS, false, true>), g, b, lds, s, a, e, zpage, inv);
  else hipLaunchKernelGGL((conv_gemm5_kernel<NS, false, false>), g, b, lds, s, a, e, zpage, inv);
  return SVC_OK;
}

// ns = ring slots (4 or 5)
int conv_gemm5(const ConvGemmArgs& a0, const EpiArgs& e, const f16* zpage, int ns, hipStream_t s) {
  ConvGemmArgs a = a0;
  SVC_REQUIRE(a.Cp % 8 == 0 && a.ldx % 8 == 0 && a.Kpad % 64 == 0 && a.N % 4 == 0, "conv_gemm5: layout");
  SVC_REQUIRE(((uintptr_t)a.X & 15) == 0 && ((uintptr_t)a.W & 15) == 0, "conv_gemm5: 16-B alignment");
  SVC_REQUIRE(ns == 4 || ns == 5, "conv_gemm5: ns=%d", ns);
  const bool pair = e.kind == EPI_GATE;
  SVC_REQUIRE(!pair || a.N % 64 == 0, "conv_gemm5: paired epilogue needs N %% 64 == 0");
  const int M = a.B * a.T_out;
  a.ntiles_n = cdiv(a.N, G5_BN);
  a.halo = 0;
  const int64_t grid = (int64_t)cdiv(M, G5_BM) * a.ntiles_n;
  SVC_REQUIRE(grid > 0 && grid < (1ll << 31), "conv_gemm5: bad grid");
  const bool cp32 = a.Cp % 32 == 0 && a.K == a.Kpad;
  const double kreal = (double)(a.K / a.Cp) * a.Cvalid;
  const char* tag = ns == 4 ? (pair ? "conv_gemm5<4,pair>" : "conv_gemm5<4>") : (pair ? "conv_gemm5<5,pair>" : "conv_gemm5<5>");
  const int tok = prof_begin(tag, 2.0 * M * (double)a.N * kreal, 0.0, s);
  const float inv = 1.0f / (float)a.Cp;
  const int st = ns == 4 ? launch_g5<4>(a, e, zpage, cp32, pair, grid, inv, s) : launch_g5<5>(a, e, zpage, cp32, pair, grid, inv, s);
  prof_end(tok, s);
  if (st != SVC_OK) return st;
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
