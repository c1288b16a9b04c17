// BigVGAN AMP-block convolution for small channel counts (C = 24 / 48 / 96, the late generator stages),
// with the Activation1d that precedes it fused in (modules/bigvgan.py:424-431 AMPBlock1.forward:
// xt = a1(x); xt = c1(xt); xt = a2(xt); xt = c2(xt); x = xt + x — Activation1d :234-307, SnakeBeta :146-159).
//
// At these widths a conv is HBM-bound: per output element it does 2*k*C MACs (<= 2.1 kFLOP) against 8+ B of
// traffic. So the kernel is built for memory, not the matrix pipe. A workgroup owns BT consecutive output
// rows of one utterance, i.e. one contiguous [BT][C] block of every time-major tensor:
//   1. act -> LDS: SnakeBeta (x2 up-sample, snake, x2 down-sample) of rows [t0-P, t0+BT+P), P = (k-1)/2*d,
//      streamed from x (f32) with per-thread sliding register windows (as activation1d_rs_kernel), stored
//      f16 into an LDS image. Rows outside [0, L) are zeros: the conv's own zero padding.
//   2. conv: v_mfma_f32_16x16x32_f16 with A fragments read from the LDS image at row r + tap*d (row stride
//      padded so 16-row fragment reads are conflict-free) and B = the packed weights [Npad][Kpad] (L1/L2).
//   3. epilogue: bias, residual add (add_row), resblock mean accumulation (acc32 / acc_div), f32 and/or f16 stores
//      as 16-B / 8-B vectors over whole contiguous rows (the C tile staged through the dead image's LDS in row blocks).
// The activation never round-trips through HBM, and every HBM access is a coalesced 16-byte stream.
#include <type_traits>

#include "common.h"
#include "snake.h"
#include "amp_conv.h"

namespace svc {

constexpr int AMP_NT = 256;

// Activation run length for an image of `rows` rows: the shortest multiple of the row block that gives every
// (channel group, run) task to its own thread (one exposed load latency per thread). The image is allocated for
// whole runs (nruns * RUN rows), so that no run is partial: a partial run would take the edge form of the channel-pair
// activation, and its lanes would make their whole wave run both forms before the barrier.
__host__ __device__ constexpr int amp_run_len(int C, int rows, int nt = AMP_NT) {
  const int blk = 4, ngrp = C / 2;
  const int nr_fit = nt / ngrp > 1 ? nt / ngrp : 1;
  return ((rows + nr_fit - 1) / nr_fit + blk - 1) / blk * blk;
}

template <int C, bool NOACT = false>
struct AmpCfg {
  // 256 output rows per workgroup (halo share of the act work). C = 96 (fused, and NOACT, the plain conv) on 2 x 2 waves
  // (each 128 rows x 48 columns), so that the weight fragments a wave reads from L1 / L2 per K-step serve 8 row
  // fragments: the round-5 128-row tiles on 4 x 1 waves (every wave reading all of W per k-loop, 2 row fragments each)
  // were L2-bound, 11.5 against 8.3 ms per step for the C = 96 convs (profiles/r06_ab/r06v_*, r06w_*)
  // C = 24 / 48: 512-row tiles on 4 x 1 waves (128 rows each, the same weight reuse), 2 workgroups per CU: against the
  // round-5 256-row tiles at 4 per CU, 16.95 -> 16.0 ms per step (profiles/r06_ab/r06y_amp_narrow_512rows.txt)
  // C = 192: 8 waves on 2 x 4 (each 128 rows x 48 columns), one workgroup per CU (the image is 127-133 KiB).
  static constexpr bool WIDE = C >= 96;
  static constexpr int NT = C == 192 ? 512 : AMP_NT;    // threads
#ifndef AMP_BT192
#define AMP_BT192 256
#endif
  static constexpr int BT = C == 192 ? AMP_BT192 : (WIDE ? 256 : 512);
  static constexpr int WN = C == 192 ? 4 : (WIDE ? 2 : 1), WM = NT / 64 / WN;  // wave grid: WM row x WN column blocks
  static constexpr int NPART = 4;                       // epilogue staging parts (row blocks of BT / NPART)
  static constexpr int OCC = (C == 192 && BT == 256) ? 1 : 2;  // workgroups per CU (launch bound)
  static constexpr int MAXP = 32;                   // max conv padding (k-1)/2*d supported
  // f16 row stride (96 / 96 / 224 B). A K-step's ds_read_b128 mixes lanes of two taps (rows tap*d apart) and CPT
  // chunks per tap, so the bank pattern depends on the stride: modelled over k in {3,7,11}, d in {1,3,5} with the
  // guide's 4 x 16 lane groups, the round-4 strides 24 / 56 / 104 cost 1.94 / 1.94 / 2.0 LDS cycles per ideal one,
  // these 1.44 / 1.06 / 1.0 (r05 search; C = 24 takes 48 halves, twice its row: the image stays within 4 WGs per CU)
  // (C = 192: 26 chunks, the stride class of C = 96's 14: 8 consecutive rows on distinct bank slots)
  static constexpr int LDA = C == 192 ? 208 : (C == 96 ? 112 : 48);
  static constexpr int ROWS = BT + 2 * MAXP;
  static constexpr int FN = (C + 15) / 16;          // 16-column fragments
  static constexpr int FNW = FN / WN;               // per wave
  static constexpr int A_BYTES = (NOACT ? ROWS : ROWS + amp_run_len(C, ROWS, NT)) * LDA * 2;  // whole runs of the largest image
  // the epilogue stages the C tile in NPART row blocks through the same LDS (the image is dead by then)
  static constexpr int LDC = C + 4;  // f32 staging row stride
  static constexpr int STG_BYTES = BT / NPART * LDC * 4;
  static constexpr int LDS = A_BYTES > STG_BYTES ? A_BYTES : STG_BYTES;
  static_assert(C % 8 == 0 && LDA % 8 == 0 && FN % WN == 0 && (BT / 16) % WM == 0, "16-B fragment rows, wave grid");
  static_assert(BT / WM <= BT / NPART || (BT / WM) % (BT / NPART) == 0, "a wave's rows: within one part or whole parts");
};

// SnakeBeta of the channel pair (c, c+1) for global rows [rs, re) into the LDS image (row r of the image = global row
// r0 + r), in blocks of BLK rows on packed f32 ops (snake.h); re - rs is a multiple of BLK. EDGE: the run lies within 6
// rows of an utterance end: clamped loads, the up-sampled signal's replicate padding at both ends and zero rows outside
// [0, Lb) (the conv's own zero padding). Other runs take none of these.
template <typename TX, int BLK, int LDA, bool EDGE>
__device__ __forceinline__ void amp_act_pair(__amdgpu_buffer_rsrc_t rx, uint32_t xo, uint32_t xs, f16* img, int r0,
                                             int rs, int re, int Lb, int c, const float (&f)[12],
                                             const float (&f2)[12], const SnakeCoef2& kc) {
  auto xl = [&](int t) __attribute__((always_inline)) {
    if (EDGE) t = t < 0 ? 0 : (t >= Lb ? Lb - 1 : t);
    return act_load<TX>(rx, xo + (uint32_t)t * xs, 0);
  };
  f32x2 s0 = {0.f, 0.f}, sE = {0.f, 0.f};  // s at j = 0 and j = 2Lb-1
  if (EDGE) {
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      s0 += xl(-3 + a) * f2[11 - 2 * a];
      sE += xl(Lb - 3 + a) * f2[10 - 2 * a];
    }
    s0 = snake2(s0, kc);
    sE = snake2(sE, kc);
  }
  auto s_at = [&](const f32x2* xw, int i, int j) __attribute__((always_inline)) {
    const f32x2 o = snake_up(xw, i, f2, kc);
    return EDGE ? (j < 0 ? s0 : (j > 2 * Lb - 1 ? sE : o)) : o;
  };
  // the next block's rows are loaded while this block computes, kept in their loaded form (f16: one raw word per
  // channel pair): one exposed load latency per run instead of one per block (C = 24 launches 4.5-6 % faster, C = 48
  // 2-3 %, profiles/r06_ab/r06n_amp_act_prefetch.txt)
  auto xlr = [&](int t) __attribute__((always_inline)) {
    if (EDGE) t = t < 0 ? 0 : (t >= Lb ? Lb - 1 : t);
    return act_load_raw<TX>(rx, xo + (uint32_t)t * xs, 0);
  };
  f32x2 xw[BLK + 10], sw[2 * BLK + 10];
  act_raw_t<TX> xn[BLK];
#pragma unroll
  for (int k = 0; k < 10; ++k) xw[k] = xl(rs - 5 + k);
#pragma unroll
  for (int k = 0; k < BLK; ++k) xn[k] = xlr(rs + 5 + k);
#pragma unroll
  for (int i = 0; i < 10; ++i) sw[i] = s_at(xw, i, 2 * rs - 5 + i);
  for (int t = rs; t < re; t += BLK) {
    const uint32_t xrow = xo + (uint32_t)(t + 5) * xs;
#pragma unroll
    for (int k = 0; k < BLK; ++k) xw[10 + k] = act_cvt<TX>(xn[k]);
    if (t + BLK < re) {
#pragma unroll
      for (int k = 0; k < BLK; ++k) xn[k] = EDGE ? xlr(t + BLK + 5 + k) : act_load_raw<TX>(rx, xrow, (BLK + k) * xs);
    }
#pragma unroll
    for (int p = 0; p < BLK; ++p) {
      sw[10 + 2 * p] = s_at(xw, 10 + 2 * p, 2 * t + 5 + 2 * p);
      sw[11 + 2 * p] = s_at(xw, 11 + 2 * p, 2 * t + 6 + 2 * p);
      const int row = t + p;
      f32x2 y = snake_down(sw + 2 * p, f);
      if (EDGE && (row < 0 || row >= Lb)) y = f32x2{0.f, 0.f};
      *reinterpret_cast<unsigned*>(img + (row - r0) * LDA + c) = f16x2_sat(y);
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) xw[k] = xw[BLK + k];
#pragma unroll
    for (int i = 0; i < 10; ++i) sw[i] = sw[2 * BLK + i];
  }
}

// Launch bound: AmpCfg::OCC workgroups (waves per SIMD), under which the compiler keeps the accumulators in the unified
// VGPR file (round 5, 4 per CU: without an occupancy target it split the file into VGPRs + AGPRs at 5 waves). The activation runs on channel pairs with packed
// f32 ops in 4-row blocks for every C (round 4: C = 96 had a single-channel 8-row form, removed with the packed
// clamp-free form).
// NOACT: the plain conv of an f16 input with no activation before it (p.x16; svc_bigvgan's rate-2 up-sampling as one
// conv, VStage::upc): phase 1 copies the rows into the image (16-B loads, zeros outside [0, Lb)) and the conv reads
// every tap from it, so each input row leaves HBM / L2 once per workgroup instead of once per tap as in conv_gemm3's
// implicit GEMM. (Round 6 also ran the C = 96 / 192 resblock convs after activation1d this way: 8.3 against conv_gemm3's
// 11.5 ms per step at C = 96, but fused with the activation it is faster still, r06w / r06x / r06z.)
template <int C, bool X16 = false, bool NOACT = false>
__global__ __launch_bounds__((AmpCfg<C, NOACT>::NT), (AmpCfg<C, NOACT>::OCC)) void amp_conv_kernel(AmpConvArgs p, EpiArgs e) {
  using CF = AmpCfg<C, NOACT>;
  extern __shared__ __align__(16) unsigned char amp_sm[];
  f16* As = reinterpret_cast<f16*>(amp_sm);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int L = p.L;
  const int ntiles = (L + CF::BT - 1) / CF::BT;
  const int b = blockIdx.x / ntiles, t0 = (blockIdx.x - b * ntiles) * CF::BT;
  // ragged batches: this utterance ends at Lb (activation replicate padding, conv zero padding); the rows keep the
  // batch stride L. Tiles wholly past Lb have nothing to compute (block-uniform exit before any barrier).
  const int Lb = p.tv ? min(L, p.tv[b] * p.tv_mul) : L;
  if (t0 >= Lb) return;
  // a negative dilation walks the taps downwards (tap 0 reads row t + P): the ConvTranspose phase pairs of
  // svc_bigvgan's combined up-sampling conv, whose per-phase tap order this keeps
  const int ad = p.d < 0 ? -p.d : p.d;
  const int P = (p.k - 1) / 2 * ad;
  const int rows = CF::BT + 2 * P;
  const int tap0 = p.d < 0 ? 2 * P : 0;

  // ------------------------------------------------------------------ 1. SnakeBeta -> LDS (f16)
  if constexpr (NOACT) {
    if (!(p.dbg & 1)) {
      constexpr int CH = C / 8;                                      // 16-B chunks per row
      constexpr int IT = ((CF::BT + 2 * CF::MAXP) * CH + CF::NT - 1) / CF::NT;  // chunks per thread, largest image
      const int r0 = t0 - P, n = rows * CH;
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<f16*>(p.x16 + (int64_t)b * L * C), (short)0, Lb * C * 2, 0x00020000);
      uint4 v[IT];
      // rows outside [0, Lb) lie outside the descriptor's range (a negative row wraps past it): they load as zeros
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int idx = tid + it * CF::NT, r = idx / CH, q = idx - r * CH;
        const uint32_t vo = (idx < n && r0 + r >= 0) ? (uint32_t)(((r0 + r) * C + q * 8) * 2) : 0x80000000u;
        v[it] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, vo, 0, 0));
      }
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int idx = tid + it * CF::NT, r = idx / CH, q = idx - r * CH;
        if (idx < n) *reinterpret_cast<uint4*>(As + r * CF::LDA + q * 8) = v[it];
      }
    }
  } else if (!(p.dbg & 1)) {
    constexpr int BLK = 4;
    using TX = typename std::conditional<X16, f16, float>::type;
    float f[12], f2[12];  // f2: the up-sampling taps with its factor 2 (exact)
#pragma unroll
    for (int q = 0; q < 12; ++q) {
      f[q] = p.filt[q];
      f2[q] = 2.0f * f[q];
    }
    constexpr int ngrp = C / 2;
    // (LDS conflicts, VERDICT r03 item 4: making the activation stores conflict-free by the choice of RUN moved the
    // kernel's conflict share only 0.47 -> 0.41 and no timing, r04q; the rest are the conv phase's fragment reads)
    const int RUN = amp_run_len(C, rows, CF::NT);
    const int nruns = (rows + RUN - 1) / RUN;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(X16 ? (const void*)p.x16 : (const void*)p.x), (short)0,
        (int)((int64_t)p.B * L * C * sizeof(TX)), 0x00020000);
    for (int task = tid; task < ngrp * nruns; task += CF::NT) {
      const int cg = task % ngrp, ru = task / ngrp;
      const int c = cg * 2;
      const int rs = t0 - P + ru * RUN, re = rs + RUN;  // global rows of this run (whole runs: the image has room)
      const SnakeCoef2 kc = snake_coef2(p.alpha_log, p.beta_log, c);
      const uint32_t xo = (uint32_t)(((int64_t)b * L * C + c) * sizeof(TX)), xs = (uint32_t)(C * sizeof(TX));
      if (rs - 6 < 0 || re + 6 > Lb)
        amp_act_pair<TX, BLK, CF::LDA, true>(rx, xo, xs, As, t0 - P, rs, re, Lb, c, f, f2, kc);
      else
        amp_act_pair<TX, BLK, CF::LDA, false>(rx, xo, xs, As, t0 - P, rs, re, Lb, c, f, f2, kc);
    }
  }
  __syncthreads();

  // ------------------------------------------------------------------ 2. conv on the matrix pipe
  constexpr int MW = CF::BT / 16 / CF::WM;  // 16-row fragments per wave
  constexpr int FNW = CF::FNW;              // 16-column fragments per wave
  constexpr int CPT = C / 8;                // 8-wide k chunks per tap
  const int wm = wave / CF::WN, wn = wave - wm * CF::WN;
  floatx4 acc[MW][FNW];
#pragma unroll
  for (int i = 0; i < MW; ++i)
#pragma unroll
    for (int j = 0; j < FNW; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int ks = (p.k * C + 31) / 32;
  const int fr = lane & 15, fk = lane >> 4;
  const f16* wrow = p.W + (int64_t)(wn * FNW * 16 + fr) * p.Kpad + fk * 8;
  half8 bn[FNW];  // weight fragments of the next k-step, loaded one step ahead (L2 latency off the MFMA path)
#pragma unroll
  for (int j = 0; j < FNW; ++j) bn[j] = *reinterpret_cast<const half8*>(wrow + (int64_t)j * 16 * p.Kpad);
  for (int s = 0; s < ((p.dbg & 2) ? 0 : ks); ++s) {
    const int q = 4 * s + fk;
    int tap = q / CPT, cc = q - tap * CPT;
    if (tap >= p.k) tap = cc = 0;  // K tail: zero weights, any finite A
    half8 af[MW], bf[FNW];
#pragma unroll
    for (int j = 0; j < FNW; ++j) bf[j] = bn[j];
    if (s + 1 < ks) {
#pragma unroll
      for (int j = 0; j < FNW; ++j)
        bn[j] = *reinterpret_cast<const half8*>(wrow + (int64_t)j * 16 * p.Kpad + (s + 1) * 32);
    }
#pragma unroll
    for (int i = 0; i < MW; ++i) {
      const int r = (wm * MW + i) * 16 + fr + tap0 + tap * p.d;
      af[i] = *reinterpret_cast<const half8*>(As + r * CF::LDA + cc * 8);
    }
#pragma unroll
    for (int i = 0; i < MW; ++i)
#pragma unroll
      for (int j = 0; j < FNW; ++j)  // C^T fragment: acc[i][j][r] = C[row fr of block i][channel j*16 + fk*4 + r]
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0);
  }
  // ------------------------------------------------------------------ 3. epilogue: each lane owns 4 consecutive
  // channels of one row (operand-swapped MFMAs). The workgroup's output block is [BT][C] contiguous in every tensor, so
  // the C tile goes through LDS in NPART row blocks (the activation image is dead after the k-loop) and the epilogue
  // operands and outputs move as whole contiguous rows: a wave's 16-B accesses cover 1 KiB in a row instead of 16
  // pieces of 64 B at the row stride (SVC_AMP_DBG 4: no epilogue; 8: that register epilogue instead).
  const int nvalid = (p.dbg & 4) ? 0 : min(CF::BT, Lb - t0);
  const int64_t base = ((int64_t)b * L + t0) * C;
  auto epi = [&](float4 w, int64_t g) __attribute__((always_inline)) {
    if (e.add_row) {
      const float4 ar = *reinterpret_cast<const float4*>(e.add_row + g);
      w.x += ar.x; w.y += ar.y; w.z += ar.z; w.w += ar.w;
    }
    if (e.acc32) {
      const float4 ac = *reinterpret_cast<const float4*>(e.acc32 + g);
      w.x = ac.x + w.x; w.y = ac.y + w.y; w.z = ac.z + w.z; w.w = ac.w + w.w;
      if (e.acc_div != 1.0f) {
        w.x = w.x / e.acc_div; w.y = w.y / e.acc_div; w.z = w.z / e.acc_div; w.w = w.w / e.acc_div;
      }
    }
    if (e.out32) *reinterpret_cast<float4*>(e.out32 + g) = w;  // may alias add_row / acc32: same element, same thread
    if (e.out16) {
      union { uint2 u2; f16 h[4]; } pk;
      pk.h[0] = f16_sat(w.x); pk.h[1] = f16_sat(w.y); pk.h[2] = f16_sat(w.z); pk.h[3] = f16_sat(w.w);
      *reinterpret_cast<uint2*>(e.out16 + g) = pk.u2;
    }
  };
  if (!(p.dbg & 8)) {
    float* stg = reinterpret_cast<float*>(amp_sm);
    constexpr int HB = CF::BT / CF::NPART, C4 = C / 4;
    // A half's epilogue operands (add_row / acc32 rows) are loaded for all of the thread's chunks at once, through
    // buffer descriptors over this workgroup's block (a missing operand or a row past nvalid reads 0: no per-lane or
    // per-operand branch), and waited for once. Loaded chunk by chunk inside the loop, each chunk's load waited for every
    // store before it (in-order vmcnt) and the branches made the compiler's wait a vmcnt(0) before every use: two load
    // round trips and a store drain per chunk (assembly, r06).
    constexpr int IT = (HB * C4 + CF::NT - 1) / CF::NT;  // chunks per thread and half
    const int blk_bytes = nvalid * C * 4;
    const __amdgpu_buffer_rsrc_t r_ar =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(e.add_row ? e.add_row + base : e.bias), (short)0,
                                          e.add_row ? blk_bytes : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t r_ac =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(e.acc32 ? e.acc32 + base : e.bias), (short)0,
                                          e.acc32 ? blk_bytes : 0, 0x00020000);
    auto epi2 = [&](float4 w, const float4& ar, const float4& ac, int64_t g) __attribute__((always_inline)) {
      if (e.add_row) {
        w.x += ar.x; w.y += ar.y; w.z += ar.z; w.w += ar.w;
      }
      if (e.acc32) {
        w.x = ac.x + w.x; w.y = ac.y + w.y; w.z = ac.z + w.z; w.w = ac.w + w.w;
        if (e.acc_div != 1.0f) {
          w.x = w.x / e.acc_div; w.y = w.y / e.acc_div; w.z = w.z / e.acc_div; w.w = w.w / e.acc_div;
        }
      }
      if (e.out32) *reinterpret_cast<float4*>(e.out32 + g) = w;  // may alias add_row / acc32: same element, same thread
      if (e.out16) {
        union { uint2 u2; f16 h[4]; } pk;
        pk.h[0] = f16_sat(w.x); pk.h[1] = f16_sat(w.y); pk.h[2] = f16_sat(w.z); pk.h[3] = f16_sat(w.w);
        *reinterpret_cast<uint2*>(e.out16 + g) = pk.u2;
      }
    };
    const bool has_ops = e.add_row || e.acc32;  // (the c1 convs have none: no loads at all)
#pragma unroll
    for (int h = 0; h < CF::NPART; ++h) {
      if (h * HB >= nvalid) break;  // (block-uniform)
      float4 ar[IT], ac[IT];
#pragma unroll
      for (int it = 0; it < IT; ++it) ar[it] = ac[it] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (has_ops) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
          const uint32_t vo = (uint32_t)((h * HB * C4 + tid + it * CF::NT) * 16);  // chunk h * HB * C4 + idx
          ar[it] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r_ar, vo, 0, 0));
          ac[it] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r_ac, vo, 0, 0));
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
          asm volatile("" : "+v"(ar[it].x), "+v"(ar[it].y), "+v"(ar[it].z), "+v"(ar[it].w));
          asm volatile("" : "+v"(ac[it].x), "+v"(ac[it].y), "+v"(ac[it].z), "+v"(ac[it].w));
        }
      }
      __syncthreads();  // h = 0: the k-loop's image reads are done; h > 0: the previous part has been consumed
#pragma unroll
      for (int j = 0; j < FNW; ++j) {
        const int c0 = (wn * FNW + j) * 16 + fk * 4;
        if (c0 >= C) continue;
        const float4 bi = *reinterpret_cast<const float4*>(p.bias + c0);
#pragma unroll
        for (int i = 0; i < MW; ++i) {
          const int rt = (wm * MW + i) * 16;  // the fragment's first tile row (wave-uniform)
          if (rt / HB != h) continue;
          const int r = rt - h * HB + fr;
          *reinterpret_cast<float4*>(stg + r * CF::LDC + c0) =
              make_float4(acc[i][j][0] + bi.x, acc[i][j][1] + bi.y, acc[i][j][2] + bi.z, acc[i][j][3] + bi.w);
        }
      }
      __syncthreads();
      const int nv = min(HB, nvalid - h * HB);
      if (has_ops) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
          const int idx = tid + it * CF::NT;
          if (idx >= nv * C4) break;
          const int r = idx / C4, c4 = idx - r * C4;
          epi2(*reinterpret_cast<const float4*>(stg + r * CF::LDC + 4 * c4), ar[it], ac[it],
               base + (int64_t)(h * HB + r) * C + 4 * c4);
        }
      } else {  // (c1: stores only; the rolled loop measured 3-5 % faster than the unrolled one here, r06e)
        for (int idx = tid; idx < nv * C4; idx += CF::NT) {
          const int r = idx / C4, c4 = idx - r * C4;
          epi(*reinterpret_cast<const float4*>(stg + r * CF::LDC + 4 * c4), base + (int64_t)(h * HB + r) * C + 4 * c4);
        }
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < FNW; ++j) {
      const int c0 = (wn * FNW + j) * 16 + fk * 4;
      if (c0 >= C) continue;
      const float4 bi = *reinterpret_cast<const float4*>(p.bias + c0);
#pragma unroll
      for (int i = 0; i < MW; ++i) {
        const int row = (wm * MW + i) * 16 + fr;
        if (row >= nvalid) continue;
        epi(make_float4(acc[i][j][0] + bi.x, acc[i][j][1] + bi.y, acc[i][j][2] + bi.z, acc[i][j][3] + bi.w),
            base + (int64_t)row * C + c0);
      }
    }
  }
}

template <int C, bool X16, bool NOACT = false>
static int launch_amp(const AmpConvArgs& p, const EpiArgs& e, hipStream_t s) {
  using CF = AmpCfg<C, NOACT>;
  if (int st = ensure_dyn_lds((const void*)amp_conv_kernel<C, X16, NOACT>, CF::LDS)) return st;
  const int64_t grid = (int64_t)p.B * cdiv(p.L, CF::BT);
  SVC_REQUIRE(grid > 0 && grid < (1ll << 31), "amp_conv: bad grid");
  const double elems = (double)p.B * p.L * C;
  // algorithmic bytes: x in (f32 or f16), output out (f32 and/or f16), epilogue operands in (f32)
  const double bytes =
      elems * ((X16 ? 2.0 : 4.0) + (e.out32 ? 4 : 0) + (e.out16 ? 2 : 0) + (e.add_row ? 4 : 0) + (e.acc32 ? 4 : 0));
  const char* tag = NOACT ? (C == 48 ? "amp_conv<48,conv>" : (C == 96 ? "amp_conv<96,conv>" : "amp_conv<192,conv>"))
                          : (C == 24 ? "amp_conv<24>" : (C == 48 ? "amp_conv<48>" : (C == 96 ? "amp_conv<96>" : "amp_conv<192>")));
  const int tok = prof_begin(tag, 2.0 * elems * C * p.k, bytes, s);
  // the activation image needs BT + 2P rows, not BT + 2 MAXP: sized per launch, C = 48 fits 5 workgroups per CU
  // (instead of 4) for every conv with P <= 15
  const int P = (p.k - 1) / 2 * (p.d < 0 ? -p.d : p.d);
  const int rows = CF::BT + 2 * P, run = amp_run_len(C, rows, CF::NT);
  const int img_rows = NOACT ? rows : (rows + run - 1) / run * run;
  const int lds = std::max(img_rows * CF::LDA * 2, CF::STG_BYTES);
  static const int dbg = getenv("SVC_AMP_DBG") ? atoi(getenv("SVC_AMP_DBG")) : 0;
  AmpConvArgs pa = p;
  pa.dbg = dbg;
  hipLaunchKernelGGL((amp_conv_kernel<C, X16, NOACT>), dim3((unsigned)grid), dim3(CF::NT), lds, s, pa, e);
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

bool amp_conv_supported(int C, int k, int d) {
  return (C == 24 || C == 48 || C == 96 || C == 192) && k >= 1 && k % 2 == 1 && d != 0 &&
         (k - 1) / 2 * (d < 0 ? -d : d) <= AmpCfg<24>::MAXP;
}

// act + conv + epilogue; e uses out32 / out16 / add_row / acc32 with leading dimension C (contiguous rows)
int amp_conv(const AmpConvArgs& p, int C, const EpiArgs& e, hipStream_t s) {
  SVC_REQUIRE(amp_conv_supported(C, p.k, p.d) && (!p.noact || ((C == 48 || C == 96 || C == 192) && p.x16)) && (p.noact || p.d > 0),
              "amp_conv: C=%d k=%d d=%d noact=%d unsupported", C, p.k, p.d, (int)p.noact);
  SVC_REQUIRE(p.L >= 1 && p.Kpad >= p.k * C && p.Kpad % 32 == 0, "amp_conv: L=%d Kpad=%d", p.L, p.Kpad);
  SVC_REQUIRE((!e.out32 || e.ld32 == C) && (!e.out16 || e.ld16 == C) && (!e.add_row || e.ld_add_row == C) &&
                  (!e.acc32 || e.ld_acc == C) && !e.add16 && e.act == ACT_NONE && e.kind == EPI_GENERIC,
              "amp_conv: epilogue must be contiguous rows of C channels (bias / add_row / acc32 / out32 / out16)");
  const void* xin = p.x16 ? (const void*)p.x16 : (const void*)p.x;
  SVC_REQUIRE(((uintptr_t)xin & 15) == 0 && ((uintptr_t)p.W & 15) == 0, "amp_conv: alignment");
  // the activation reads x through a buffer descriptor (32-bit record count and offsets): utterances per launch such
  // that one launch's x span stays below 2^31 bytes; the rows of every tensor are contiguous [B*L][C]
  const int64_t per_b = (int64_t)p.L * C * (p.x16 ? 2 : 4);
  // one utterance must fit the 32-bit offsets itself (the split is per utterance; svc_bigvgan bounds T accordingly)
  SVC_REQUIRE(per_b < ((int64_t)1 << 31), "amp_conv: one utterance spans %lld bytes (L=%d C=%d), >= 2 GiB",
              (long long)per_b, p.L, C);
  const int bchunk = (int)std::max<int64_t>(1, std::min<int64_t>(p.B, ((int64_t)1 << 31) / per_b - 1));
  for (int b0 = 0; b0 < p.B; b0 += bchunk) {
    const int64_t off = (int64_t)b0 * p.L * C;
    AmpConvArgs q = p;
    EpiArgs f = e;
    q.B = std::min(bchunk, p.B - b0);
    if (q.x) q.x += off;
    if (q.x16) q.x16 += off;
    if (q.tv) q.tv += b0;
    if (f.out32) f.out32 += off;
    if (f.out16) f.out16 += off;
    if (f.acc32) f.acc32 += off;
    if (f.add_row) f.add_row += off;
    int st;
    if (C == 24)
      st = q.x16 ? launch_amp<24, true>(q, f, s) : launch_amp<24, false>(q, f, s);
    else if (C == 48 && q.noact)
      st = launch_amp<48, true, true>(q, f, s);
    else if (C == 48)
      st = q.x16 ? launch_amp<48, true>(q, f, s) : launch_amp<48, false>(q, f, s);
    else if (C == 96 && q.noact)
      st = launch_amp<96, true, true>(q, f, s);
    else if (C == 96)
      st = q.x16 ? launch_amp<96, true>(q, f, s) : launch_amp<96, false>(q, f, s);
    else if (q.noact)
      st = launch_amp<192, true, true>(q, f, s);
    else
      st = q.x16 ? launch_amp<192, true>(q, f, s) : launch_amp<192, false>(q, f, s);
    if (st) return st;
  }
  return SVC_OK;
}

}  // namespace svc
