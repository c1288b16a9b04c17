// BigVGAN Activation1d (anti-aliased SnakeBeta) on gfx950, HBM-bound: read x (f32, or f16 for an AMPBlock1
// intermediate) once, write y (f16) once. modules/bigvgan.py:234-307 + SnakeBeta :146-159, per channel sequence x[0..L-1]:
//   u[2q]   = 2 * sum_{a=0..5} x[clamp(q-3+a)] * f[11-2a]      (UpSample1d: replicate pad 5, crop 15)
//   u[2q+1] = 2 * sum_{a=0..5} x[clamp(q-2+a)] * f[10-2a]
//   s[j]    = u + 1/(exp(beta)+1e-9) * sin(u*exp(alpha))^2
//   y[t]    = sum_{k=0..11} f[k] * s[clamp(2t+k-5, 0, 2L-1)]   (LowPassFilter1d: replicate pad (5,6), stride 2)
// sin uses v_sin_f32 on the fractional revolution of u*alpha/2pi: its error (~|u|*6e-8) is the size of the f32
// rounding of the argument u*alpha that the reference itself incurs.
#include "common.h"
#include "snake.h"

namespace svc {

// ---------------------------------------------------------------------------------------------------
// Register-streaming form. A thread owns a channel pair of one utterance and walks a run of R outputs in
// blocks of P. It keeps sliding windows in registers: xw = x[t-5 .. t+P+4] (10 carried + P loaded per block)
// and sw = s[2t-5 .. 2t+2P+4] (10 carried + 2P computed per block); the next block's P rows are loaded while
// this block computes. No LDS, no barriers; loads are coalesced across lanes (adjacent lanes = adjacent
// channel pairs). The arithmetic is VALU-bound, not HBM-bound, at ~45 VALU per output element in the
// per-channel form (r04final: 240-270 us per 184 M-element launch = 3.1-4.1 TB/s), so it runs on channel
// pairs with packed f32 ops (v_pk_fma_f32): the up-sampling taps carry the factor 2 (exact: powers of two
// scale without rounding), the sine's argument is taken in revolutions with alpha / 2pi folded into the
// channel constant, and runs clear of both utterance ends (all but the first and last per utterance) take
// a form without the clamps, the replicate padding and the per-output tail test.
// One run. Addresses are 32-bit buffer offsets: a lane's row-0 offset (xo / yo) plus the row's offset, which for the
// k-th row of a block is the wave-uniform k * row stride (soffset), so a block's loads and stores hold no per-row
// address registers (64-bit per-row addresses had been a quarter of the register budget).
template <int P, int R, bool EDGE, typename TX>
__device__ __forceinline__ void act_run(__amdgpu_buffer_rsrc_t rx, __amdgpu_buffer_rsrc_t ry, uint32_t xo, uint32_t yo,
                                        uint32_t xs, uint32_t ys, int t0, int Lb, const float (&f)[12],
                                        const float (&f2)[12], const SnakeCoef2& kc) {
  auto xl = [&](int t) __attribute__((always_inline)) {
    t = t < 0 ? 0 : (t >= Lb ? Lb - 1 : t);
    return act_load<TX>(rx, xo + (uint32_t)t * xs, 0);
  };
  // prefetched rows stay in their loaded form (f16 input: one raw word per channel pair), converted when used
  using XR = act_raw_t<TX>;
  auto xlr = [&](int t) __attribute__((always_inline)) {
    t = t < 0 ? 0 : (t >= Lb ? Lb - 1 : t);
    return act_load_raw<TX>(rx, xo + (uint32_t)t * xs, 0);
  };
  auto s_win = [&](const f32x2* xw, int i) __attribute__((always_inline)) { return snake_up(xw, i, f2, kc); };
  const int t_end = EDGE ? min(t0 + R, Lb) : t0 + R;
  // the next block's rows are loaded while this block computes (f32: 106 registers, launches 3 % faster, r04u;
  // f16 as converted pairs was 2-3 % slower, r04u; as raw words, 98 registers = 4 waves per SIMD instead of 5, its
  // launches are 5-8 % faster, profiles/r06_ab/r06g_act_f16_prefetch.txt)
  constexpr bool PF = true;
  f32x2 xw[P + 10], sw[2 * P + 10];
  XR xn[PF ? P : 1];
#pragma unroll
  for (int k = 0; k < 10; ++k) xw[k] = xl(t0 - 5 + k);
  if constexpr (PF) {
#pragma unroll
    for (int k = 0; k < P; ++k) xn[k] = xlr(t0 + 5 + k);
  }
#pragma unroll
  for (int i = 0; i < 10; ++i) sw[i] = s_win(xw, i);
  if (EDGE) {
    // replicate padding of the upsampled signal: s[j] = s[2L-1] past the end, s[0] before the start
#pragma unroll
    for (int i = 1; i < 10; ++i)
      if (2 * t0 - 5 + i > 2 * Lb - 1) sw[i] = sw[i - 1];
#pragma unroll
    for (int i = 8; i >= 0; --i)
      if (2 * t0 - 5 + i < 0) sw[i] = sw[i + 1];
  }
  for (int t = t0; t < t_end; t += P) {
    const uint32_t xrow = xo + (uint32_t)(t + 5) * xs, yrow = yo + (uint32_t)t * ys;
    if constexpr (PF) {
#pragma unroll
      for (int k = 0; k < P; ++k) xw[10 + k] = act_cvt<TX>(xn[k]);
      if (t + P < t_end) {
#pragma unroll
        for (int k = 0; k < P; ++k) xn[k] = EDGE ? xlr(t + P + 5 + k) : act_load_raw<TX>(rx, xrow, (P + k) * xs);
      }
    } else {
#pragma unroll
      for (int k = 0; k < P; ++k) xw[10 + k] = EDGE ? xl(t + 5 + k) : act_load<TX>(rx, xrow, k * xs);
    }
    // output p needs s up to index 2p+11, i.e. x up to window row 10+p
#pragma unroll
    for (int p = 0; p < P; ++p) {
      sw[10 + 2 * p] = s_win(xw, 10 + 2 * p);
      sw[11 + 2 * p] = s_win(xw, 11 + 2 * p);
      if (EDGE && 2 * t + 2 * p + 6 > 2 * Lb - 1) {
        if (2 * t + 2 * p + 5 > 2 * Lb - 1) sw[10 + 2 * p] = sw[9 + 2 * p];
        sw[11 + 2 * p] = sw[10 + 2 * p];
      }
      if (!EDGE || t + p < t_end) {
        __builtin_amdgcn_raw_buffer_store_b32(f16x2_sat(snake_down(sw + 2 * p, f)), ry, yrow, p * ys, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) xw[k] = xw[P + k];
#pragma unroll
    for (int i = 0; i < 10; ++i) sw[i] = sw[2 * P + i];
  }
}

// x / y: B utterances of L rows (x row stride C, y row stride ldy); 32-bit buffer offsets (the host splits B so that
// one launch addresses < 2 GiB of either tensor)
template <int P, int R, typename TX = float>
__global__ __launch_bounds__(256) void activation1d_rs_kernel(const TX* __restrict__ x, f16* __restrict__ y,
                                                              int B, int L, int C, int ldy,
                                                              const float* __restrict__ alpha_log,
                                                              const float* __restrict__ beta_log,
                                                              const float* __restrict__ filt,
                                                              const int* __restrict__ tv, int tv_mul) {
  static_assert(R % P == 0, "run = whole blocks");
  const int ngroups = C / 2;
  const int nruns = (L + R - 1) / R;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (int64_t)B * nruns * ngroups) return;
  const int g = (int)(gid % ngroups);
  const int64_t rest = gid / ngroups;
  const int run = (int)(rest % nruns), b = (int)(rest / nruns);
  const int c = g * 2;
  // ragged batches: this utterance's sequence ends at Lb (replicate padding there); rows keep the stride L
  const int Lb = tv ? min(L, tv[b] * tv_mul) : L;
  const int t0 = run * R;
  if (t0 >= Lb) return;
  float f[12], f2[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    f[k] = filt[k];
    f2[k] = 2.0f * f[k];
  }
  const SnakeCoef2 kc = snake_coef2(alpha_log, beta_log, c);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<TX*>(x), (short)0,
                                                                      (int)((int64_t)B * L * C * sizeof(TX)), 0x00020000);
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(y, (short)0, (int)((int64_t)B * L * ldy * 2), 0x00020000);
  const uint32_t xo = (uint32_t)(((int64_t)b * L * C + c) * sizeof(TX)), yo = (uint32_t)(((int64_t)b * L * ldy + c) * 2);
  const uint32_t xs = (uint32_t)(C * sizeof(TX)), ys = (uint32_t)(ldy * 2);
  if (t0 >= 5 && t0 + R + 5 <= Lb)
    act_run<P, R, false, TX>(rx, ry, xo, yo, xs, ys, t0, Lb, f, f2, kc);
  else
    act_run<P, R, true, TX>(rx, ry, xo, yo, xs, ys, t0, Lb, f, f2, kc);
}

template <int P, int R, typename TX>
static int launch_rs(const TX* x, f16* y, int B, int L, int C, int ldy, const float* al, const float* bl,
                      const float* filt, const int* tv, int tv_mul, hipStream_t s) {
  // utterances per launch: both tensors' spans below 2^31 bytes (buffer offsets and record counts are 32-bit)
  const int64_t per_b = (int64_t)L * std::max<int64_t>((int64_t)C * sizeof(TX), (int64_t)ldy * 2);
  // one utterance must fit the 32-bit offsets itself (the split is per utterance; svc_bigvgan bounds T accordingly)
  SVC_REQUIRE(per_b < ((int64_t)1 << 31), "activation1d: one utterance spans %lld bytes (L=%d C=%d), >= 2 GiB",
                (long long)per_b, L, C);
  const int bchunk = (int)std::max<int64_t>(1, std::min<int64_t>(B, ((int64_t)1 << 31) / per_b - 1));
  for (int b0 = 0; b0 < B; b0 += bchunk) {
    const int nb = std::min(bchunk, B - b0);
    const int64_t n = (int64_t)nb * cdiv(L, R) * (C / 2);
    hipLaunchKernelGGL((activation1d_rs_kernel<P, R, TX>), dim3((unsigned)cdiv64(n, 256)), dim3(256), 0, s,
                       x + (int64_t)b0 * L * C, y + (int64_t)b0 * L * ldy, nb, L, C, ldy, al, bl, filt,
                       tv ? tv + b0 : nullptr, tv_mul);
  }
  return SVC_OK;
}

// tv / tv_mul (optional): ragged batches, utterance b's sequence is min(L, tv[b] * tv_mul) rows long.
// x is f32 (the generator's residual stream) or f16 (x16: an AMPBlock1 convs1 output, stored f16)
int activation1d(const float* x, f16* y, int B, int L, int C, int ldy, const float* alpha_log, const float* beta_log,
                 const float* filt, hipStream_t s, const int* tv, int tv_mul, const f16* x16) {
  SVC_REQUIRE(L >= 1 && C >= 4 && C % 4 == 0 && ldy % 4 == 0, "activation1d: L=%d C=%d ldy=%d", L, C, ldy);
  SVC_REQUIRE(((uintptr_t)(x16 ? (const void*)x16 : (const void*)x) & 15) == 0 && ((uintptr_t)y & 7) == 0,
              "activation1d: alignment");
  const int tok = prof_begin("activation1d", 0.0, (double)B * L * C * ((x16 ? 2 : 4) + 2), s);
  // a channel pair per thread, 8-output blocks, 128-output runs (the register-streaming shape that measured fastest
  // in rounds 1-2, against other block / run shapes and an LDS-tiled form)
  // (f16 input in 4-row blocks, 82 registers = 6 waves per SIMD: 10 % slower per launch, r04af)
  const int st = x16 ? launch_rs<8, 128>(x16, y, B, L, C, ldy, alpha_log, beta_log, filt, tv, tv_mul, s)
                     : launch_rs<8, 128>(x, y, B, L, C, ldy, alpha_log, beta_log, filt, tv, tv_mul, s);
  prof_end(tok, s);
  if (st) return st;
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
