// BigVGAN Activation1d (anti-aliased SnakeBeta) on gfx950, HBM-bound: read x (f32, or f16 for an AMPBlock1
// intermediate) once, write y (f16) once. modules/bigvgan.py:234-307 + SnakeBeta :146-159, per channel sequence x[0..L-1]:
//   u[2q]   = 2 * sum_{a=0..5} x[clamp(q-3+a)] * f[11-2a]      (UpSample1d: replicate pad 5, crop 15)
//   u[2q+1] = 2 * sum_{a=0..5} x[clamp(q-2+a)] * f[10-2a]
//   s[j]    = u + 1/(exp(beta)+1e-9) * sin(u*exp(alpha))^2
//   y[t]    = sum_{k=0..11} f[k] * s[clamp(2t+k-5, 0, 2L-1)]   (LowPassFilter1d: replicate pad (5,6), stride 2)
// sin uses v_sin_f32 after an explicit reduction to [-0.5, 0.5] revolutions: its error (~|u|*6e-8) is the
// size of the f32 rounding of the argument u*alpha that the reference itself incurs.
#include "common.h"
#include "snake.h"

namespace svc {

// ---------------------------------------------------------------------------------------------------
// Register-streaming form. A thread owns VEC adjacent channels of one utterance and walks a run
// of R outputs in blocks of P. It keeps sliding windows in registers: xw = x[t-5 .. t+P+4] (10 carried +
// P loaded per block) and sw = s[2t-5 .. 2t+2P+4] (10 carried + 2P computed per block). No LDS, no
// barriers; loads are coalesced across lanes (adjacent lanes = adjacent channel groups). Window values
// are computed from replicate-clamped x loads, which is exact for every upsampled index inside [0, 2L-1];
// indices outside take their neighbour's value (the low-pass filter's replicate padding).
template <int VEC, int P, int R, typename TX = float>
__global__ __launch_bounds__(256) void activation1d_rs_kernel(const TX* __restrict__ x, f16* __restrict__ y,
                                                              int B, int L, int C, int ldy,
                                                              const float* __restrict__ alpha_log,
                                                              const float* __restrict__ beta_log,
                                                              const float* __restrict__ filt,
                                                              const int* __restrict__ tv, int tv_mul) {
  static_assert(R % P == 0, "run = whole blocks");
  using V = ActVec<VEC>;
  const int ngroups = C / VEC;
  const int nruns = (L + R - 1) / R;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (int64_t)B * nruns * ngroups) return;
  const int g = (int)(gid % ngroups);
  const int64_t rest = gid / ngroups;
  const int run = (int)(rest % nruns), b = (int)(rest / nruns);
  const int c = g * VEC;
  const TX* xb = x + (int64_t)b * L * C + c;
  f16* yb = y + (int64_t)b * L * ldy + c;
  // ragged batches: this utterance's sequence ends at Lb (replicate padding there); rows keep the stride L
  const int Lb = tv ? min(L, tv[b] * tv_mul) : L;
  if (run * R >= Lb) return;
  float f[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) f[k] = filt[k];
  float as[VEC], ib[VEC];
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    as[v] = expf(alpha_log[c + v]);
    ib[v] = 1.0f / (expf(beta_log[c + v]) + 0.000000001f);
  }
  auto xload = [&](int t, float* o) {
    t = t < 0 ? 0 : (t >= Lb ? Lb - 1 : t);
    V::load(xb + (int64_t)t * C, o);
  };
  auto snake = [&](float* u) {
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const float sn = sin_rev(u[v] * as[v]);
      u[v] = u[v] + ib[v] * (sn * sn);
    }
  };
  // s[2tb-5+i] from the window xw[k] = x[tb-5+k] (valid when that index lies inside [0, 2L-1])
  auto s_win = [&](const float (*xw)[VEC], int i, float* o) {
    const int odd = (i + 1) & 1;           // parity of j = 2tb-5+i
    const int base = ((i - 5) >> 1) + 2 + odd;
#pragma unroll
    for (int v = 0; v < VEC; ++v) o[v] = 0.f;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const float w = f[11 - odd - 2 * a];
#pragma unroll
      for (int v = 0; v < VEC; ++v) o[v] += xw[base + a][v] * w;
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) o[v] *= 2.0f;
    snake(o);
  };

  const int t0 = run * R;
  const int t_end = t0 + R < Lb ? t0 + R : Lb;
  float xw[P + 10][VEC], sw[2 * P + 10][VEC];
#pragma unroll
  for (int k = 0; k < 10; ++k) xload(t0 - 5 + k, xw[k]);
#pragma unroll
  for (int i = 0; i < 10; ++i) s_win(xw, i, sw[i]);
  // replicate padding of the upsampled signal: s[j] = s[2L-1] past the end, s[0] before the start
#pragma unroll
  for (int i = 1; i < 10; ++i)
    if (2 * t0 - 5 + i > 2 * Lb - 1)
#pragma unroll
      for (int v = 0; v < VEC; ++v) sw[i][v] = sw[i - 1][v];
#pragma unroll
  for (int i = 8; i >= 0; --i)
    if (2 * t0 - 5 + i < 0)
#pragma unroll
      for (int v = 0; v < VEC; ++v) sw[i][v] = sw[i + 1][v];
  for (int t = t0; t < t_end; t += P) {
#pragma unroll
    for (int k = 0; k < P; ++k) xload(t + 5 + k, xw[10 + k]);
#pragma unroll
    for (int i = 10; i < 2 * P + 10; ++i) s_win(xw, i, sw[i]);
    if (2 * t + 2 * P + 4 > 2 * Lb - 1) {
#pragma unroll
      for (int i = 10; i < 2 * P + 10; ++i)
        if (2 * t - 5 + i > 2 * Lb - 1)
#pragma unroll
          for (int v = 0; v < VEC; ++v) sw[i][v] = sw[i - 1][v];
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      if (t + p < t_end) {
        float acc[VEC];
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
#pragma unroll
        for (int k = 0; k < 12; ++k)
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[v] += f[k] * sw[2 * p + k][v];
        V::store(yb + (int64_t)(t + p) * ldy, acc);
      }
    }
#pragma unroll
    for (int k = 0; k < 10; ++k)
#pragma unroll
      for (int v = 0; v < VEC; ++v) xw[k][v] = xw[P + k][v];
#pragma unroll
    for (int i = 0; i < 10; ++i)
#pragma unroll
      for (int v = 0; v < VEC; ++v) sw[i][v] = sw[2 * P + i][v];
  }
}

template <int VEC, int P, int R, typename TX>
static void launch_rs(const TX* x, f16* y, int B, int L, int C, int ldy, const float* al, const float* bl,
                      const float* filt, const int* tv, int tv_mul, hipStream_t s) {
  const int64_t n = (int64_t)B * cdiv(L, R) * (C / VEC);
  hipLaunchKernelGGL((activation1d_rs_kernel<VEC, P, R, TX>), dim3((unsigned)cdiv64(n, 256)), dim3(256), 0, s, x, y, B,
                     L, C, ldy, al, bl, filt, tv, tv_mul);
}

// tv / tv_mul (optional): ragged batches, utterance b's sequence is min(L, tv[b] * tv_mul) rows long.
// x is f32 (the generator's residual stream) or f16 (x16: an AMPBlock1 convs1 output, stored f16)
int activation1d(const float* x, f16* y, int B, int L, int C, int ldy, const float* alpha_log, const float* beta_log,
                 const float* filt, hipStream_t s, const int* tv, int tv_mul, const f16* x16) {
  SVC_REQUIRE(L >= 1 && C >= 4 && C % 4 == 0 && ldy % 4 == 0, "activation1d: L=%d C=%d ldy=%d", L, C, ldy);
  SVC_REQUIRE(((uintptr_t)(x16 ? (const void*)x16 : (const void*)x) & 15) == 0 && ((uintptr_t)y & 7) == 0,
              "activation1d: alignment");
  const int tok = prof_begin("activation1d", 0.0, (double)B * L * C * ((x16 ? 2 : 4) + 2), s);
  // 2 channels per thread, 8-output blocks, 128-output runs: the fastest of the register-streaming shapes and of an
  // LDS-tiled form measured in rounds 1-2 (4.0-4.1 TB/s; the others were removed in round 3)
  if (x16)
    launch_rs<2, 8, 128>(x16, y, B, L, C, ldy, alpha_log, beta_log, filt, tv, tv_mul, s);
  else
    launch_rs<2, 8, 128>(x, y, B, L, C, ldy, alpha_log, beta_log, filt, tv, tv_mul, s);
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
