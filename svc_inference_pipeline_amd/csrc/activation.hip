// BigVGAN Activation1d (anti-aliased SnakeBeta) on gfx950, HBM-bound: read x (f32) once, write y (f16)
// once. modules/bigvgan.py:234-307 + SnakeBeta :146-159, per channel sequence x[0..L-1]:
//   u[2q]   = 2 * sum_{a=0..5} x[clamp(q-3+a)] * f[11-2a]      (UpSample1d: replicate pad 5, crop 15)
//   u[2q+1] = 2 * sum_{a=0..5} x[clamp(q-2+a)] * f[10-2a]
//   s[j]    = u + 1/(exp(beta)+1e-9) * sin(u*exp(alpha))^2
//   y[t]    = sum_{k=0..11} f[k] * s[clamp(2t+k-5, 0, 2L-1)]   (LowPassFilter1d: replicate pad (5,6), stride 2)
// A workgroup owns 64 outputs x CG groups of 4 channels of one utterance; each thread keeps one channel
// group (float4 loads, 8-byte fp16 stores) and walks time. x rows [t0-6, t0+70) and the 140 needed s
// values live in LDS, so every x element is read once and every s once per 64 outputs.
// sin uses v_sin_f32 after an explicit reduction to [-0.5, 0.5] revolutions: its error (~|u|*6e-8) is the
// size of the f32 rounding of the argument u*alpha that the reference itself incurs.
#include "common.h"
#include "snake.h"

namespace svc {

constexpr int A2_TT = 64;

template <int CG>
__global__ __launch_bounds__(256) void activation1d_v2_kernel(const float* __restrict__ x, f16* __restrict__ y, int L,
                                                              int C, int ldy, const float* __restrict__ alpha_log,
                                                              const float* __restrict__ beta_log,
                                                              const float* __restrict__ filt, const int* __restrict__ tv,
                                                              int tv_mul) {
  constexpr int NL = 256 / CG;  // time lanes
  __shared__ float4 xs[(A2_TT + 12) * CG];
  __shared__ float4 ss[(2 * A2_TT + 12) * CG];
  const int tid = threadIdx.x;
  if (tid >= NL * CG) return;  // (no barrier is skipped: idle threads leave before the first one)
  const int g = tid % CG, tl = tid / CG;
  const int t0 = blockIdx.x * A2_TT;
  const int c = blockIdx.y * (4 * CG) + 4 * g;
  const int b = blockIdx.z;
  const bool cok = c < C;
  const float* xb = x + (int64_t)b * L * C;
  // ragged batches: the sequence ends at Lb (replicate padding there); rows keep the batch stride L
  const int Lb = tv ? min(L, tv[b] * tv_mul) : L;
  if (t0 >= Lb) return;
  float f[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) f[k] = filt[k];
  float4 as = make_float4(1.f, 1.f, 1.f, 1.f), ib = make_float4(0.f, 0.f, 0.f, 0.f);
  if (cok) {
    as = make_float4(expf(alpha_log[c]), expf(alpha_log[c + 1]), expf(alpha_log[c + 2]), expf(alpha_log[c + 3]));
    ib = make_float4(1.0f / (expf(beta_log[c]) + 0.000000001f), 1.0f / (expf(beta_log[c + 1]) + 0.000000001f),
                     1.0f / (expf(beta_log[c + 2]) + 0.000000001f), 1.0f / (expf(beta_log[c + 3]) + 0.000000001f));
  }
  for (int r = tl; r < A2_TT + 12; r += NL) {
    int t = t0 - 6 + r;
    t = t < 0 ? 0 : (t >= Lb ? Lb - 1 : t);
    xs[r * CG + g] = cok ? *reinterpret_cast<const float4*>(xb + (int64_t)t * C + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  for (int jj = tl; jj < 2 * A2_TT + 12; jj += NL) {
    int j = 2 * t0 - 5 + jj;
    j = j < 0 ? 0 : (j >= 2 * Lb ? 2 * Lb - 1 : j);
    const int qq = j >> 1;
    const int odd = j & 1;
    float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      int xt = qq - 3 + odd + a;
      xt = xt < 0 ? 0 : (xt >= Lb ? Lb - 1 : xt);
      const float w = f[11 - odd - 2 * a];
      const float4 xv = xs[(xt - (t0 - 6)) * CG + g];
      u.x += xv.x * w;
      u.y += xv.y * w;
      u.z += xv.z * w;
      u.w += xv.w * w;
    }
    u.x *= 2.0f;
    u.y *= 2.0f;
    u.z *= 2.0f;
    u.w *= 2.0f;
    float sx = sin_rev(u.x * as.x), sy = sin_rev(u.y * as.y), sz = sin_rev(u.z * as.z), sw = sin_rev(u.w * as.w);
    ss[jj * CG + g] = make_float4(u.x + ib.x * (sx * sx), u.y + ib.y * (sy * sy), u.z + ib.z * (sz * sz),
                                  u.w + ib.w * (sw * sw));
  }
  __syncthreads();
  if (!cok) return;
  for (int r = tl; r < A2_TT; r += NL) {
    const int t = t0 + r;
    if (t >= Lb) break;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const float4 sv = ss[(2 * r + k) * CG + g];
      acc.x += f[k] * sv.x;
      acc.y += f[k] * sv.y;
      acc.z += f[k] * sv.z;
      acc.w += f[k] * sv.w;
    }
    union { uint2 u; f16 h[4]; } pk;
    pk.h[0] = f16_sat(acc.x);
    pk.h[1] = f16_sat(acc.y);
    pk.h[2] = f16_sat(acc.z);
    pk.h[3] = f16_sat(acc.w);
    *reinterpret_cast<uint2*>(y + ((int64_t)b * L + t) * ldy + c) = pk.u;
  }
}

// ---------------------------------------------------------------------------------------------------
// Register-streaming form (default). A thread owns VEC adjacent channels of one utterance and walks a run
// of R outputs in blocks of P. It keeps sliding windows in registers: xw = x[t-5 .. t+P+4] (10 carried +
// P loaded per block) and sw = s[2t-5 .. 2t+2P+4] (10 carried + 2P computed per block). No LDS, no
// barriers; loads are coalesced across lanes (adjacent lanes = adjacent channel groups). Window values
// are computed from replicate-clamped x loads, which is exact for every upsampled index inside [0, 2L-1];
// indices outside take their neighbour's value (the low-pass filter's replicate padding).
template <int VEC, int P, int R>
__global__ __launch_bounds__(256) void activation1d_rs_kernel(const float* __restrict__ x, f16* __restrict__ y,
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
  const float* xb = x + (int64_t)b * L * C + c;
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

template <int VEC, int P, int R>
static void launch_rs(const float* x, f16* y, int B, int L, int C, int ldy, const float* al, const float* bl,
                      const float* filt, const int* tv, int tv_mul, hipStream_t s) {
  const int64_t n = (int64_t)B * cdiv(L, R) * (C / VEC);
  hipLaunchKernelGGL((activation1d_rs_kernel<VEC, P, R>), dim3((unsigned)cdiv64(n, 256)), dim3(256), 0, s, x, y, B, L,
                     C, ldy, al, bl, filt, tv, tv_mul);
}

// tv / tv_mul (optional): ragged batches, utterance b's sequence is min(L, tv[b] * tv_mul) rows long
int activation1d(const float* x, f16* y, int B, int L, int C, int ldy, const float* alpha_log, const float* beta_log,
                 const float* filt, hipStream_t s, const int* tv, int tv_mul) {
  SVC_REQUIRE(L >= 1 && C >= 4 && C % 4 == 0 && ldy % 4 == 0, "activation1d: L=%d C=%d ldy=%d", L, C, ldy);
  SVC_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 7) == 0, "activation1d: alignment");
  const int tok = prof_begin("activation1d", 0.0, (double)B * L * C * (4 + 2), s);
  // tuning act_variant (A/B runs, tests): 0 = LDS-tiled kernel, 1..4 = register streaming
  const int variant = tuning().act_variant;
  if (variant == 1) {
    launch_rs<4, 8, 128>(x, y, B, L, C, ldy, alpha_log, beta_log, filt, tv, tv_mul, s);
  } else if (variant == 2) {
    launch_rs<2, 8, 128>(x, y, B, L, C, ldy, alpha_log, beta_log, filt, tv, tv_mul, s);
  } else if (variant == 3) {
    launch_rs<4, 4, 64>(x, y, B, L, C, ldy, alpha_log, beta_log, filt, tv, tv_mul, s);
  } else if (variant == 4) {
    launch_rs<1, 8, 128>(x, y, B, L, C, ldy, alpha_log, beta_log, filt, tv, tv_mul, s);
  } else if (C % 64 == 0) {
    hipLaunchKernelGGL(activation1d_v2_kernel<16>, dim3(cdiv(L, A2_TT), C / 64, B), dim3(256), 0, s, x, y, L, C, ldy,
                       alpha_log, beta_log, filt, tv, tv_mul);
  } else if (C % 48 == 0) {
    hipLaunchKernelGGL(activation1d_v2_kernel<12>, dim3(cdiv(L, A2_TT), C / 48, B), dim3(256), 0, s, x, y, L, C, ldy,
                       alpha_log, beta_log, filt, tv, tv_mul);
  } else {
    hipLaunchKernelGGL(activation1d_v2_kernel<6>, dim3(cdiv(L, A2_TT), cdiv(C, 24), B), dim3(256), 0, s, x, y, L, C,
                       ldy, alpha_log, beta_log, filt, tv, tv_mul);
  }
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
