// SnakeBeta building blocks shared by activation.hip and amp_conv.hip (modules/bigvgan.py:146-159).
#pragma once
#include "common.h"

namespace svc {

// Channel pairs on the packed f32 VALU (v_pk_fma_f32 / v_pk_mul_f32: two channels per issue; f32x2 in common.h).

// SnakeBeta constants of channels c, c+1: alpha / 2pi (the sine's argument in revolutions) and 1 / (beta + 1e-9)
struct SnakeCoef2 {
  f32x2 ar, ib;
};
__device__ __forceinline__ SnakeCoef2 snake_coef2(const float* alpha_log, const float* beta_log, int c) {
  SnakeCoef2 k;
  k.ar = f32x2{expf(alpha_log[c]), expf(alpha_log[c + 1])} * 0.15915494309189535f;
  k.ib = f32x2{1.0f / (expf(beta_log[c]) + 0.000000001f), 1.0f / (expf(beta_log[c + 1]) + 0.000000001f)};
  return k;
}
// u + sin(u * alpha)^2 / beta: v_sin_f32 on the fractional revolution fract(u * alpha / 2pi) (exact reduction of the
// rounded argument; one v_fract instead of the round-and-subtract of sin_rev). 3 packed ops + 2 x (fract, sin).
__device__ __forceinline__ f32x2 snake2(f32x2 u, const SnakeCoef2& k) {
  const f32x2 r = u * k.ar;
  f32x2 sn;
  sn.x = __builtin_amdgcn_sinf(__builtin_amdgcn_fractf(r.x));
  sn.y = __builtin_amdgcn_sinf(__builtin_amdgcn_fractf(r.y));
  return u + k.ib * (sn * sn);
}
// f16 pair, saturating at +-65504 (v_med3_f32 + v_cvt_pk_f16_f32)
__device__ __forceinline__ unsigned f16x2_sat(f32x2 v) {
  union { unsigned u; f16 h[2]; } pk;
  pk.h[0] = (f16)__builtin_amdgcn_fmed3f(v.x, -65504.f, 65504.f);
  pk.h[1] = (f16)__builtin_amdgcn_fmed3f(v.y, -65504.f, 65504.f);
  return pk.u;
}
// a channel pair of an f32 or f16 tensor at a 32-bit buffer offset (vo per lane, so wave-uniform)
template <typename TX>
__device__ __forceinline__ f32x2 act_load(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
  if constexpr (sizeof(TX) == 4) {
    return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
  } else {
    union { unsigned u; f16 h[2]; } v;
    v.u = __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0);
    return f32x2{(float)v.h[0], (float)v.h[1]};
  }
}
// the loaded form of a channel pair (f32: the pair; f16: one raw word) and its conversion
template <typename TX>
using act_raw_t = typename std::conditional<sizeof(TX) == 4, f32x2, unsigned>::type;
template <typename TX>
__device__ __forceinline__ act_raw_t<TX> act_load_raw(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
  if constexpr (sizeof(TX) == 4)
    return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
  else
    return __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0);
}
template <typename TX>
__device__ __forceinline__ f32x2 act_cvt(act_raw_t<TX> v) {
  if constexpr (sizeof(TX) == 4) {
    return v;
  } else {
    union { unsigned u; f16 h[2]; } w;
    w.u = v;
    return f32x2{(float)w.h[0], (float)w.h[1]};
  }
}
// s[2tb-5+i] (UpSample1d then SnakeBeta) from the window xw[k] = x[tb-5+k], exact for every index inside [0, 2L-1]:
//   u[2q] = sum_a x[q-3+a] * 2f[11-2a],  u[2q+1] = sum_a x[q-2+a] * 2f[10-2a]   (f2 = 2f: the factor 2 is exact)
__device__ __forceinline__ f32x2 snake_up(const f32x2* xw, int i, const float (&f2)[12], const SnakeCoef2& kc) {
  const int odd = (i + 1) & 1;  // parity of j = 2tb-5+i
  const int base = ((i - 5) >> 1) + 2 + odd;
  f32x2 o = xw[base] * f2[11 - odd];
#pragma unroll
  for (int a = 1; a < 6; ++a) o += xw[base + a] * f2[11 - odd - 2 * a];
  return snake2(o, kc);
}
// LowPassFilter1d output t from s[2t-5 .. 2t+6] = sw[0..11]
__device__ __forceinline__ f32x2 snake_down(const f32x2* sw, const float (&f)[12]) {
  f32x2 acc = sw[0] * f[0];
#pragma unroll
  for (int k = 1; k < 12; ++k) acc += sw[k] * f[k];
  return acc;
}

}  // namespace svc
