// SnakeBeta building blocks shared by activation.hip and amp_conv.hip (modules/bigvgan.py:146-159).
#pragma once
#include "common.h"

namespace svc {

// sin(x) by v_sin_f32 after an explicit reduction to [-0.5, 0.5] revolutions: its error (~|x|*6e-8) is the
// size of the f32 rounding of the argument u*alpha that the reference itself incurs.
__device__ __forceinline__ float sin_rev(float x) {
  float r = x * 0.15915494309189535f;
  r = r - rintf(r);
  return __builtin_amdgcn_sinf(r);
}

// VEC adjacent channels: f32 or f16 loads, saturating f16 stores
template <int VEC>
struct ActVec;
template <>
struct ActVec<1> {
  __device__ static void load(const float* p, float* o) { o[0] = *p; }
  __device__ static void load(const f16* p, float* o) { o[0] = (float)*p; }
  __device__ static void store(f16* p, const float* v) { *p = f16_sat(v[0]); }
};
template <>
struct ActVec<2> {
  __device__ static void load(const float* p, float* o) {
    const float2 v = *reinterpret_cast<const float2*>(p);
    o[0] = v.x; o[1] = v.y;
  }
  __device__ static void load(const f16* p, float* o) {
    union { unsigned u; f16 h[2]; } v;
    v.u = *reinterpret_cast<const unsigned*>(p);
    o[0] = (float)v.h[0]; o[1] = (float)v.h[1];
  }
  __device__ static void store(f16* p, const float* v) {
    union { unsigned u; f16 h[2]; } pk;
    pk.h[0] = f16_sat(v[0]);
    pk.h[1] = f16_sat(v[1]);
    *reinterpret_cast<unsigned*>(p) = pk.u;
  }
};
template <>
struct ActVec<4> {
  __device__ static void load(const float* p, float* o) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  __device__ static void load(const f16* p, float* o) {
    union { uint2 u; f16 h[4]; } v;
    v.u = *reinterpret_cast<const uint2*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (float)v.h[i];
  }
  __device__ static void store(f16* p, const float* v) {
    union { uint2 u; f16 h[4]; } pk;
#pragma unroll
    for (int i = 0; i < 4; ++i) pk.h[i] = f16_sat(v[i]);
    *reinterpret_cast<uint2*>(p) = pk.u;
  }
};

}  // namespace svc
