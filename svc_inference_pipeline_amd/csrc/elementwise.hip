// Bandwidth-bound kernels of the SVC path on gfx950: LayerNorm (fp32 statistics), content mapping,
// conditioner bucketize,
// sampler updates (DDPM / PLMS), mel de-normalisation, conv_post+tanh+fade.
// All tensors are time-major [rows = b*T + t][channels].
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace svc {

// ============================================================================ LayerNorm
// utils/whisper_extractor/model.py:29-31 (LayerNorm in fp32), eps 1e-5, biased variance.
// 16-bit outputs are GEMM operands: binary16, or bfloat16 bits when bf (the bf16 operand variant, common.h Op16)
template <typename OutT, bool SPLIT = false>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, const float* __restrict__ gam,
                                                        const float* __restrict__ bet, OutT* __restrict__ y, int rows,
                                                        int D, int ldy, bool bf) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * D;
  float v[16];
  const int per = D / 64;  // D in {64..1024}, multiple of 64
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < per) {
      v[i] = xr[i * 64 + lane];
      s += v[i];
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < per) {
      float d = v[i] - mean;
      ss += d * d;
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  const float rstd = 1.0f / sqrtf(ss / (float)D + 1e-5f);
  OutT* yr = y + (int64_t)row * ldy;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < per) {
      int c = i * 64 + lane;
      const float o = (v[i] - mean) * rstd * gam[c] + bet[c];
      if constexpr (std::is_same<OutT, float>::value) {
        yr[c] = o;
      } else {
        yr[c] = enc16_lo(o, bf);
        if constexpr (SPLIT) {  // split-fp16 operand [hi | lo | hi] (ldy >= 3 D)
          yr[D + c] = enc16_lo(o - dec16(yr[c], bf), bf);
          yr[2 * D + c] = yr[c];
        }
      }
    }
}

// D % 256 == 0 (Whisper 1024, HuBERT 768): element c = q * 256 + 4 * lane + k, so every load / store instruction of
// the wave is one contiguous 1 KiB (f32) / 512 B (f16) run: 16-B loads and 8-B stores instead of 4-B / 2-B ones
template <typename OutT, bool SPLIT>
__global__ __launch_bounds__(256) void layernorm_v4_kernel(const float* __restrict__ x, const float* __restrict__ gam,
                                                           const float* __restrict__ bet, OutT* __restrict__ y,
                                                           int rows, int D, int ldy, bool bf) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * D;
  const int nq = D / 256;  // <= 4
  float4 v[4];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < nq) {
      v[q] = *reinterpret_cast<const float4*>(xr + q * 256 + 4 * lane);
      s += (v[q].x + v[q].y) + (v[q].z + v[q].w);
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < nq) {
      const float a = v[q].x - mean, b = v[q].y - mean, c = v[q].z - mean, d = v[q].w - mean;
      ss += (a * a + b * b) + (c * c + d * d);
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  const float rstd = 1.0f / sqrtf(ss / (float)D + 1e-5f);
  OutT* yr = y + (int64_t)row * ldy;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < nq) {
      const int c = q * 256 + 4 * lane;
      const float4 g = *reinterpret_cast<const float4*>(gam + c);
      const float4 bb = *reinterpret_cast<const float4*>(bet + c);
      const float o[4] = {(v[q].x - mean) * rstd * g.x + bb.x, (v[q].y - mean) * rstd * g.y + bb.y,
                          (v[q].z - mean) * rstd * g.z + bb.z, (v[q].w - mean) * rstd * g.w + bb.w};
      if constexpr (std::is_same<OutT, float>::value) {
        *reinterpret_cast<float4*>(yr + c) = make_float4(o[0], o[1], o[2], o[3]);
        continue;
      }
      union { uint2 u; f16 h[4]; } hi, lo;
#pragma unroll
      for (int k = 0; k < 4; ++k) hi.h[k] = enc16_lo(o[k], bf);
      *reinterpret_cast<uint2*>(yr + c) = hi.u;
      if constexpr (SPLIT) {  // split-fp16 operand [hi | lo | hi] (ldy >= 3 D)
#pragma unroll
        for (int k = 0; k < 4; ++k) lo.h[k] = enc16_lo(o[k] - dec16(hi.h[k], bf), bf);
        *reinterpret_cast<uint2*>(yr + D + c) = lo.u;
        *reinterpret_cast<uint2*>(yr + 2 * D + c) = hi.u;
      }
    }
}

int layernorm_f16(const float* x, const float* g, const float* b, f16* y, int rows, int D, int ldy, hipStream_t s,
                  bool bf) {
  SVC_REQUIRE(D % 64 == 0 && D <= 1024, "layernorm: D=%d", D);
  if (D % 256 == 0 && ldy % 4 == 0)
    hipLaunchKernelGGL((layernorm_v4_kernel<f16, false>), dim3(cdiv(rows, 4)), dim3(256), 0, s, x, g, b, y, rows, D,
                       ldy, bf);
  else
    hipLaunchKernelGGL(layernorm_kernel<f16>, dim3(cdiv(rows, 4)), dim3(256), 0, s, x, g, b, y, rows, D, ldy, bf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}
int layernorm_f16x3(const float* x, const float* g, const float* b, f16* y, int rows, int D, hipStream_t s, bool bf) {
  SVC_REQUIRE(D % 64 == 0 && D <= 1024, "layernorm: D=%d", D);
  if (D % 256 == 0)
    hipLaunchKernelGGL((layernorm_v4_kernel<f16, true>), dim3(cdiv(rows, 4)), dim3(256), 0, s, x, g, b, y, rows, D,
                       3 * D, bf);
  else
    hipLaunchKernelGGL((layernorm_kernel<f16, true>), dim3(cdiv(rows, 4)), dim3(256), 0, s, x, g, b, y, rows, D,
                       3 * D, bf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}
int layernorm_f32(const float* x, const float* g, const float* b, float* y, int rows, int D, int ldy, hipStream_t s) {
  SVC_REQUIRE(D % 64 == 0 && D <= 1024, "layernorm: D=%d", D);
  if (D % 256 == 0 && ldy % 4 == 0)
    hipLaunchKernelGGL((layernorm_v4_kernel<float, false>), dim3(cdiv(rows, 4)), dim3(256), 0, s, x, g, b, y, rows, D,
                       ldy, false);
  else
    hipLaunchKernelGGL(layernorm_kernel<float>, dim3(cdiv(rows, 4)), dim3(256), 0, s, x, g, b, y, rows, D, ldy, false);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// Activation1d (anti-aliased SnakeBeta) lives in activation.hip.

// ============================================================================ conversions
__global__ void f32_to_f16_kernel(const float* __restrict__ x, int ldx, f16* __restrict__ y, int ldy, int rows, int C,
                                  int Cpad, bool bf) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t n = (int64_t)rows * Cpad;
  if (i >= n) return;
  int r = (int)(i / Cpad), c = (int)(i - (int64_t)r * Cpad);
  y[(int64_t)r * ldy + c] = c < C ? enc16(x[(int64_t)r * ldx + c], bf) : (f16)0.0f;  // +0 in both formats
}

int f32_to_f16(const float* x, int ldx, f16* y, int ldy, int rows, int C, int Cpad, hipStream_t s, bool bf) {
  int64_t n = (int64_t)rows * Cpad;
  hipLaunchKernelGGL(f32_to_f16_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, x, ldx, y, ldy, rows, C, Cpad, bf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// Split-fp16 operand ("fp16x3"): x f32 [rows][ldx] -> y f16 [rows][3C] = [hi | lo | hi], hi = f16(x),
// lo = f16(x - hi). A GEMM over these 3C columns against weights packed [W_hi; W_hi; W_lo] (pack_gemm_split3)
// computes x_hi W_hi + x_lo W_hi + x_hi W_lo: ~19 significand bits instead of fp16's 11, at 3x the MFMA work.
__global__ void f32_to_f16x3_kernel(const float* __restrict__ x, int ldx, f16* __restrict__ y, int rows, int C,
                                    bool bf) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * C) return;
  const int r = (int)(i / C), c = (int)(i - (int64_t)r * C);
  const float v = x[(int64_t)r * ldx + c];
  const f16 hi = enc16(v, bf);
  const f16 lo = enc16_lo(v - dec16(hi, bf), bf);
  f16* yr = y + (int64_t)r * 3 * C;
  yr[c] = hi;
  yr[C + c] = lo;
  yr[2 * C + c] = hi;
}

// grouped layout for grouped convolutions: group g's split operand is contiguous, [g][hi | lo | hi] of Cg columns
__global__ void f32_to_f16x3_grouped_kernel(const float* __restrict__ x, f16* __restrict__ y, int rows, int C, int Cg,
                                            bool bf) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * C) return;
  const int r = (int)(i / C), c = (int)(i - (int64_t)r * C);
  const int g = c / Cg, j = c - g * Cg;
  const float v = x[i];
  const f16 hi = enc16(v, bf);
  f16* yg = y + (int64_t)r * 3 * C + (int64_t)g * 3 * Cg;
  yg[j] = hi;
  yg[Cg + j] = enc16_lo(v - dec16(hi, bf), bf);
  yg[2 * Cg + j] = hi;
}

int f32_to_f16x3_grouped(const float* x, f16* y, int rows, int C, int Cg, hipStream_t s, bool bf) {
  SVC_REQUIRE(C % Cg == 0, "f16x3 grouped: C=%d Cg=%d", C, Cg);
  const int64_t n = (int64_t)rows * C;
  hipLaunchKernelGGL(f32_to_f16x3_grouped_kernel, dim3((unsigned)cdiv64(n, 256)), dim3(256), 0, s, x, y, rows, C, Cg,
                     bf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

int f32_to_f16x3(const float* x, int ldx, f16* y, int rows, int C, hipStream_t s, bool bf) {
  const int64_t n = (int64_t)rows * C;
  hipLaunchKernelGGL(f32_to_f16x3_kernel, dim3((unsigned)cdiv64(n, 256)), dim3(256), 0, s, x, ldx, y, rows, C, bf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

__global__ void f16_to_f32_kernel(const f16* __restrict__ x, float* __restrict__ y, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = (float)x[i];
}

int f16_to_f32(const f16* x, float* y, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(f16_to_f32_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, x, y, n);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// q,k,v f32 [rows][D] -> f16 [rows][3D] with q,k scaled and q also by log2(e) (the QKV GEMM epilogue's layout;
// op-level tests)
__global__ void pack_qkv_kernel(const float* q, const float* k, const float* v, f16* o, int64_t rows, int D, float sc) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * D) return;
  int64_t r = i / D;
  int c = (int)(i - r * D);
  o[r * 3 * D + c] = (f16)(q[i] * (sc * ATT_LOG2E));
  o[r * 3 * D + D + c] = (f16)(k[i] * sc);
  o[r * 3 * D + 2 * D + c] = (f16)v[i];
}

int pack_qkv(const float* q, const float* k, const float* v, f16* qkv, int64_t rows, int D, float scale, hipStream_t s) {
  hipLaunchKernelGGL(pack_qkv_kernel, dim3(cdiv(rows * D, 256)), dim3(256), 0, s, q, k, v, qkv, rows, D, scale);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// mel de-normalisation (utils/acoustic_feature_extraction.py:83-97) fused with the f16 conversion
// of the vocoder input: y = (x+1)/2*(max-min+1e-12)+min, x f32 [rows][100] -> f16 [rows][ldy]
__global__ void denorm_mel_kernel(const float* __restrict__ x, f16* __restrict__ y, float* __restrict__ y32, int ldy,
                                  int rows, int C, const float* __restrict__ mn, const float* __restrict__ mx) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * ldy) return;
  int r = (int)(i / ldy), c = (int)(i - (int64_t)r * ldy);
  float v = 0.f;
  if (c < C) {
    v = (x[(int64_t)r * C + c] + 1.0f) / 2.0f * (mx[c] - mn[c] + 1e-12f) + mn[c];
    if (y32) y32[(int64_t)r * C + c] = v;
  }
  y[i] = f16_sat(v);
}

int denorm_mel(const float* x, f16* y, float* y32, int ldy, int rows, int C, const float* mn, const float* mx,
               hipStream_t s) {
  int64_t n = (int64_t)rows * ldy;
  hipLaunchKernelGGL(denorm_mel_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, x, y, y32, ldy, rows, C, mn, mx);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// ============================================================================ content mapping
// utils/whisper.py:31-81: 15:8 repeat/average. Row j of the output averages the 8 repeated rows
// 8j..8j+7 of np.repeat(raw, 15): source rows (8j+i)//15, summed sequentially in f32 then /8.
__global__ void content_map_kernel(const float* __restrict__ src, int src_rows_per_utt, int ld_src,
                                   f16* __restrict__ dst, int ld_dst, int T, int D, int n_down, bool bf) {
  const int jo = blockIdx.x;  // output frame
  const int j = min(jo, n_down - 1);  // HuBERT: frames past the mapped length repeat the last one
  const int b = blockIdx.y;
  const float* sb = src + (int64_t)b * src_rows_per_utt * ld_src;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += sb[(int64_t)((8 * j + i) / 15) * ld_src + c];
    dst[((int64_t)b * T + jo) * ld_dst + c] = enc16_lo(acc / 8.0f, bf);
  }
}

int content_map(const float* src, int B, int src_rows, int ld_src, int T, int D, f16* dst, int ld_dst, hipStream_t s,
                bool bf) {
  // the reference caps the target at 2812 frames (utils/whisper.py:56); longer clips are chunked by the host
  SVC_REQUIRE(T >= 1 && T <= 2812 && (T * 8 / 15 + 1) <= src_rows, "content_map: T=%d src_rows=%d", T, src_rows);
  hipLaunchKernelGGL(content_map_kernel, dim3(T, B), dim3(256), 0, s, src, src_rows, ld_src, dst, ld_dst, T, D, T, bf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// utils/hubert.py:83-134 (get_mapped_features): the same 15:8 average over all src_rows frames, no cap;
// n_down = src_rows*15//8 mapped frames, at most 3 missing frames repeat the last one, and a larger
// mismatch is an error (the reference calls exit()).
int content_map_hubert(const float* src, int B, int src_rows, int ld_src, int T, int D, f16* dst, int ld_dst,
                       hipStream_t s, bool bf) {
  const int n_down = (int)((int64_t)src_rows * 15 / 8);
  SVC_REQUIRE(T >= 1 && src_rows >= 1 && n_down >= 1 && std::abs(T - n_down) <= 3,
              "content_map_hubert: %d content frames map to %d rows but T=%d (|diff| > 3; utils/hubert.py:114-120)",
              src_rows, n_down, T);
  hipLaunchKernelGGL(content_map_kernel, dim3(T, B), dim3(256), 0, s, src, src_rows, ld_src, dst, ld_dst, T, D, n_down,
                     bf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// ============================================================================ bucketize
// torch.bucketize(x, bins) with right=False = number of bins < x. f0 is float64 and the f32 bins are
// widened exactly (torch promotes to f64); energy is compared in f32 (modules/encoder.py:70,115).
// The search step is torch's own `!(bins[mid] >= x)` (ATen Bucketization cus_lower_bound), not `bins[mid] < x`:
// the two differ for NaN, which torch places past the last bin (index nb). NaN f0 is what pitch_shift gives an
// utterance with no voiced frame (np.median of an empty array).
__global__ void bucketize_kernel(const double* __restrict__ f0, const float* __restrict__ en,
                                 const float* __restrict__ mbins, const float* __restrict__ ebins, int nb,
                                 int* __restrict__ im, int* __restrict__ ie, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double fv = f0[i];
  const float ev = en[i];
  int lo = 0, hi = nb;  // first index with bins[idx] >= x
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (!((double)mbins[mid] >= fv)) lo = mid + 1; else hi = mid;
  }
  im[i] = lo;
  lo = 0; hi = nb;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (!(ebins[mid] >= ev)) lo = mid + 1; else hi = mid;
  }
  ie[i] = lo;
}

int bucketize(const double* f0, const float* en, const float* mbins, const float* ebins, int nb, int* im, int* ie,
              int n, hipStream_t s) {
  hipLaunchKernelGGL(bucketize_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, f0, en, mbins, ebins, nb, im, ie, n);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// ============================================================================ samplers
// x, eps, hist: f32 [rows][100]; x16: f16 copy [rows][ld16] for the next mel_preprocess GEMM.
// PLMS (modules/diffsvcrepo_inference.py:91-151): e' = sum_i c_i * e_i / div ; x = x + d*(A*x - Bc*e')

__global__ void plms_kernel(PlmsArgs p, int rows, int C) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * C) return;
  // signed combination in the reference's left-to-right order:
  // first step (e0 + e1) / 2 ; AB2 (3 e0 - e1) / 2 ; AB3 (23 e0 - 16 e1 + 5 e2) / 12 ;
  // AB4 (55 e0 - 59 e1 + 37 e2 - 9 e3) / 24
  float e = p.c[0] * p.e[0][i];
  if (p.ne >= 2) e = e + p.c[1] * p.e[1][i];
  if (p.ne >= 3) e = e + p.c[2] * p.e[2][i];
  if (p.ne >= 4) e = e + p.c[3] * p.e[3][i];
  e = e / p.div;
  if (p.e_avg_out) p.e_avg_out[i] = e;
  const float x = p.xin[i];
  const float xn = x + p.d * (p.A * x - p.Bc * e);
  p.xout[i] = xn;
  if (p.x16) {
    int64_t r = i / C;
    int c = (int)(i - r * C);
    p.x16[r * p.ld16 + c] = enc16(xn, p.bf16);
  }
}

// the same update on 4 consecutive channels per thread (C % 4 == 0, 16-B aligned rows): 16-B loads and stores, an 8-B
// f16 store, a quarter of the threads; per element the identical operations in the identical order
__global__ void plms4_kernel(PlmsArgs p, int rows, int C) {
  const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int C4 = C >> 2;
  if (i4 >= (int64_t)rows * C4) return;
  const int64_t i = i4 * 4;
  auto ld = [&](const float* q) { return *reinterpret_cast<const float4*>(q + i); };
  float4 ev[4];
  ev[0] = ld(p.e[0]);
#pragma unroll
  for (int k = 1; k < 4; ++k)
    if (p.ne > k) ev[k] = ld(p.e[k]);
  float4 e, xn;
  plms_math4(p, ev, ld(p.xin), e, xn);
  if (p.e_avg_out) *reinterpret_cast<float4*>(p.e_avg_out + i) = e;
  *reinterpret_cast<float4*>(p.xout + i) = xn;
  if (p.x16) {
    const int64_t r = i4 / C4;
    const int c = (int)(i4 - r * C4) * 4;
    union { uint2 u; f16 h[4]; } pk;
    const bool bf = p.bf16;
    pk.h[0] = enc16(xn.x, bf); pk.h[1] = enc16(xn.y, bf); pk.h[2] = enc16(xn.z, bf); pk.h[3] = enc16(xn.w, bf);
    *reinterpret_cast<uint2*>(p.x16 + r * p.ld16 + c) = pk.u;
  }
}

// the 4-channel form's layout conditions (plms4_kernel)
static bool plms_vec4_ok(const PlmsArgs& p, int C) {
  bool vec = C % 4 == 0 && (!p.x16 || p.ld16 % 4 == 0);
  const void* ptrs[] = {p.e[0], p.ne > 1 ? p.e[1] : nullptr, p.ne > 2 ? p.e[2] : nullptr, p.ne > 3 ? p.e[3] : nullptr,
                        p.xin, p.xout, p.e_avg_out, p.x16};
  for (int k = 0; k < 8; ++k) vec = vec && ((uintptr_t)ptrs[k] & (k == 7 ? 7 : 15)) == 0;
  return vec;
}

int plms_update(const PlmsArgs& p, int rows, int C, hipStream_t s) {
  int64_t n = (int64_t)rows * C;
  if (plms_vec4_ok(p, C))
    hipLaunchKernelGGL(plms4_kernel, dim3(cdiv(n / 4, 256)), dim3(256), 0, s, p, rows, C);
  else
    hipLaunchKernelGGL(plms_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, p, rows, C);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// counter-based normal noise (Philox4x32-10 + Box-Muller), keyed by (seed, utterance, step, element)
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ float philox_normal(uint64_t seed, uint32_t utt, uint32_t step, uint32_t elem) {
  uint32_t c[4] = {elem, step, utt, 0x5356434Bu};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  float u1 = ((c[0] >> 8) + 1) * (1.0f / 16777216.0f);  // (0,1]
  float u2 = (c[1] >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// x_T ~ N(0, (1/1.2)^2) generated on device (modules/diffsvcrepo_inference.py:208-214)
__global__ void init_noise_kernel(float* x, f16* x16, int ld16, int T, int C, uint64_t seed, const int* utt_ids,
                                  int rows, float std, bool bf) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * C) return;
  int64_t r = i / C;
  int c = (int)(i - r * C);
  int b = (int)(r / T), t = (int)(r - (int64_t)b * T);
  float v = std * philox_normal(seed, (uint32_t)utt_ids[b], 0xFFFFFFFFu, (uint32_t)(t * C + c));
  x[i] = v;
  x16[r * ld16 + c] = enc16(v, bf);
}

int init_noise(float* x, f16* x16, int ld16, int B, int T, int C, uint64_t seed, const int* utt_ids, float std,
               hipStream_t s, bool bf) {
  int rows = B * T;
  int64_t n = (int64_t)rows * C;
  hipLaunchKernelGGL(init_noise_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, x, x16, ld16, T, C, seed, utt_ids, rows,
                     std, bf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// DDPM p_sample (modules/diffsvcrepo_inference.py:56-88), clip_denoised=True. z either given
// (parity mode, [rows][C] already transposed from the reference's [B,1,C,T] draw) or generated.
struct DdpmArgs {
  float sra, srm1, c1, c2, sigma;  // sigma = exp(0.5*logvar) * (t > 0)
  const float* z; uint64_t seed; const int* utt_ids; int step;
  int bf16;  // x16 holds bfloat16 operands
};

__global__ void ddpm_kernel(float* x, const float* eps, f16* x16, int ld16, int T, int C, int rows, DdpmArgs a) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * C) return;
  int64_t r = i / C;
  int c = (int)(i - r * C);
  const float xv = x[i];
  float x0 = a.sra * xv - a.srm1 * eps[i];
  x0 = fminf(fmaxf(x0, -1.0f), 1.0f);
  float mean = a.c1 * x0 + a.c2 * xv;
  float z;
  if (a.z) {
    z = a.z[i];
  } else {
    int b = (int)(r / T), t = (int)(r - (int64_t)b * T);
    // keyed by (t, c) like x_T, not by c * T + t: an utterance draws the same noise in any batch (ragged or not)
    z = philox_normal(a.seed, (uint32_t)a.utt_ids[b], (uint32_t)a.step, (uint32_t)(t * C + c));
  }
  float xn = mean + a.sigma * z;
  x[i] = xn;
  x16[r * ld16 + c] = enc16(xn, a.bf16);
}

int ddpm_update(float* x, const float* eps, f16* x16, int ld16, int B, int T, int C, const DdpmArgs& a, hipStream_t s) {
  int rows = B * T;
  int64_t n = (int64_t)rows * C;
  hipLaunchKernelGGL(ddpm_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, x, eps, x16, ld16, T, C, rows, a);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// ============================================================================ conv_post + tanh + fade
// modules/bigvgan.py:593,619-620 (Conv1d(ch,1,7,pad 3) + tanh) and modules/bigvgan_inference.py:37-42
// (trim to T*256 and linear fade-out of the last 20*256 samples). a: f16 [B*L][C], w: f32 [C][7].
// Ragged batches (tv != NULL): utterance b has Lb = tv[b] * tv_mul samples; its conv zero padding, trim and fade-out
// are at Lb, and the samples [Lb, L) of its output row are written as zeros.
__global__ void conv_post_kernel(const f16* __restrict__ a, int lda, int L, int C, const float* __restrict__ w,
                                 float bias, const float* __restrict__ fade, int nfade, float* __restrict__ out,
                                 const int* __restrict__ tv, int tv_mul) {
  __shared__ float ws[96 * 7];
  for (int i = threadIdx.x; i < C * 7; i += blockDim.x) ws[i] = w[i];
  __syncthreads();
  const int b = blockIdx.y;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L) return;
  const int Lb = tv ? min(L, tv[b] * tv_mul) : L;
  if (t >= Lb) {
    out[(int64_t)b * L + t] = 0.f;
    return;
  }
  const f16* ab = a + (int64_t)b * L * lda;
  float acc = 0.f;
  for (int k = 0; k < 7; ++k) {
    int tt = t + k - 3;
    if (tt < 0 || tt >= Lb) continue;
    const f16* row = ab + (int64_t)tt * lda;
    for (int c = 0; c < C; ++c) acc += (float)row[c] * ws[c * 7 + k];
  }
  float y = tanhf(acc + bias);
  int fs = Lb - nfade;
  if (t >= fs) y *= fade[t - fs];
  out[(int64_t)b * L + t] = y;
}

int conv_post(const f16* a, int lda, int B, int L, int C, const float* w, float bias, const float* fade, int nfade,
              float* out, hipStream_t s, const int* tv, int tv_mul) {
  SVC_REQUIRE(C <= 96 && L >= nfade, "conv_post: C=%d L=%d", C, L);
  hipLaunchKernelGGL(conv_post_kernel, dim3(cdiv(L, 256), B), dim3(256), 0, s, a, lda, L, C, w, bias, fade, nfade, out,
                     tv, tv_mul);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc

namespace svc {
// ============================================================================ pitch shift
// utils/acoustic_feature_extraction.py:33-52: factor = target_median / median(voiced f0); f0 *= factor.
// The median of the voiced frames (np.median: middle element, or the mean of the two middle ones)
// is found with a 64-pass radix select over order-preserving integer keys; one workgroup per utterance.
__device__ __forceinline__ uint64_t dkey(double v) {
  uint64_t b = (uint64_t)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ double block_select(const double* f, int T, int k, int* red) {
  uint64_t prefix = 0, mask = 0;
  for (int bit = 63; bit >= 0; --bit) {
    const uint64_t bm = 1ull << bit;
    int cnt = 0;
    for (int i = threadIdx.x; i < T; i += blockDim.x) {
      double v = f[i];
      if (v != 0.0) {
        uint64_t kk = dkey(v);
        cnt += ((kk & mask) == prefix) && !(kk & bm);
      }
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
    __syncthreads();
    int tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += red[w];
    if (k >= tot) {
      k -= tot;
      prefix |= bm;
    }
    mask |= bm;
  }
  uint64_t b = (prefix >> 63) ? (prefix & 0x7FFFFFFFFFFFFFFFull) : ~prefix;
  return __longlong_as_double((long long)b);
}

__global__ __launch_bounds__(256) void pitch_shift_kernel(double* f0, int T, double target) {
  __shared__ int red[4];
  double* f = f0 + (int64_t)blockIdx.x * T;
  int n = 0;
  for (int i = threadIdx.x; i < T; i += blockDim.x) n += f[i] != 0.0;
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = n;
  __syncthreads();
  n = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  double med;
  if (n == 0) {
    med = __longlong_as_double(0x7FF8000000000000ll);  // np.median of an empty selection is NaN
  } else if (n & 1) {
    med = block_select(f, T, n / 2, red);
  } else {
    double a = block_select(f, T, n / 2 - 1, red);
    double b = block_select(f, T, n / 2, red);
    med = (a + b) / 2.0;
  }
  const double factor = target / med;
  __syncthreads();
  for (int i = threadIdx.x; i < T; i += blockDim.x) f[i] = f[i] * factor;
}

int pitch_shift(double* f0, int B, int T, double target, hipStream_t s) {
  hipLaunchKernelGGL(pitch_shift_kernel, dim3(B), dim3(256), 0, s, f0, T, target);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}
}  // namespace svc
