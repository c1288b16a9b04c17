// HuBERT / ContentVec content encoder helpers (utils/hubert.py:31-47): the pieces of
// fairseq's HubertModel.extract_features that are not implicit GEMMs. The convolutions, projections and
// attention reuse conv_gemm3 / conv_gemm / attention (engine.hip: svc_hubert_encode).
//
//   frames5       : wav f32 [B][n] -> f16 [B][ceil(n/5)][8]: row r holds samples 5r..5r+4 (cols 5..7 zero), so
//                   conv_layers[0] (k=10, stride 5) becomes a 2-tap stride-1 implicit GEMM over these rows.
//   colstats      : Fp32GroupNorm(C, C) statistics — per (utterance, channel) sum / sum of squares over time, f64
//                   partials per row chunk (coalesced: a block streams whole rows, each lane owns 2 channels).
//   gn_finalize   : partials -> per (utterance, channel) scale = gamma * rstd, shift = beta - mean * scale.
//   gn_gelu_apply : y16 = GELU(x * scale + shift), f32 -> f16, 16-byte vectors.
//   layernorm_dual: LayerNorm writing both the f32 residual stream and its f16 GEMM operand (post-LN layers).
#include "common.h"

namespace svc {

// SPLIT: 16 halves per row = [hi(5) | lo(5) | hi(5) | 0] (split-fp16 operand of the split-packed conv_layers[0])
template <bool SPLIT>
__global__ void frames5_kernel(const float* __restrict__ wav, int64_t n, int64_t rows, f16* __restrict__ out, bool bf) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one output row (8 or 16 halves)
  const int b = blockIdx.y;
  if (i >= rows) return;
  const float* w = wav + (int64_t)b * n;
  constexpr int W = SPLIT ? 16 : 8;
  union { uint4 u[W / 8]; f16 h[W]; } pk;
#pragma unroll
  for (int j = 0; j < W; ++j) pk.h[j] = (f16)0.0f;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int64_t k = 5 * i + j;
    const float v = k < n ? w[k] : 0.0f;
    const f16 hi = enc16_lo(v, bf);
    pk.h[j] = hi;
    if constexpr (SPLIT) {
      pk.h[5 + j] = enc16_lo(v - dec16(hi, bf), bf);
      pk.h[10 + j] = hi;
    }
  }
#pragma unroll
  for (int q = 0; q < W / 8; ++q) *reinterpret_cast<uint4*>(out + ((int64_t)b * rows + i) * W + q * 8) = pk.u[q];
}

int hubert_frames5(const float* wav, int B, int64_t n, f16* out, bool split, hipStream_t s, bool bf) {
  const int64_t rows = cdiv64(n, 5);
  if (split)
    hipLaunchKernelGGL(frames5_kernel<true>, dim3(cdiv(rows, 256), B), dim3(256), 0, s, wav, n, rows, out, bf);
  else
    hipLaunchKernelGGL(frames5_kernel<false>, dim3(cdiv(rows, 256), B), dim3(256), 0, s, wav, n, rows, out, bf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// grid (chunks, B), 256 threads; lane pair p = 2 adjacent channels
__global__ __launch_bounds__(256) void colstats_kernel(const float* __restrict__ x, int T, int C, int chunk,
                                                       double* __restrict__ part) {
  const int ck = blockIdx.x, b = blockIdx.y, nck = gridDim.x;
  const int r0 = ck * chunk, r1 = min(T, r0 + chunk);
  const float* xb = x + (int64_t)b * T * C;
  for (int p = threadIdx.x; p < C / 2; p += blockDim.x) {
    double s0 = 0, s1 = 0, q0 = 0, q1 = 0;
    int r = r0;
    for (; r + 4 <= r1; r += 4) {
      float2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float2*>(xb + (int64_t)(r + u) * C + 2 * p);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s0 += v[u].x; q0 += (double)v[u].x * v[u].x;
        s1 += v[u].y; q1 += (double)v[u].y * v[u].y;
      }
    }
    for (; r < r1; ++r) {
      const float2 v = *reinterpret_cast<const float2*>(xb + (int64_t)r * C + 2 * p);
      s0 += v.x; q0 += (double)v.x * v.x;
      s1 += v.y; q1 += (double)v.y * v.y;
    }
    double* o = part + (((int64_t)b * nck + ck) * C + 2 * p) * 2;
    o[0] = s0; o[1] = q0; o[2] = s1; o[3] = q1;
  }
}

__global__ void gn_finalize_kernel(const double* __restrict__ part, int nck, int T, int C, const float* __restrict__ g,
                                   const float* __restrict__ be, float eps, float2* __restrict__ ss) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x, b = blockIdx.y;
  if (c >= C) return;
  double s = 0, q = 0;
  for (int k = 0; k < nck; ++k) {
    const double* p = part + (((int64_t)b * nck + k) * C + c) * 2;
    s += p[0];
    q += p[1];
  }
  const double mean = s / T;
  const double var = fmax(q / T - mean * mean, 0.0);  // biased, as F.group_norm
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float scale = g[c] * rstd;
  ss[(int64_t)b * C + c] = make_float2(scale, be[c] - (float)mean * scale);
}

template <bool SPLIT>
__global__ void gn_gelu_apply_kernel(const float* __restrict__ x, const float2* __restrict__ ss, f16* __restrict__ y,
                                     int64_t rows_per_utt, int C, int64_t nvec, bool bf) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one vector of 8 channels
  if (i >= nvec) return;
  const int cpr = C / 8;
  const int64_t row = i / cpr;
  const int c0 = (int)(i - row * cpr) * 8;
  const int b = (int)(row / rows_per_utt);
  const float4 a0 = *reinterpret_cast<const float4*>(x + row * C + c0);
  const float4 a1 = *reinterpret_cast<const float4*>(x + row * C + c0 + 4);
  const float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  union { uint4 u; f16 h[8]; } pk, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float2 t = ss[(int64_t)b * C + c0 + j];
    const float o = gelu_erf(v[j] * t.x + t.y);
    pk.h[j] = enc16(o, bf);
    lo.h[j] = enc16_lo(o - dec16(pk.h[j], bf), bf);
  }
  if constexpr (SPLIT) {  // [hi | lo | hi] rows of 3 C
    f16* yr = y + row * 3 * C;
    *reinterpret_cast<uint4*>(yr + c0) = pk.u;
    *reinterpret_cast<uint4*>(yr + C + c0) = lo.u;
    *reinterpret_cast<uint4*>(yr + 2 * C + c0) = pk.u;
  } else {
    *reinterpret_cast<uint4*>(y + row * C + c0) = pk.u;
  }
}

// Fp32GroupNorm(C, C) + GELU over x f32 [B][T][C] -> y f16 [B][T][C]. part: >= B * chunks * C * 2 doubles,
// ss: B * C float2.
int groupnorm_gelu(const float* x, int B, int T, int C, const float* gamma, const float* beta, double* part,
                   int max_chunks, float2* ss, f16* y, bool split, hipStream_t s, bool bf) {
  SVC_REQUIRE(C % 8 == 0 && T > 0 && B > 0, "groupnorm: B=%d T=%d C=%d", B, T, C);
  const int chunks = std::max(1, std::min(max_chunks, cdiv(T, 256)));
  const int chunk = cdiv(T, chunks);
  const int nck = cdiv(T, chunk);
  const int tok = prof_begin("groupnorm_gelu", 0.0, (double)B * T * C * (4 + 4 + 2), s);
  hipLaunchKernelGGL(colstats_kernel, dim3(nck, B), dim3(256), 0, s, x, T, C, chunk, part);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(cdiv(C, 256), B), dim3(256), 0, s, part, nck, T, C, gamma, beta, 1e-5f,
                     ss);
  const int64_t nvec = (int64_t)B * T * C / 8;
  if (split)
    hipLaunchKernelGGL(gn_gelu_apply_kernel<true>, dim3((unsigned)cdiv64(nvec, 256)), dim3(256), 0, s, x, ss, y,
                       (int64_t)T, C, nvec, bf);
  else
    hipLaunchKernelGGL(gn_gelu_apply_kernel<false>, dim3((unsigned)cdiv64(nvec, 256)), dim3(256), 0, s, x, ss, y,
                       (int64_t)T, C, nvec, bf);
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// One wave per row (D <= 1024, multiple of 64): y32 and y16 both written (y32 may alias x); SPLIT: y16 rows are
// the split-fp16 operand [hi | lo | hi] of 3 D columns.
template <bool SPLIT>
__global__ __launch_bounds__(256) void layernorm_dual_kernel(const float* x, const float* __restrict__ gam,
                                                             const float* __restrict__ bet, float* y32,
                                                             f16* __restrict__ y16, int rows, int D, bool bf) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * D;
  float v[16];
  const int per = D / 64;
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
      const float d = v[i] - mean;
      ss += d * d;
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  const float rstd = 1.0f / sqrtf(ss / (float)D + 1e-5f);
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < per) {
      const int c = i * 64 + lane;
      const float o = (v[i] - mean) * rstd * gam[c] + bet[c];
      y32[(int64_t)row * D + c] = o;
      const f16 hi = enc16(o, bf);
      if constexpr (SPLIT) {
        f16* yr = y16 + (int64_t)row * 3 * D;
        yr[c] = hi;
        yr[D + c] = enc16_lo(o - dec16(hi, bf), bf);
        yr[2 * D + c] = hi;
      } else {
        y16[(int64_t)row * D + c] = hi;
      }
    }
}

int layernorm_dual(const float* x, const float* g, const float* b, float* y32, f16* y16, int rows, int D, bool split,
                   hipStream_t s, bool bf) {
  SVC_REQUIRE(D % 64 == 0 && D <= 1024, "layernorm_dual: D=%d", D);
  if (split)
    hipLaunchKernelGGL(layernorm_dual_kernel<true>, dim3(cdiv(rows, 4)), dim3(256), 0, s, x, g, b, y32, y16, rows, D,
                       bf);
  else
    hipLaunchKernelGGL(layernorm_dual_kernel<false>, dim3(cdiv(rows, 4)), dim3(256), 0, s, x, g, b, y32, y16, rows, D,
                       bf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
