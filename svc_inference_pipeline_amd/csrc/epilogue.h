// Shared GEMM epilogue (conv_gemm2 / conv_gemm3): applied to a BM x BNP pass of the f32 C tile staged
// in LDS (row stride LDC floats), on 4-column chunks with 16-byte vector loads/stores (coalesced rows).
//   generic : v = act(acc + bias) (*col_scale) (+add_t) (+add_row) ((acc32 + v) / acc_div) -> out32 / out16
//   COND    : acc + bias + emb_m[idx_m] + emb_l[idx_l] + emb_s[singer] (modules/encoder.py conditioner sum)
//   GATE    : sigmoid(gate + cp) * tanh(filter + cp) (modules/diffsvc.py:217-227), paired columns: packed
//             column n (n & 32 == 0) holds channel (n >> 6) * 32 + (n & 31) of the gate half and n + 32
//             the same channel of the filter half.
#pragma once
#include "common.h"

namespace svc {

// Each thread handles its chunks in groups of EPI_U: every global operand of the group is loaded into
// registers first, then the group is computed and stored. (One load/compute/store chunk at a time would
// serialise on memory latency: out32 may alias acc32 / add_row, and y16 may alias cp, so the compiler
// cannot hoist the next chunk's loads above the previous chunk's stores.)
constexpr int EPI_U = 4;

__device__ __forceinline__ void f4add(float4& v, const float4& a) {
  v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
}

template <int BM, int BNP, int LDC, int NT, bool PAIR>
__device__ __forceinline__ void epilogue_pass(const float* Cs, int m0, int nbase, int M, const ConvGemmArgs& a,
                                              const EpiArgs& e, int tid) {
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (!PAIR) {
    constexpr int CPR = BNP / 4, TOTAL = BM * CPR;
    for (int g0 = 0; g0 < TOTAL; g0 += NT * EPI_U) {
      float4 v[EPI_U], o1[EPI_U], o2[EPI_U], o3[EPI_U];
      int64_t orow[EPI_U];
      int nn[EPI_U];
      bool ok[EPI_U];
#pragma unroll
      for (int u = 0; u < EPI_U; ++u) {
        const int idx = g0 + u * NT + tid;
        const int row = idx / CPR, cc = idx - row * CPR;
        const int m = m0 + row, n = nbase + 4 * cc;
        ok[u] = idx < TOTAL && m < M && n < a.N;
        nn[u] = n;
        v[u] = o1[u] = o2[u] = o3[u] = z4;
        orow[u] = 0;
        if (!ok[u]) continue;
        const int b = m / a.T_out, t = m - b * a.T_out;
        orow[u] = (int64_t)b * e.T_ostore + (int64_t)t * e.ostride + e.ophase;
        v[u] = *reinterpret_cast<const float4*>(Cs + row * LDC + 4 * cc);  // pass-local columns
        f4add(v[u], *reinterpret_cast<const float4*>(e.bias + n));
        if (e.kind == EPI_COND) {
          o1[u] = *reinterpret_cast<const float4*>(e.emb_m + (int64_t)e.idx_m[m] * e.ld_emb + n);
          o2[u] = *reinterpret_cast<const float4*>(e.emb_l + (int64_t)e.idx_l[m] * e.ld_emb + n);
          o3[u] = *reinterpret_cast<const float4*>(e.emb_s + (int64_t)e.singer[b] * e.ld_emb + n);
        } else {
          if (e.add_t) o1[u] = *reinterpret_cast<const float4*>(e.add_t + (int64_t)t * e.ld_add_t + n);
          if (e.add_row) o2[u] = *reinterpret_cast<const float4*>(e.add_row + orow[u] * e.ld_add_row + n);
          if (e.acc32) o3[u] = *reinterpret_cast<const float4*>(e.acc32 + orow[u] * e.ld_acc + n);
        }
      }
#pragma unroll
      for (int u = 0; u < EPI_U; ++u) {
        if (!ok[u]) continue;
        const int n = nn[u];
        float4 w = v[u];
        if (e.kind == EPI_COND) {
          w.x = ((w.x + o1[u].x) + o2[u].x) + o3[u].x;
          w.y = ((w.y + o1[u].y) + o2[u].y) + o3[u].y;
          w.z = ((w.z + o1[u].z) + o2[u].z) + o3[u].z;
          w.w = ((w.w + o1[u].w) + o2[u].w) + o3[u].w;
        } else {
          if (e.act == ACT_GELU) {
            w.x = gelu_erf(w.x); w.y = gelu_erf(w.y); w.z = gelu_erf(w.z); w.w = gelu_erf(w.w);
          } else if (e.act == ACT_RELU) {
            w.x = fmaxf(w.x, 0.f); w.y = fmaxf(w.y, 0.f); w.z = fmaxf(w.z, 0.f); w.w = fmaxf(w.w, 0.f);
          }
          if (n < e.scale_cols) {
            w.x *= e.col_scale; w.y *= e.col_scale; w.z *= e.col_scale; w.w *= e.col_scale;
          }
          if (e.add_t) f4add(w, o1[u]);
          if (e.add_row) f4add(w, o2[u]);
          if (e.acc32) {
            w.x = o3[u].x + w.x; w.y = o3[u].y + w.y; w.z = o3[u].z + w.z; w.w = o3[u].w + w.w;
            if (e.acc_div != 1.0f) {
              w.x = w.x / e.acc_div; w.y = w.y / e.acc_div; w.z = w.z / e.acc_div; w.w = w.w / e.acc_div;
            }
          }
        }
        if (e.out32) *reinterpret_cast<float4*>(e.out32 + orow[u] * e.ld32 + n) = w;
        if (e.out16) {
          if (e.add16) f4add(w, *reinterpret_cast<const float4*>(e.add16 + n));
          union { uint2 u2; f16 h[4]; } pk;
          pk.h[0] = f16_sat(w.x); pk.h[1] = f16_sat(w.y); pk.h[2] = f16_sat(w.z); pk.h[3] = f16_sat(w.w);
          *reinterpret_cast<uint2*>(e.out16 + orow[u] * e.ld16 + n) = pk.u2;
        }
      }
    }
  } else {
    // pairs: chunk = 4 first-half columns n..n+3 and their partners n+32..n+35 -> channels ch..ch+3
    constexpr int CPR = BNP / 8, TOTAL = BM * CPR;
    for (int g0 = 0; g0 < TOTAL; g0 += NT * EPI_U) {
      float4 v1[EPI_U], v2[EPI_U];
      uint2 c1[EPI_U], c2[EPI_U];
      int mm[EPI_U], nn[EPI_U];
      bool ok[EPI_U];
#pragma unroll
      for (int u = 0; u < EPI_U; ++u) {
        const int idx = g0 + u * NT + tid;
        const int row = idx / CPR, cc = idx - row * CPR;
        const int m = m0 + row;
        const int nl = (cc >> 3) * 64 + 4 * (cc & 7);  // pass-local packed column of the first-half element
        const int n = nbase + nl;
        ok[u] = idx < TOTAL && m < M && n < a.N;
        mm[u] = m;
        nn[u] = n;
        v1[u] = v2[u] = z4;
        c1[u] = c2[u] = make_uint2(0u, 0u);
        if (!ok[u]) continue;
        v1[u] = *reinterpret_cast<const float4*>(Cs + row * LDC + nl);
        v2[u] = *reinterpret_cast<const float4*>(Cs + row * LDC + nl + 32);
        f4add(v1[u], *reinterpret_cast<const float4*>(e.bias + n));
        f4add(v2[u], *reinterpret_cast<const float4*>(e.bias + n + 32));
        c1[u] = *reinterpret_cast<const uint2*>(e.cp + (int64_t)m * e.ld_cp + n);
        c2[u] = *reinterpret_cast<const uint2*>(e.cp + (int64_t)m * e.ld_cp + n + 32);
      }
#pragma unroll
      for (int u = 0; u < EPI_U; ++u) {
        if (!ok[u]) continue;
        union { uint2 u2; f16 h[4]; } pk, q1, q2;  // EPI_GATE
        q1.u2 = c1[u];
        q2.u2 = c2[u];
        pk.h[0] = f16_sat(sigmoidf_(v1[u].x + (float)q1.h[0]) * tanhf(v2[u].x + (float)q2.h[0]));
        pk.h[1] = f16_sat(sigmoidf_(v1[u].y + (float)q1.h[1]) * tanhf(v2[u].y + (float)q2.h[1]));
        pk.h[2] = f16_sat(sigmoidf_(v1[u].z + (float)q1.h[2]) * tanhf(v2[u].z + (float)q2.h[2]));
        pk.h[3] = f16_sat(sigmoidf_(v1[u].w + (float)q1.h[3]) * tanhf(v2[u].w + (float)q2.h[3]));
        const int n = nn[u];
        const int ch = (n >> 6) * 32 + (n & 31);
        *reinterpret_cast<uint2*>(e.y16 + (int64_t)mm[u] * e.ldy16 + ch) = pk.u2;
      }
    }
  }
}

}  // namespace svc
