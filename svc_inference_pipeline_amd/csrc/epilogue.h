// Shared GEMM epilogue (conv_gemm3 / conv_gemm4 LDS-staged forms): applied to a BM x BNP pass of the f32 C tile staged
// in LDS (row stride LDC floats), on 4-column chunks with 16-byte vector loads/stores (coalesced rows).
//   generic : v = act(acc + bias) (*col_scale) (+add_t) (+add_row) ((acc32 + v) / acc_div) -> out32 / out16
//   COND    : acc + bias + emb_m[idx_m] + emb_l[idx_l] + emb_s[singer] (modules/encoder.py conditioner sum)
//   GATE    : sigmoid(gate + cp) * tanh(filter + cp) (modules/diffsvc.py:217-227), paired columns: packed
//             column n (n & 32 == 0) holds channel (n >> 6) * 32 + (n & 31) of the gate half and n + 32
//             the same channel of the filter half.
#pragma once
#include "common.h"

namespace svc {

template <int BM, int BNP, int LDC, int NT, bool PAIR, bool BF = false>
__device__ __forceinline__ void epilogue_pass(const float* Cs, int m0, int nbase, int M, const ConvGemmArgs& a,
                                              const EpiArgs& e, int tid) {
  using O = Op16<BF>;
  if constexpr (!PAIR) {
    constexpr int CPR = BNP / 4;
    for (int idx = tid; idx < BM * CPR; idx += NT) {
      const int row = idx / CPR, cc = idx - row * CPR;
      const int m = m0 + row, n = nbase + 4 * cc;
      if (m >= M || n >= a.N) continue;
      const int b = m / a.T_out, t = m - b * a.T_out;
      const int64_t orow = (int64_t)b * e.T_ostore + (int64_t)t * e.ostride + e.ophase;
      float4 v = *reinterpret_cast<const float4*>(Cs + row * LDC + 4 * cc);  // pass-local columns
      const float4 bi = *reinterpret_cast<const float4*>(e.bias + n);
      v.x += bi.x; v.y += bi.y; v.z += bi.z; v.w += bi.w;
      if (e.kind == EPI_COND) {
        const float4 em = *reinterpret_cast<const float4*>(e.emb_m + (int64_t)e.idx_m[m] * e.ld_emb + n);
        const float4 el = *reinterpret_cast<const float4*>(e.emb_l + (int64_t)e.idx_l[m] * e.ld_emb + n);
        const float4 es = *reinterpret_cast<const float4*>(e.emb_s + (int64_t)e.singer[b] * e.ld_emb + n);
        v.x = ((v.x + em.x) + el.x) + es.x;
        v.y = ((v.y + em.y) + el.y) + es.y;
        v.z = ((v.z + em.z) + el.z) + es.z;
        v.w = ((v.w + em.w) + el.w) + es.w;
      } else {
        if (e.act == ACT_GELU) {
          v.x = gelu_erf(v.x); v.y = gelu_erf(v.y); v.z = gelu_erf(v.z); v.w = gelu_erf(v.w);
        } else if (e.act == ACT_RELU) {
          v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
        }
        if (n < e.scale_cols) {
          const float cs = n < e.scale_cols2 ? e.col_scale2 : e.col_scale;
          v.x *= cs; v.y *= cs; v.z *= cs; v.w *= cs;
        }
        if (e.add_t) {
          const float4 at = *reinterpret_cast<const float4*>(e.add_t + (int64_t)t * e.ld_add_t + n);
          v.x += at.x; v.y += at.y; v.z += at.z; v.w += at.w;
        }
        if (e.add_row) {
          const float4 ar = *reinterpret_cast<const float4*>(e.add_row + orow * e.ld_add_row + n);
          v.x += ar.x; v.y += ar.y; v.z += ar.z; v.w += ar.w;
        }
        if (e.acc32 || e.acc16_hi) {
          float4 ac;
          if (e.acc32) {
            ac = *reinterpret_cast<const float4*>(e.acc32 + orow * e.ld_acc + n);
          } else {  // split residual: (hi + lo) - the add16 it was stored with
            union { uint2 u; f16 h[4]; } hi, lo;
            hi.u = *reinterpret_cast<const uint2*>(e.acc16_hi + orow * e.ld_acc + n);
            lo.u = *reinterpret_cast<const uint2*>(e.acc16_lo + orow * e.ld_acc + n);
            const float4 sb = *reinterpret_cast<const float4*>(e.acc_sub + n);
            ac.x = (O::dec(hi.h[0]) + O::dec(lo.h[0])) - sb.x; ac.y = (O::dec(hi.h[1]) + O::dec(lo.h[1])) - sb.y;
            ac.z = (O::dec(hi.h[2]) + O::dec(lo.h[2])) - sb.z; ac.w = (O::dec(hi.h[3]) + O::dec(lo.h[3])) - sb.w;
          }
          v.x = ac.x + v.x; v.y = ac.y + v.y; v.z = ac.z + v.z; v.w = ac.w + v.w;
          if (e.acc_div != 1.0f) {
            v.x = v.x / e.acc_div; v.y = v.y / e.acc_div; v.z = v.z / e.acc_div; v.w = v.w / e.acc_div;
          }
        }
      }
      if (e.out32) *reinterpret_cast<float4*>(e.out32 + orow * e.ld32 + n) = v;
      if (e.out16) {
        float4 w = v;
        if (e.add16) {
          const float4 ad = *reinterpret_cast<const float4*>(e.add16 + n);
          w.x += ad.x; w.y += ad.y; w.z += ad.z; w.w += ad.w;
        }
        union { uint2 u; f16 h[4]; } pk;
        pk.h[0] = O::enc(w.x); pk.h[1] = O::enc(w.y); pk.h[2] = O::enc(w.z); pk.h[3] = O::enc(w.w);
        const int64_t ocol = e.col_block ? (int64_t)(n / e.col_block) * e.col_block_stride + n % e.col_block : n;
        *reinterpret_cast<uint2*>(e.out16 + orow * e.ld16 + ocol) = pk.u;
        if (e.lo16) {
          union { uint2 u; f16 h[4]; } lo;
          lo.h[0] = O::enc_lo(w.x - O::dec(pk.h[0])); lo.h[1] = O::enc_lo(w.y - O::dec(pk.h[1]));
          lo.h[2] = O::enc_lo(w.z - O::dec(pk.h[2])); lo.h[3] = O::enc_lo(w.w - O::dec(pk.h[3]));
          *reinterpret_cast<uint2*>(e.lo16 + orow * e.ld16 + n) = lo.u;
        }
        if (e.split16) {
          union { uint2 u; f16 h[4]; } lo;
          lo.h[0] = O::enc_lo(w.x - O::dec(pk.h[0])); lo.h[1] = O::enc_lo(w.y - O::dec(pk.h[1]));
          lo.h[2] = O::enc_lo(w.z - O::dec(pk.h[2])); lo.h[3] = O::enc_lo(w.w - O::dec(pk.h[3]));
          *reinterpret_cast<uint2*>(e.out16 + orow * e.ld16 + e.split16 + n) = lo.u;
          *reinterpret_cast<uint2*>(e.out16 + orow * e.ld16 + 2 * e.split16 + n) = pk.u;
        }
      }
    }
  } else {
    // pairs: chunk = 4 first-half columns n..n+3 and their partners n+32..n+35 -> channels ch..ch+3
    constexpr int CPR = BNP / 8;
    for (int idx = tid; idx < BM * CPR; idx += NT) {
      const int row = idx / CPR, cc = idx - row * CPR;
      const int m = m0 + row;
      const int nl = (cc >> 3) * 64 + 4 * (cc & 7);  // pass-local packed column of the first-half element
      const int n = nbase + nl;
      if (m >= M || n >= a.N) continue;
      const int ch = (n >> 6) * 32 + (n & 31);
      float4 v1 = *reinterpret_cast<const float4*>(Cs + row * LDC + nl);
      float4 v2 = *reinterpret_cast<const float4*>(Cs + row * LDC + nl + 32);
      const float4 b1 = *reinterpret_cast<const float4*>(e.bias + n);
      const float4 b2 = *reinterpret_cast<const float4*>(e.bias + n + 32);
      v1.x += b1.x; v1.y += b1.y; v1.z += b1.z; v1.w += b1.w;
      v2.x += b2.x; v2.y += b2.y; v2.z += b2.z; v2.w += b2.w;
      union { uint2 u; f16 h[4]; } pk, c1, c2;  // EPI_GATE
      c1.u = *reinterpret_cast<const uint2*>(e.cp + (int64_t)m * e.ld_cp + n);
      c2.u = *reinterpret_cast<const uint2*>(e.cp + (int64_t)m * e.ld_cp + n + 32);
      pk.h[0] = O::enc_lo(gate_act(v1.x + O::dec(c1.h[0]), v2.x + O::dec(c2.h[0])));
      pk.h[1] = O::enc_lo(gate_act(v1.y + O::dec(c1.h[1]), v2.y + O::dec(c2.h[1])));
      pk.h[2] = O::enc_lo(gate_act(v1.z + O::dec(c1.h[2]), v2.z + O::dec(c2.h[2])));
      pk.h[3] = O::enc_lo(gate_act(v1.w + O::dec(c1.h[3]), v2.w + O::dec(c2.h[3])));
      *reinterpret_cast<uint2*>(e.y16 + (int64_t)m * e.ldy16 + ch) = pk.u;
    }
  }
}

}  // namespace svc
