// Whisper encoder self-attention (non-causal, head dim 64) as a flash-style MFMA kernel for gfx950.
// Restates MultiHeadAttention.qkv_attention (utils/whisper_extractor/model.py:88-101): q and k are
// pre-scaled by dh^-1/4 in the QKV GEMM epilogue, softmax in f32, P rounded to f16 for P.V.
//
// Layout: qkv f16 [B*L][3*D] (q | k | v, head h at columns h*64..h*64+63 of each third),
// out f16 [B*L][D]. One workgroup = 4 waves = 128 queries of one (utterance, head); each wave owns
// 32 queries (two 16-column fragments). Scores are computed TRANSPOSED (S^T = K Q^T) so that a
// lane's accumulator column is one query: the row max / row sum need only two cross-lane shuffles
// (xor 16, xor 32), and the f32 accumulator, converted to f16, is directly the B operand of
// O^T = V^T P^T (k-order permuted; V^T staged in LDS with the same permutation read as 2 x b64).
#include "common.h"

namespace svc {

constexpr int ATT_QT = 128;   // queries per workgroup
constexpr int ATT_KT = 64;    // keys per tile
constexpr int VT_LD = 68;     // padded row (f16) of the V^T image: conflict-free ds_read_b64

__device__ __forceinline__ int kswz(int row, int kv) { return row * 64 + ((kv ^ ((row >> 1) & 7)) << 3); }

__global__ __launch_bounds__(256, 2) void attention_kernel(const f16* __restrict__ qkv, f16* __restrict__ out, int L,
                                                           int D) {
  // double-buffered K / V^T tiles: tile kt + 1 is loaded into registers while tile kt is multiplied, then written to
  // the other buffer (one barrier per tile)
  __shared__ __align__(16) f16 Ksb[2][ATT_KT * 64];
  __shared__ __align__(16) f16 Vtb[2][64 * VT_LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int qblk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int ld = 3 * D;
  const f16* base = qkv + (int64_t)b * L * ld;
  const int qw0 = qblk * ATT_QT + wave * 32;  // first query of this wave
  const int g = lane >> 4, c16 = lane & 15;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[q = qf*16 + c16][d = ks*32 + 8g + 0..7]
  half8 qf[2][2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    int q = qw0 + f * 16 + c16;
    int qc = q < L ? q : L - 1;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[f][ks] = *reinterpret_cast<const half8*>(base + (int64_t)qc * ld + h * 64 + ks * 32 + 8 * g);
  }

  floatx4 o[4][2];  // O^T[d = df*16 + 4g + r][q = qf*16 + c16]
#pragma unroll
  for (int df = 0; df < 4; ++df)
#pragma unroll
    for (int f = 0; f < 2; ++f) o[df][f] = (floatx4){0.f, 0.f, 0.f, 0.f};
  float mrun[2] = {-INFINITY, -INFINITY}, lrun[2] = {0.f, 0.f};
  const float LOG2E = 1.4426950408889634f;

  const int ntiles = (L + ATT_KT - 1) / ATT_KT;
  uint4 kreg[2], vreg[2];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + 256 * i;  // 512 vectors of 8 f16
      const int row = v >> 3, kvv = v & 7;
      const int key = kt * ATT_KT + row;
      kreg[i] = vreg[i] = make_uint4(0, 0, 0, 0);
      if (key < L) {
        kreg[i] = *reinterpret_cast<const uint4*>(base + (int64_t)key * ld + D + h * 64 + kvv * 8);
        vreg[i] = *reinterpret_cast<const uint4*>(base + (int64_t)key * ld + 2 * D + h * 64 + kvv * 8);
      }
    }
  };
  auto lstore = [&](int buf) {  // K row-major (swizzled), V transposed
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int v = tid + 256 * i;
      const int row = v >> 3, kvv = v & 7;
      *reinterpret_cast<uint4*>(Ksb[buf] + kswz(row, kvv)) = kreg[i];
      union { uint4 u; f16 e[8]; } vv;
      vv.u = vreg[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) Vtb[buf][(kvv * 8 + j) * VT_LD + row] = vv.e[j];
    }
  };
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int k0 = kt * ATT_KT;
    const f16* Ks = Ksb[kt & 1];
    const f16* Vt = Vtb[kt & 1];
    if (kt + 1 < ntiles) gload(kt + 1);  // lands while this tile is multiplied

    // ---- S^T = K Q^T : s[kf][f][r] = S[q = f*16 + c16][key = kf*16 + 4g + r]
    floatx4 s[4][2];
#pragma unroll
    for (int kf = 0; kf < 4; ++kf) {
#pragma unroll
      for (int f = 0; f < 2; ++f) s[kf][f] = (floatx4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        half8 kfrag = *reinterpret_cast<const half8*>(Ks + kswz(kf * 16 + c16, ks * 4 + g));
#pragma unroll
        for (int f = 0; f < 2; ++f) s[kf][f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kfrag, qf[f][ks], s[kf][f], 0, 0, 0);
      }
    }
    // ---- online softmax per query column
    half8 pb[2][2];  // P^T as B operand: [f][ks'] element j <-> key 32ks' + 4g + (j&3) + 16(j>>2)
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      float mx = -INFINITY;
#pragma unroll
      for (int kf = 0; kf < 4; ++kf)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int key = k0 + kf * 16 + 4 * g + r;
          float v = key < L ? s[kf][f][r] : -INFINITY;
          s[kf][f][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16));
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      const float mnew = fmaxf(mrun[f], mx);
      const float alpha = __builtin_amdgcn_exp2f((mrun[f] - mnew) * LOG2E);  // v_exp_f32 (arguments <= 0)
      mrun[f] = mnew;
      float psum = 0.f;
      float p[4][4];
#pragma unroll
      for (int kf = 0; kf < 4; ++kf)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[kf][r] = __builtin_amdgcn_exp2f((s[kf][f][r] - mnew) * LOG2E);
          psum += p[kf][r];
        }
      lrun[f] = lrun[f] * alpha + psum;
#pragma unroll
      for (int df = 0; df < 4; ++df) o[df][f] *= alpha;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        half8 hv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          hv[j] = (f16)p[2 * ks][j];
          hv[4 + j] = (f16)p[2 * ks + 1][j];
        }
        pb[f][ks] = hv;
      }
    }
    // ---- O^T += V^T P^T
#pragma unroll
    for (int df = 0; df < 4; ++df) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const f16* vrow = Vt + (df * 16 + c16) * VT_LD + ks * 32 + 4 * g;
        union { uint2 u[2]; half8 h; } va;
        va.u[0] = *reinterpret_cast<const uint2*>(vrow);
        va.u[1] = *reinterpret_cast<const uint2*>(vrow + 16);
#pragma unroll
        for (int f = 0; f < 2; ++f) o[df][f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va.h, pb[f][ks], o[df][f], 0, 0, 0);
      }
    }
    if (kt + 1 < ntiles) lstore((kt + 1) & 1);  // that buffer was last read in iteration kt - 1, before its barrier
    __syncthreads();
  }

  // ---- normalise and store: lane holds O[q = f*16 + c16][d = df*16 + 4g + r]
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    float l = lrun[f];
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    const float inv = 1.0f / l;
    const int q = qw0 + f * 16 + c16;
    if (q >= L) continue;
    f16* orow = out + ((int64_t)b * L + q) * D + h * 64;
#pragma unroll
    for (int df = 0; df < 4; ++df) {
      union { uint2 u; f16 e[4]; } pk;
#pragma unroll
      for (int r = 0; r < 4; ++r) pk.e[r] = (f16)(o[df][f][r] * inv);
      *reinterpret_cast<uint2*>(orow + df * 16 + 4 * g) = pk.u;
    }
  }
}

int attention(const f16* qkv, f16* out, int B, int L, int D, hipStream_t s) {
  SVC_REQUIRE(D % 64 == 0 && L > 0 && B > 0, "attention: bad shape B=%d L=%d D=%d", B, L, D);
  dim3 grid((L + ATT_QT - 1) / ATT_QT, D / 64, B);
  const int tok = prof_begin("attention", 4.0 * B * (double)L * L * D, 0.0, s);
  hipLaunchKernelGGL(attention_kernel, grid, dim3(256), 0, s, qkv, out, L, D);
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
