// Whisper encoder self-attention (non-causal, head dim 64) as a flash-style MFMA kernel for gfx950.
// Restates MultiHeadAttention.qkv_attention (utils/whisper_extractor/model.py:88-101): q and k are
// pre-scaled by dh^-1/4 in the QKV GEMM epilogue, q also by log2(e) (ATT_LOG2E), so the scores leave the MFMAs in
// exp2 units; softmax in f32, P rounded to f16 for P.V.
//
// Layout: qkv f16 [B*L][3*D] (q | k | v, head h at columns h*64..h*64+63 of each third),
// out f16 [B*L][D]. One workgroup = 4 waves = 128 queries of one (utterance, head); each wave owns
// 32 queries (two 16-column fragments). Scores are computed TRANSPOSED (S^T = K Q^T) so that a
// lane's accumulator column is one query: the row max / row sum need only two cross-lane shuffles
// (xor 16, xor 32), and the f32 accumulator, converted to f16, is directly the B operand of
// O^T = V^T P^T (k-order permuted). V stays row-major in LDS (one ds_write_b128 per 8 values, as K) and the V^T
// A operand is read with gfx950's transposing ds_read_b64_tr_b16 (a 16-lane group reads 4 keys x 16 head columns and
// each lane receives its column), from an image whose 16-B chunks are XOR-swizzled so those reads are conflict-free.
// Softmax VALU work per score: the score MFMAs accumulate onto -m (the running max as their C operand), so S - m
// comes out of the matrix core and goes straight into v_exp_f32 and an f16 conversion. The row sum l is a fifth P.V
// product against a block of ones (round 3): 4 MFMAs per tile instead of 16 packed f32 adds per lane and a final
// cross-lane reduction. The same tile sums bound every P of their column, so the deferred rescale needs no per-tile max:
// only when some column's tile sum exceeds ATT_PSUM (rare after the first tile) does the running max move (its v_max3
// tree, the cross-lane column max, O / l rescaled, P made again). The first tile sets m exactly; the key mask runs on the
// last tile only. The kernel is VALU-issue bound (round 2 PMC: ~9.6 VALU instructions per MFMA, 0.30 MFMA busy).
#include <type_traits>

#include "common.h"

namespace svc {

constexpr int ATT_QT = 128;   // queries per workgroup
constexpr int ATT_KT = 64;    // keys per tile
constexpr float ATT_PSUM = 16384.0f;  // deferred rescale: a tile's P column sum above this moves the running max

__device__ __forceinline__ int kswz(int row, int kv) { return row * 64 + ((kv ^ ((row >> 1) & 7)) << 3); }
// V image: [key][64 f16] rows, 16-B chunk c of row r stored at chunk c ^ (((r >> 1) & 3) << 1). A transposing read of
// keys r0 + 4g + q (q < 4), head columns 16df + 4p (p < 4) then maps the 32 lanes of a half (g < 2) to distinct
// (r & 1, chunk, 8-B half) = 64 distinct banks; the row-major ds_write_b128 of 8 lanes covers one whole 128-B row.
__device__ __forceinline__ int vswz(int row, int c) { return row * 64 + ((c ^ (((row >> 1) & 3) << 1)) << 3); }

// cross-lane reductions over the lane pairs (l, l ^ 16) and (l, l ^ 32) on the VALU (gfx950 v_permlane16/32_swap: each
// lane ends up holding its own value and its partner's), instead of ds_bpermute round trips through the LDS crossbar
__device__ __forceinline__ float max_xor16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_xor16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float sum_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// max of three as nested fmaxf with single-use inner results, which the backend folds into one v_max3_f32 (inline asm
// here would hide MFMA-result read hazards from the compiler's hazard recognizer)
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

typedef short short4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef _Float16 half4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ half4v lds_tr16(const f16* p) {
  return __builtin_bit_cast(half4v, __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)p));
}

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// BF: q / k / v and the output are bfloat16 (the bf16 operand variant, Op16<true>), P is rounded to bf16
template <bool BF>
__global__ __launch_bounds__(256, 3) void attention_kernel(const f16* __restrict__ qkv, f16* __restrict__ out, int L,
                                                           int D) {
  using O = Op16<BF>;
  // double-buffered K / V^T tiles: tile kt + 1 is loaded into registers while tile kt is multiplied, then written to
  // the other buffer (one barrier per tile)
  __shared__ __align__(16) f16 Ksb[2][ATT_KT * 64];
  __shared__ __align__(16) f16 Vsb[2][ATT_KT * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // 1-D grid, remapped so that consecutive logical workgroups (the query blocks of one utterance and head, which read
  // the same K / V) run on one XCD: K / V are fetched into each XCD's L2 once instead of by all eight
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int nq = (L + ATT_QT - 1) / ATT_QT, H = D / 64;
  const int qblk = wg % nq, h = (wg / nq) % H, b = wg / (nq * H);
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
  // running max m (exp2 units; set exactly by the first tile), its negation as the score MFMAs' C operand, and the
  // lane's share of the row sum
  float mrun[2] = {0.f, 0.f};
  floatx4 negm[2] = {(floatx4){0.f, 0.f, 0.f, 0.f}, (floatx4){0.f, 0.f, 0.f, 0.f}};
  // the row sum l = P . 1 on the matrix core: a 16-row block of ones as V^T's A operand, so every r of ol[f] holds the
  // column's sum over all keys so far (of the rounded P that the P.V MFMAs use; no VALU adds, no final cross-lane sum)
  floatx4 ol[2] = {(floatx4){0.f, 0.f, 0.f, 0.f}, (floatx4){0.f, 0.f, 0.f, 0.f}};
  const half8 ones = BF ? __builtin_bit_cast(half8, (bf16x8){1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f})
                        : (half8){1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f};

  const int ntiles = (L + ATT_KT - 1) / ATT_KT;
  u32x4 kreg[2], vreg[2];  // (a native vector type: the uint4 struct copies were kept in scratch)
  // K / V rows of tile kt: a wave-uniform base (this utterance and head) plus a 32-bit per-lane byte offset, so the
  // loads take the SGPR-base form. Keys past L (last tile only) load the last key's row: their scores are masked to
  // -inf, so P = 0 multiplies a finite V row (no zero fill, no exec-masked branch around the loads).
  const char* kbase = reinterpret_cast<const char*>(base + D + h * 64);
  const char* vbase = reinterpret_cast<const char*>(base + 2 * D + h * 64);
  const int krow = tid >> 3, kvv = tid & 7;  // vectors tid + 256 i: key row krow + 32 i, 16-B column chunk kvv
  // per-lane offsets of the two rows within a tile (loop-invariant); the tile's row base is a wave-uniform add
  uint32_t loff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) loff[i] = (uint32_t)((krow + 32 * i) * ld + kvv * 8) * 2u;
  auto gload = [&](int kt) {
    const int k0 = kt * ATT_KT;
    if (k0 + ATT_KT > L) {  // last tile only (wave-uniform)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int key = min(k0 + krow + 32 * i, L - 1);
        const uint32_t off = (uint32_t)(key * ld + kvv * 8) * 2u;
        kreg[i] = *reinterpret_cast<const u32x4*>(kbase + off);
        vreg[i] = *reinterpret_cast<const u32x4*>(vbase + off);
      }
    } else {
      const char* kb = kbase + (size_t)k0 * ld * 2;
      const char* vb = vbase + (size_t)k0 * ld * 2;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        kreg[i] = *reinterpret_cast<const u32x4*>(kb + loff[i]);
        vreg[i] = *reinterpret_cast<const u32x4*>(vb + loff[i]);
      }
    }
  };
  auto lstore = [&](int buf) {  // K and V row-major (swizzled)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = krow + 32 * i;
      *reinterpret_cast<u32x4*>(Ksb[buf] + kswz(row, kvv)) = kreg[i];
      *reinterpret_cast<u32x4*>(Vsb[buf] + vswz(row, kvv)) = vreg[i];
    }
  };
  // transposing-read lane roles: lane 4q + p of its 16-lane group supplies key row q, head columns 4p .. 4p + 3
  const int trq = c16 >> 2, trp = c16 & 3;
  gload(0);
  lstore(0);
  __syncthreads();
  // one 64-key tile; FIRST (tile 0) sets the running max, TAIL (the last tile) masks the keys past L: both peeled out
  // of the loop, so neither the exact max nor the key compares run on the other tiles
  auto key_tile = [&](int kt, auto first_c, auto tail_c) {
    constexpr bool FIRST = decltype(first_c)::value;
    constexpr bool TAIL = decltype(tail_c)::value;
    const int k0 = kt * ATT_KT;
    const f16* Ks = Ksb[kt & 1];
    const f16* Vs = Vsb[kt & 1];
    if (kt + 1 < ntiles) gload(kt + 1);  // lands while this tile is multiplied

    // ---- S^T - m = K Q^T - m : s[kf][f][r] = S[q = f*16 + c16][key = kf*16 + 4g + r] - m[q]
    floatx4 s[4][2];
#pragma unroll
    for (int kf = 0; kf < 4; ++kf) {
      const half8 k0f = *reinterpret_cast<const half8*>(Ks + kswz(kf * 16 + c16, g));
      const half8 k1f = *reinterpret_cast<const half8*>(Ks + kswz(kf * 16 + c16, 4 + g));
#pragma unroll
      for (int f = 0; f < 2; ++f) s[kf][f] = O::mfma(k1f, qf[f][1], O::mfma(k0f, qf[f][0], negm[f]));
    }
    // ---- online softmax per query column
    const bool tail = TAIL && k0 + ATT_KT > L;  // keys past L only in the last tile (wave-uniform)
    half8 pb[2][2];  // P^T as B operand: [f][ks'] element j <-> key 32ks' + 4g + (j&3) + 16(j>>2)
    // P = 2^(S - m) straight from the accumulators, converted to f16 in packed pairs
    auto make_p = [&](int f) {
      half2v ph[4][2];
#pragma unroll
      for (int kf = 0; kf < 4; ++kf)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          float2v a;
          a.x = __builtin_amdgcn_exp2f(s[kf][f][2 * hh]);
          a.y = __builtin_amdgcn_exp2f(s[kf][f][2 * hh + 1]);
          if constexpr (BF)
            ph[kf][hh] = __builtin_bit_cast(half2v, __builtin_convertvector(a, bf16x2));
          else
            ph[kf][hh] = __builtin_convertvector(a, half2v);
        }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        pb[f][ks] = (half8){ph[2 * ks][0].x, ph[2 * ks][0].y, ph[2 * ks][1].x, ph[2 * ks][1].y,
                            ph[2 * ks + 1][0].x, ph[2 * ks + 1][0].y, ph[2 * ks + 1][1].x, ph[2 * ks + 1][1].y};
    };
    // move column f's running max by its tile max where that grew (all of it on the first tile): the lane's max of
    // its 16 scores as a v_max3_f32 tree, the column's by two lane swaps
    auto move_max = [&](int f, auto first_c) {
      constexpr bool F1 = decltype(first_c)::value;
      const float x0 = max3f(s[0][f][0], s[0][f][1], s[0][f][2]), x1 = max3f(s[0][f][3], s[1][f][0], s[1][f][1]);
      const float x2 = max3f(s[1][f][2], s[1][f][3], s[2][f][0]), x3 = max3f(s[2][f][1], s[2][f][2], s[2][f][3]);
      const float x4 = max3f(s[3][f][0], s[3][f][1], s[3][f][2]);
      const float mx = fmaxf(max3f(x0, x1, x2), max3f(x3, x4, s[3][f][3]));
      const float cm = max_xor32(max_xor16(mx));   // the column's max of S - m over the tile
      const float d = F1 ? cm : fmaxf(cm, 0.f);     // how far m moves (0: this column keeps its max)
      if constexpr (!F1) {
        const float alpha = __builtin_amdgcn_exp2f(-d);  // exactly 1 where d = 0
        ol[f] *= alpha;
#pragma unroll
        for (int df = 0; df < 4; ++df) o[df][f] *= alpha;
      }
      mrun[f] += d;
      negm[f] = (floatx4){-mrun[f], -mrun[f], -mrun[f], -mrun[f]};
#pragma unroll
      for (int kf = 0; kf < 4; ++kf) s[kf][f] -= d;
    };
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      if (TAIL && tail) {
#pragma unroll
        for (int kf = 0; kf < 4; ++kf)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (k0 + kf * 16 + 4 * g + r >= L) s[kf][f][r] = -INFINITY;
      }
    }
    if constexpr (FIRST) {
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        move_max(f, std::true_type{});
        make_p(f);
      }
    } else {
      // deferred rescale (cdna_hip_programming.md T13) without a per-tile max: P is made against the running max, and
      // the tile's column sums (the ones-block MFMAs, needed for l anyway) bound every P of the column. While they stay
      // <= ATT_PSUM (2^14, so no P reaches f16's 65504) the tile is taken as is; otherwise (rare after the first tile)
      // the running max moves and P is made again
#pragma unroll
      for (int f = 0; f < 2; ++f) make_p(f);
      floatx4 ts[2];
#pragma unroll
      for (int f = 0; f < 2; ++f)
        ts[f] = O::mfma(ones, pb[f][1], O::mfma(ones, pb[f][0], (floatx4){0.f, 0.f, 0.f, 0.f}));
      if (__ballot(!(ts[0][0] <= ATT_PSUM && ts[1][0] <= ATT_PSUM))) {
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          move_max(f, std::false_type{});
          make_p(f);
          ts[f] = O::mfma(ones, pb[f][1], O::mfma(ones, pb[f][0], (floatx4){0.f, 0.f, 0.f, 0.f}));
        }
      }
#pragma unroll
      for (int f = 0; f < 2; ++f) ol[f] += ts[f];
    }
    // ---- O^T += V^T P^T
#pragma unroll
    for (int df = 0; df < 4; ++df) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        // A operand V^T[d = 16df + c16][keys 32ks + 4g + 0..3 | + 16]: two transposing reads of 4 keys x 16 columns
        const int r0 = ks * 32 + 4 * g + trq, c = 2 * df + (trp >> 1), e = 4 * (trp & 1);
        const half4v lo = lds_tr16(Vs + vswz(r0, c) + e);
        const half4v hi = lds_tr16(Vs + vswz(r0 + 16, c) + e);
        const half8 va = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int f = 0; f < 2; ++f) o[df][f] = O::mfma(va, pb[f][ks], o[df][f]);
      }
    }
    if constexpr (FIRST) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int f = 0; f < 2; ++f) ol[f] = O::mfma(ones, pb[f][ks], ol[f]);
    }
    if (kt + 1 < ntiles) lstore((kt + 1) & 1);  // that buffer was last read in iteration kt - 1, before its barrier
    __syncthreads();
  };
  if (ntiles == 1) {
    key_tile(0, std::true_type{}, std::true_type{});
  } else {
    key_tile(0, std::true_type{}, std::false_type{});
    for (int kt = 1; kt + 1 < ntiles; ++kt) key_tile(kt, std::false_type{}, std::false_type{});
    key_tile(ntiles - 1, std::false_type{}, std::true_type{});
  }

  // ---- normalise and store: lane holds O[q = f*16 + c16][d = df*16 + 4g + r]
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const float inv = 1.0f / ol[f][0];
    const int q = qw0 + f * 16 + c16;
    if (q >= L) continue;
    f16* orow = out + ((int64_t)b * L + q) * D + h * 64;
#pragma unroll
    for (int df = 0; df < 4; ++df) {
      union { uint2 u; f16 e[4]; } pk;
#pragma unroll
      for (int r = 0; r < 4; ++r) pk.e[r] = O::enc_lo(o[df][f][r] * inv);
      *reinterpret_cast<uint2*>(orow + df * 16 + 4 * g) = pk.u;
    }
  }
}

int attention(const f16* qkv, f16* out, int B, int L, int D, hipStream_t s, bool bf16) {
  SVC_REQUIRE(D % 64 == 0 && L > 0 && B > 0, "attention: bad shape B=%d L=%d D=%d", B, L, D);
  const int64_t nwg = (int64_t)((L + ATT_QT - 1) / ATT_QT) * (D / 64) * B;
  SVC_REQUIRE(nwg < (1ll << 31), "attention: grid");
  dim3 grid((unsigned)nwg);
  const int tok = prof_begin("attention", 4.0 * B * (double)L * L * D, 0.0, s);
  if (bf16)
    hipLaunchKernelGGL(attention_kernel<true>, grid, dim3(256), 0, s, qkv, out, L, D);
  else
    hipLaunchKernelGGL(attention_kernel<false>, grid, dim3(256), 0, s, qkv, out, L, D);
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
