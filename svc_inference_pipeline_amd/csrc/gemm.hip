// Implicit-GEMM Conv1d / ConvTranspose1d-phase / Linear on gfx950 MFMA (v_mfma_f32_16x16x32_f16).
//
// One kernel family serves every GEMM-shaped op of the SVC path (SURVEY.md §2.2 K5,K7,K10-K15,
// K19,K20,K22): the A operand is the time-major f16 activation tensor read through a per-tap row
// shift (zero padding per utterance), the B operand is the weight packed [N][taps*Cp] f16, the
// accumulator is f32, and a runtime-selected epilogue fuses bias / GELU / ReLU / positional add /
// residual add / conditioner embedding sum (the paired DiffSVC gate runs in gemm2.hip).
//
// Tiling: 256 threads = 4 waves (2x2), tile BM x BN x 64, register-staged global->LDS prefetch of
// tile k+1 overlapping the MFMAs of tile k, LDS double buffer, one barrier per K-tile. LDS rows are
// 128 B ([row][64] f16) XOR-swizzled on 16-B chunks with (row>>1)&7 so ds_read_b128 fragment reads
// (16 distinct rows per lane group) and ds_write_b128 stores are conflict-free.
// Block->tile mapping is XCD-aware: blocks sharing an A row-panel land on one XCD (shared L2).
#include "common.h"

namespace svc {

template <int BM, int BN>
struct TileCfg {
  static constexpr int FM = BM / 32;  // 16-row fragments per wave (2 waves along M)
  static constexpr int FN = BN / 32;  // 16-col fragments per wave (2 waves along N)
  static constexpr int AV = BM / 32;  // 16-B vectors per thread for the A tile (BM*64/8/256)
  static constexpr int BV = BN / 32;
  static constexpr int LDS_A = BM * 64;  // f16 elements per buffer
  static constexpr int LDS_B = BN * 64;
};

__device__ __forceinline__ int swz(int row, int kv) { return row * 64 + ((kv ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ float act_apply(int act, float v) {
  if (act == ACT_GELU) return gelu_erf(v);
  if (act == ACT_RELU) return fmaxf(v, 0.0f);
  return v;
}

template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void conv_gemm_kernel(ConvGemmArgs a, EpiArgs e) {
  using CF = TileCfg<BM, BN>;
  extern __shared__ __align__(16) f16 smem[];
  f16* As = smem;                    // [2][BM*64]
  f16* Bs = smem + 2 * CF::LDS_A;    // [2][BN*64]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // ---- XCD-aware tile mapping (bijective for any grid size)
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int tile_n = wgid % a.ntiles_n;
  const int tile_m = wgid / a.ntiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int M = a.B * a.T_out;

  // ---- per-thread A rows (fixed over the K loop)
  const int kv = tid & 7;
  int a_base[CF::AV], a_tt[CF::AV], a_tin[CF::AV];
#pragma unroll
  for (int i = 0; i < CF::AV; ++i) {
    int rr = (tid >> 3) + 32 * i;
    int m = m0 + rr;
    if (m < M) {
      int b = m / a.T_out;
      int t = m - b * a.T_out;
      a_base[i] = b * a.T_in;
      a_tt[i] = t * a.istride;
      a_tin[i] = valid_in_rows(a, b);
    } else {
      a_base[i] = 0;
      a_tt[i] = -(1 << 29);  // never valid
      a_tin[i] = 0;
    }
  }

  uint4 ra[CF::AV], rb[CF::BV];
  auto load_tiles = [&](int kt) {
    const int kg = kt * 64 + kv * 8;
    const int tap = kg / a.Cp;
    const int c = kg - tap * a.Cp;
    const int off = tap * a.tap_mul + a.tap_add;
    const bool kin = kg < a.K;
#pragma unroll
    for (int i = 0; i < CF::AV; ++i) {
      int st = a_tt[i] + off;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (kin && st >= 0 && st < a_tin[i]) {
        const f16* p = a.X + (int64_t)(a_base[i] + st) * a.ldx + c;
        if (c + 8 <= a.Cvalid) {
          v = *reinterpret_cast<const uint4*>(p);
        } else {
          union { uint4 u; f16 h[8]; } tmp;
#pragma unroll
          for (int j = 0; j < 8; ++j) tmp.h[j] = (c + j < a.Cvalid) ? p[j] : (f16)0.0f;
          v = tmp.u;
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < CF::BV; ++i) {
      int rr = (tid >> 3) + 32 * i;
      const f16* p = a.W + (int64_t)(n0 + rr) * a.Kpad + kt * 64 + kv * 8;
      rb[i] = *reinterpret_cast<const uint4*>(p);
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < CF::AV; ++i) {
      int rr = (tid >> 3) + 32 * i;
      *reinterpret_cast<uint4*>(As + buf * CF::LDS_A + swz(rr, kv)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < CF::BV; ++i) {
      int rr = (tid >> 3) + 32 * i;
      *reinterpret_cast<uint4*>(Bs + buf * CF::LDS_B + swz(rr, kv)) = rb[i];
    }
  };

  floatx4 acc[CF::FM][CF::FN];
#pragma unroll
  for (int i = 0; i < CF::FM; ++i)
#pragma unroll
    for (int j = 0; j < CF::FN; ++j) acc[i][j] = (floatx4){0.f, 0.f, 0.f, 0.f};

  const int nk = a.Kpad / 64;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kt + 1);
    const f16* Ab = As + cur * CF::LDS_A;
    const f16* Bb = Bs + cur * CF::LDS_B;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      half8 af[CF::FM], bf[CF::FN];
      const int kvr = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < CF::FM; ++i) {
        int row = wm * (BM / 2) + i * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const half8*>(Ab + swz(row, kvr));
      }
#pragma unroll
      for (int j = 0; j < CF::FN; ++j) {
        int row = wn * (BN / 2) + j * 16 + (lane & 15);
        bf[j] = *reinterpret_cast<const half8*>(Bb + swz(row, kvr));
      }
#pragma unroll
      for (int i = 0; i < CF::FM; ++i)
#pragma unroll
        for (int j = 0; j < CF::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  // acc[i][j][r] = C[m0 + wm*BM/2 + i*16 + (lane>>4)*4 + r][n0 + wn*BN/2 + j*16 + (lane&15)]
  const int mrow0 = m0 + wm * (BM / 2) + (lane >> 4) * 4;
  const int ncol0 = n0 + wn * (BN / 2) + (lane & 15);
#pragma unroll
  for (int i = 0; i < CF::FM; ++i) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int m = mrow0 + i * 16 + rr;
      if (m >= M) continue;
      const int b = m / a.T_out;
      const int t = m - b * a.T_out;
      const int64_t orow = (int64_t)b * e.T_ostore + (int64_t)t * e.ostride + e.ophase;
#pragma unroll
      for (int j = 0; j < CF::FN; ++j) {
        const int n = ncol0 + j * 16;
        if (n >= a.N) continue;
        float v = acc[i][j][rr];
        if (e.kind == EPI_COND) {
          v = v + e.bias[n];
          v = v + e.emb_m[(int64_t)e.idx_m[m] * e.ld_emb + n];
          v = v + e.emb_l[(int64_t)e.idx_l[m] * e.ld_emb + n];
          v = v + e.emb_s[(int64_t)e.singer[b] * e.ld_emb + n];
          e.out32[orow * e.ld32 + n] = v;
          if (e.out16) e.out16[orow * e.ld16 + n] = f16_sat(v);
          continue;
        }
        if (e.bias) v += e.bias[n];
        v = act_apply(e.act, v);
        if (n < e.scale_cols) v *= e.col_scale;
        if (e.add_t) v += e.add_t[(int64_t)t * e.ld_add_t + n];
        if (e.add_row) v += e.add_row[orow * e.ld_add_row + n];
        if (e.acc32 || e.acc16_hi) {
          const float ac = e.acc32 ? e.acc32[orow * e.ld_acc + n]
                                   : ((float)e.acc16_hi[orow * e.ld_acc + n] + (float)e.acc16_lo[orow * e.ld_acc + n]) -
                                         e.acc_sub[n];
          v = ac + v;
          if (e.acc_div != 1.0f) v = v / e.acc_div;
        }
        if (e.out32) e.out32[orow * e.ld32 + n] = v;
        if (e.out16) {
          const float w = e.add16 ? v + e.add16[n] : v;
          const f16 hi = f16_sat(w);
          e.out16[orow * e.ld16 + n] = hi;
          if (e.lo16) e.lo16[orow * e.ld16 + n] = (f16)(w - (float)hi);
          if (e.split16) {
            e.out16[orow * e.ld16 + e.split16 + n] = (f16)(w - (float)hi);
            e.out16[orow * e.ld16 + 2 * e.split16 + n] = hi;
          }
        }
      }
    }
  }
}

template <int BM, int BN>
static int launch(const ConvGemmArgs& a0, const EpiArgs& e, hipStream_t s) {
  using CF = TileCfg<BM, BN>;
  ConvGemmArgs a = a0;
  const int M = a.B * a.T_out;
  const int mt = cdiv(M, BM);
  a.ntiles_n = cdiv(a.N, BN);
  const size_t lds = (size_t)2 * (CF::LDS_A + CF::LDS_B) * sizeof(f16);
  const int64_t grid = (int64_t)mt * a.ntiles_n;
  SVC_REQUIRE(grid > 0 && grid < (1ll << 31), "conv_gemm: bad grid %lld", (long long)grid);
  static bool attr_set = false;  // > 64 KiB of dynamic LDS must be opted into once per instantiation
  if (!attr_set) {
    SVC_HIP_CHECK(hipFuncSetAttribute((const void*)conv_gemm_kernel<BM, BN>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_set = true;
  }
  const double kreal = (double)(a.K / a.Cp) * a.Cvalid;
  const int tok = prof_begin((BN == 32 ? "conv_gemm<256,32>" : (BN == 64 ? "conv_gemm<256,64>" : "conv_gemm<128,128>")),
                             2.0 * M * (double)a.N * kreal, 0.0, s);
  hipLaunchKernelGGL((conv_gemm_kernel<BM, BN>), dim3((unsigned)grid), dim3(256), lds, s, a, e);
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

int conv_gemm(const ConvGemmArgs& a, const EpiArgs& e, hipStream_t s) {
  SVC_REQUIRE(a.X && a.W, "conv_gemm: null operand");
  SVC_REQUIRE(a.Cp % 8 == 0 && a.ldx % 8 == 0 && a.Kpad % 64 == 0 && a.K <= a.Kpad && a.Cvalid <= a.Cp,
              "conv_gemm: layout (Cp=%d ldx=%d K=%d Kpad=%d)", a.Cp, a.ldx, a.K, a.Kpad);
  SVC_REQUIRE(a.Cp <= a.ldx || a.Cvalid <= a.ldx, "conv_gemm: Cp > ldx");
  SVC_REQUIRE(e.kind == EPI_GENERIC || e.kind == EPI_COND, "conv_gemm: paired epilogues run in conv_gemm2");
  if (a.N <= 32) return launch<256, 32>(a, e, s);
  if (a.N <= 64) return launch<256, 64>(a, e, s);
  return launch<128, 128>(a, e, s);
}

}  // namespace svc
