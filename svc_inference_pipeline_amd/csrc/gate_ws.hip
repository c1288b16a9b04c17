// DiffSVC dilated conv + gate as a weight-stationary row stream (modules/diffsvc.py:212-227, `ResidualBlock.forward`
// lines 220-227: y = dilated_conv(x + dproj) + conditioner_projection(cond); sigmoid(gate) * tanh(filter)), round 4.
//
// Per layer of every denoiser call: y[m][c] = sigmoid(g + cp_g) * tanh(f + cp_f), with
//   [g | f] = conv1d_k3,dil(x16)  (K = 3 taps x 384 channels = 1152, 768 packed output columns, engine.hip pair_perm).
// conv_gemm4 runs this as 128 x 128 output tiles, two 4-wave workgroups per CU, each K-tile DMA'd one step ahead: every
// tile streams its A rows and its 128 weight columns through LDS (64 FLOP per operand byte), which at the MFMA rate is the
// whole L2 -> LDS bandwidth of a CU (64 B per clock), so its K-loop runs at ~0.4 of the MFMA peak.
// Here the weights stay put instead:
//   * a workgroup owns 128 packed columns = 64 output channels, as 4 column sets of 16 gate + 16 filter columns; each set
//     belongs to a PAIR of waves on one SIMD (waves w and w + 4): wave w holds the set's weights for K-steps 0..23 (taps
//     0 and 1), wave w + 4 for K-steps 24..35 (tap 2), as MFMA fragments in VGPRs (2 x 24 / 12 x half8 = 192 / 96
//     registers each: two waves per SIMD), loaded once per launch;
//   * the workgroup walks its share of the rows in 16-row blocks: in step k the first wave of a pair runs K-steps 0..23
//     of block k and hands its two f32 accumulators to its partner through LDS, which continues them over K-steps
//     24..35 for block k - 1 (the partial sums are the partner's MFMA C operand, so the K order is one sequential chain,
//     exactly conv_gemm4's) and applies the gate in registers; one workgroup barrier per step;
//   * the input rows come through a ring of 160 rows in LDS, DMA'd in 32-row groups (25 KiB) once each: the three taps
//     of a block read its rows at offsets -dil, 0, +dil, so no row is fetched twice, and a group is issued 5 steps
//     before its first reader (the depth an HBM first touch under load needs at ~0.5 us per step);
//   * an A fragment (ds_read_b128, 16 rows x 32 channels) feeds the set's gate and filter MFMA (v_mfma_f32_16x16x32,
//     operands swapped so a lane's accumulator holds 4 consecutive columns of one row and a channel's gate and filter
//     values sit in the same lane): 128 B per clock of LDS reads per CU at the MFMA rate, half the LDS's.
// Roles: the first waves issue the ring DMAs (their only vector-memory operations after the prologue, so their vmcnt
// waits are exact); the second waves load the conditioner projection (two blocks ahead), apply the gate and store.
// Operand bytes per FLOP: the CU takes in 768 B per row for 128 x 1152 x 2 FLOP (384 FLOP per byte, 6x conv_gemm4).
// The 6 column groups x 42 row parts = 252 workgroups fill a 256-CU chip once; the 6 workgroups of a row part are placed
// on one XCD (blocks b, b + 8, ... share one under the observed round-robin placement, speed only), so each input row
// is fetched into one L2.
// Zero padding: an (output row, tap) whose input row lies outside its utterance (or past a ragged utterance's valid rows,
// ConvGemmArgs::tv) reads its A fragments from a 768-B zero row in LDS, so every ring row serves all three taps and no
// fragment needs a select.
// Bit-identical to conv_gemm4<128,128,gate> (tests/test_gpu_stages.py test_gate_ws_bit_identical).
#include <type_traits>

#include "common.h"

// gw_dma clobbers m0 (reserved for the compiler's own LDS-DMA and indexing uses, which all set it right before use)
#pragma clang diagnostic ignored "-Winline-asm"

namespace svc {

constexpr int GW_C = 384;             // channels per tap
constexpr int GW_N = 768;             // packed output columns (gate | filter per 64-column block)
constexpr int GW_K = 3 * GW_C;        // 1152 = 36 K-steps of 32
constexpr int GW_KS = 36;             // K-steps of 32
constexpr int GW_KA_DEF = 24;         // K-steps of a pair's first wave (0..23: taps 0 and 1); its partner takes 24..35
                                      // (tap 2) and also runs the gate epilogue. 18 / 18 left the partner at 2248 vs
                                      // 1672 cycles per step (r04m stamps); end to end the split barely matters:
                                      // 20 / 22 / 23 / 24: 884.0 / 883.9 / 883.3 / 885.9 and 885.2 / 883.6 / 884.0 /
                                      // 886.6 audio-s/s (r04p, alternating). SVC_GWS_KA (18 / 22) for A/B runs
constexpr int GW_HALO = 8;            // largest tap shift (dilation 8): ring row 0 = input row r_begin - 8
constexpr int GW_GR = 32;             // rows per DMA group
constexpr int GW_NG = 5;              // ring slots (groups): 160 rows
constexpr int GW_RROWS = GW_NG * GW_GR;
constexpr int GW_STRIDE = 800;        // ring row stride: 768 B + 32 B, so a row adds 2 bank slots (of 16 B) and the
                                      // 16-row fragment reads are conflict-free at any row offset (tap shift, ring wrap)
constexpr int GW_GBYTES = GW_GR * GW_STRIDE;  // 25,600 B = 25 DMA pieces of 1 KiB
constexpr int GW_GPIECES = GW_GBYTES / 1024;
constexpr int GW_PART = GW_NG * GW_GBYTES;    // partial accumulators: [2 buffers][4 pairs][2 blocks][64 lanes][16 B]
constexpr int GW_ZERO = GW_PART + 2 * 4 * 2048;  // 768 B of zeros
constexpr int GW_TVT = GW_ZERO + 768;  // ragged batches: valid input rows per utterance
constexpr int GW_MAXB = 1024;
constexpr int GW_STL = GW_TVT + GW_MAXB * 4;   // diagnostics: in-LDS step stamps [4 kinds][GW_NSTAMP] u64
constexpr int GW_NSTAMP = 128;
constexpr int GW_LDS = GW_STL;                      // 149,248 B (the production instances hold no stamp region)
constexpr int GW_LDS_STAMPS = GW_STL + 4 * GW_NSTAMP * 8;  // 153,344 B: the stamped diagnostics instance (DBG & 8)
constexpr int GW_PARTS = 42;          // row parts (x 6 column groups)
constexpr int GW_GRID = 256;
constexpr int GW_NT = 512;
constexpr uint32_t GW_OOR = 0x80000000u;  // a voffset past every descriptor's range (loads return 0, stores drop)
constexpr uint32_t GW_CFG = 0x00020000u;  // buffer descriptor dword 3 (raw, 32-bit data format)
static_assert(GW_GBYTES % 1024 == 0 && GW_STRIDE % 16 == 0, "ring geometry");

struct GateWsArgs {
  const f16* X;       // [M][384] layer input (the split residual stream's high half)
  const f16* W;       // W in fragment order (gate_ws_pack)
  const float* bias;  // [768] packed
  const f16* cp;      // [M][ld_cp] conditioner projection (packed order)
  int ld_cp;
  f16* y;             // [M][ldy] gate output
  int ldy;
  int M, T;           // rows = utterances x T
  int dil;            // tap shift (tap_mul; tap_add = -dil)
  const int* tv;      // ragged: utterance b has min(T, tv[b] * tv_mul) valid input rows (NULL = T)
  int tv_mul, B;
  float invT;
  unsigned long long* stamps;  // diagnostics (SVC_GWS_STAMPS, svc_gemm_bench only): s_memtime per workgroup and step
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 gw_desc(const void* base, int64_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return u32x4{(uint32_t)a, (uint32_t)(a >> 32) & 0xffffu, (uint32_t)(bytes > 0 ? bytes : 0), GW_CFG};
}
// LDS-DMA of 16 B per lane (lane i's bytes land at lds + 16 i), in inline asm: the compiler neither counts it nor drains
// it before the LDS reads of other ring slots; the first waves' counted vmcnt waits order it
__device__ __forceinline__ void gw_dma(u32x4 d, uint32_t voff, unsigned char* lds) {
  const uint32_t m0 =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               ::"s"(m0), "v"(voff), "s"(d) : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void gw_vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// workgroup barrier behind this wave's LDS writes (the partial accumulators, the prologue's tables)
__device__ __forceinline__ void gw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

union GwH4 { uint2 u; f16 h[4]; };

// Diagnostics (compile-time DBG, svc_gemm_bench / SVC_GWS_DBG / SVC_GWS_STAMPS only): 2 no MFMAs, 4 no gate arithmetic,
// 8 step stamps. Stamps: s_memtime at step boundaries, [workgroup][kind][GW_NSTAMP] in a buffer nothing else reads.
// Kind 0: the first second wave after each barrier; kinds 1 / 2: the first first wave before / after its ring wait,
// kind 3: the first second wave before its barrier. All kept in LDS (kind 0 in the fourth slot) and copied out after
// the loop, so the stamped kernel issues no extra vector-memory operations inside it (a first wave's vmcnt waits are
// hand-counted; a per-step store in the second waves would change their waits: kind 0 was a direct store before r05ap)
template <int DBG>
__device__ __forceinline__ void gw_stamp(unsigned char* smw, int i) {
  if constexpr ((DBG & 8) != 0)
    if (threadIdx.x == 256 && i < GW_NSTAMP)
      reinterpret_cast<unsigned long long*>(smw + GW_STL)[3 * GW_NSTAMP + i] = __builtin_amdgcn_s_memtime();
}
template <int DBG>
__device__ __forceinline__ void gw_stamp_lds(unsigned char* smw, int kind, int i, int thread) {
  if constexpr ((DBG & 8) != 0)
    if (threadIdx.x == thread && i < GW_NSTAMP)
      reinterpret_cast<unsigned long long*>(smw + GW_STL)[(kind - 1) * GW_NSTAMP + i] = __builtin_amdgcn_s_memtime();
}
template <int DBG>
__device__ __forceinline__ void gw_stamp_flush(const GateWsArgs& a, const unsigned char* smw, int kind, int n) {
  if constexpr ((DBG & 8) != 0) {
    const unsigned long long* src =
        reinterpret_cast<const unsigned long long*>(smw + GW_STL) + (kind == 0 ? 3 : kind - 1) * GW_NSTAMP;
    for (int i = threadIdx.x & 63; i < n && i < GW_NSTAMP; i += 64)
      a.stamps[((size_t)blockIdx.x * 4 + kind) * GW_NSTAMP + i] = src[i];
  }
}

// W in fragment order (gate_ws_pack): for column group c, pair p, K half kh, K-step s, gate / filter g and lane l, the
// 8 halves W[n][32 ks + 8 (l >> 4) ..], n = (g ? nf : ng) + (l & 15), K-step ks: each wave's loads are contiguous KiB
__device__ __forceinline__ size_t gw_frag_index(int c, int p, int ks, int g) {
  return (size_t)(((c * 4 + p) * GW_KS + ks) * 2 + g) * 512;
}

// The lane's row of block j of the part: utterance bb and frame t, advanced block by block without a branch (T >= 16,
// gate_ws_fits: at most one utterance boundary per block); tvt holds every utterance's valid rows (T without a table)
struct GwRow {
  int m, bb, t, tvb;
  __device__ __forceinline__ void init(const GateWsArgs& a, const int* tvt, int m0) {
    m = m0;
    bb = (int)((float)m * a.invT);
    t = m - bb * a.T;
    if (t < 0) {
      --bb;
      t += a.T;
    } else if (t >= a.T) {
      ++bb;
      t -= a.T;
    }
    tvb = tvt[min(bb, a.B - 1)];
  }
  __device__ __forceinline__ void next(const GateWsArgs& a, const int* tvt) {
    m += 16;
    t += 16;
    const bool wrap = t >= a.T;
    t = wrap ? t - a.T : t;
    bb += wrap ? 1 : 0;
    tvb = tvt[min(bb, a.B - 1)];
  }
  // LDS byte offsets of the three tap rows for row block j: ring row (8 + 16 j + fr + (tap - 1) dil) mod 160, or the
  // zero row when the tap's input frame lies outside the utterance's valid rows (or the row is past M)
  __device__ __forceinline__ void bases(const GateWsArgs& a, int j, int fr, int fk, int base[3]) const {
    const bool row_ok = m < a.M;
    const int r0 = (16 * j) % GW_RROWS + GW_HALO + fr;  // < 160 + 23
#pragma unroll
    for (int tap = 0; tap < 3; ++tap) {
      const int tp = t + (tap - 1) * a.dil;
      const bool ok = row_ok && tp >= 0 && tp < tvb;
      int rr = r0 + (tap - 1) * a.dil;  // in [0, 160 + 31)
      rr = rr >= GW_RROWS ? rr - GW_RROWS : rr;
      base[tap] = (ok ? rr * GW_STRIDE : GW_ZERO) + fk * 16;
    }
  }
};

// sched_group_barrier masks (LLVM AMDGPU): VALU, MFMA, DS read
constexpr int GW_SG_VALU = 0x002, GW_SG_MFMA = 0x008, GW_SG_DSR = 0x100;

template <bool BF, int DBG, int GW_KA = GW_KA_DEF>
__global__ __launch_bounds__(GW_NT, 1) void gate_ws_kernel(GateWsArgs a) {
  using O = Op16<BF>;
  constexpr int GW_KB = GW_KS - GW_KA;
  static_assert(GW_KA >= GW_KB && GW_KB >= 4, "K split: the weight arrays are sized for the first wave; the epilogue's 4 "
                                             "elements need 4 segments");
  extern __shared__ __align__(16) unsigned char smw[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pair = wave & 3, kh = wave >> 2;
  const int fr = lane & 15, fk = lane >> 4;

  // workgroup -> (column group, row part): the 6 groups of parts 0..39 on one XCD each; parts 40, 41 on the spares
  const int b = blockIdx.x, x = b & 7, j = b >> 3;
  int type, part;
  if (j < 30) {
    type = j % 6;
    part = x * 5 + j / 6;
  } else {
    const int s = (j - 30) * 8 + x;
    if (s >= 12) return;
    type = s % 6;
    part = 40 + s / 6;
  }
  const int nblk = (a.M + 15) >> 4;
  const int blk0 = (int)((int64_t)part * nblk / GW_PARTS);
  const int nsub = (int)((int64_t)(part + 1) * nblk / GW_PARTS) - blk0;
  if (nsub <= 0) return;
  const int r_begin = blk0 * 16;
  const int r_end = min(a.M, r_begin + nsub * 16);

  // this pair's columns: packed 64-column block q, half h: gate ng .. ng + 15, filter ng + 32 .. ng + 47
  const int q = 2 * type + (pair >> 1), h = pair & 1;
  const int ng = 64 * q + 16 * h, nf = ng + 32;
  const int ch = 32 * q + 16 * h + 4 * fk;  // the lane's 4 output channels (second waves)

  {
    int* tvt = reinterpret_cast<int*>(smw + GW_TVT);
    for (int i = tid; i < a.B; i += GW_NT) tvt[i] = a.tv ? min(a.T, a.tv[i] * a.tv_mul) : a.T;
  }
  for (int i = tid; i < 768 / 16; i += GW_NT) *reinterpret_cast<uint4*>(smw + GW_ZERO + i * 16) = make_uint4(0, 0, 0, 0);
  // the length table is read by every wave's GwRow::init before the prologue barrier (a 24 / 12 K split, whose second
  // waves reach it sooner, read it before it was written: a ragged batch differed from conv_gemm4, r04p)
  __syncthreads();
  const int* tvt = reinterpret_cast<const int*>(smw + GW_TVT);
  unsigned char* const part_buf = smw + GW_PART + pair * 2048;  // + (k & 1) * 8192

  // W fragments of the swapped MFMA (its first operand), this wave's K-steps: wg[s] / wf[s] = K-step ks0 + s
  half8 wg[GW_KA], wf[GW_KA];
  auto load_w = [&](int ks0, auto n_) __attribute__((always_inline)) {
    constexpr int N = decltype(n_)::value;
    const f16* wb = a.W + gw_frag_index(type, pair, ks0, 0) + lane * 8;
#pragma unroll
    for (int s = 0; s < N; ++s) {
      wg[s] = *reinterpret_cast<const half8*>(wb + (size_t)(2 * s) * 512);
      wf[s] = *reinterpret_cast<const half8*>(wb + (size_t)(2 * s + 1) * 512);
    }
  };
  // this wave's 18 K-steps of one block onto (ag, af). The A fragments are read four K-steps ahead of their MFMAs into
  // five registers sets, and every K-step is its own scheduling segment (sched_barrier): the read of K-step s + 4, the
  // two MFMAs of K-step s and hook(s), the caller's work for that segment (the second waves' gate epilogue, spread over
  // the segments so its VALU work sits between MFMAs). Left to itself the scheduler sank each read to just before its
  // MFMA pair (one read in flight, each pair waiting out the LDS latency: r04k / r04l assembly and step stamps).
  auto kloop = [&](const int base[3], int s_off, auto n_, floatx4& ag, floatx4& af, auto&& hook)
                   __attribute__((always_inline)) {
    constexpr int N = decltype(n_)::value;
    half8 av[5];
    auto rd = [&](int s) __attribute__((always_inline)) {
      const int ks = s_off + s;
      return *reinterpret_cast<const half8*>(smw + base[ks / 12] + (ks % 12) * 64);
    };
#pragma unroll
    for (int s = 0; s < 4; ++s) av[s] = rd(s);
#pragma unroll
    for (int s = 0; s < N; ++s) {
      __builtin_amdgcn_sched_barrier(0);
      if (s + 4 < N) av[(s + 4) % 5] = rd(s + 4);
      if constexpr (!(DBG & 2)) {
        ag = O::mfma(wg[s], av[s % 5], ag);
        af = O::mfma(wf[s], av[s % 5], af);
      }
      hook(s);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto no_hook = [](int) __attribute__((always_inline)) {};

  if (kh == 0) {
    // ------------------------------------------------------------------ first waves: K-steps 0..GW_KA - 1 + ring DMAs
    const u32x4 dx = gw_desc(a.X, (int64_t)a.M * GW_C * 2);
    // group g = input rows r_begin - 8 + 32 g .. + 31 into ring slot g % 5; its 25 pieces go to the four first waves
    // round robin (piece p = pair + 4 v): pair 0 issues 7 per group, the others 6. A lane's unit u of piece p -> row
    // u / 50 of the group, 16-B chunk u % 50 (48, 49: the row's padding, read as nothing)
    constexpr int PV = (GW_GPIECES + 3) / 4;  // 7
    uint32_t pc[PV];
#pragma unroll
    for (int v = 0; v < PV; ++v) {
      const int u = (pair + 4 * v) * 64 + lane;
      const int r = u / 50, c = u - r * 50;
      pc[v] = c < 48 ? (uint32_t)(r * GW_C * 2 + c * 16) : GW_OOR;
    }
    const bool seven = pair + 4 * (PV - 1) < GW_GPIECES;  // this wave issues PV pieces per group (else PV - 1)
    // every group index is issued, past the part's rows too (harmless rows or zeros), so each wave's count of DMAs
    // younger than a given group is the same at every step: the waits below are compile-time vmcnt values
    auto issue = [&](int g) __attribute__((always_inline)) {
      const uint32_t base = (uint32_t)((r_begin - GW_HALO + g * GW_GR) * (GW_C * 2));  // (negative: wraps, out of range)
      unsigned char* dst = smw + (g % GW_NG) * GW_GBYTES + pair * 1024;
#pragma unroll
      for (int v = 0; v < PV; ++v)
        if (v < PV - 1 || seven) gw_dma(dx, base + pc[v], dst + v * 4096);
    };
    issue(0);
    issue(1);
    load_w(0, std::integral_constant<int, GW_KA>());
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0) through the builtin, so the compiler knows W has landed too
    issue(2);
    issue(3);
    issue(4);
    GwRow row;
    row.init(a, tvt, r_begin + fr);
    gw_barrier();  // groups 0 and 1, the zero row and the length table
    // Block j reads groups j / 2 .. (j + 1) / 2, so group G's last reader is block 2 G + 1 (the second wave, step
    // 2 G + 2). Group g = (k + 7) / 2 >= 5 is issued at the start of odd steps k >= 3, into the slot of group g - 5,
    // whose last reader finished in step k - 1; its first reader is block 2 g - 1, 5 steps later. At the end of step k,
    // block k + 1's groups (up to (k + 2) / 2) must have landed: the groups issued after them are the 3 newest on odd
    // steps and the 2 newest on even ones (3 on step 0: waiting for 2 there is merely early)
    auto step = [&](int k) __attribute__((always_inline)) {  // k < nsub; ends with the step's barrier
      if ((k & 1) && k >= 3) issue((k + 7) / 2);
      int base[3];
      row.bases(a, k, fr, fk, base);
      floatx4 ag = {0.f, 0.f, 0.f, 0.f}, af = {0.f, 0.f, 0.f, 0.f};
      kloop(base, 0, std::integral_constant<int, GW_KA>(), ag, af, no_hook);
      unsigned char* pb = part_buf + (k & 1) * 8192 + lane * 16;
      *reinterpret_cast<floatx4*>(pb) = ag;
      *reinterpret_cast<floatx4*>(pb + 1024) = af;
      row.next(a, tvt);
      gw_stamp_lds<DBG>(smw, 1, k, 0);
      if (k & 1) {
        if (seven) gw_vmwait<3 * PV>(); else gw_vmwait<3 * (PV - 1)>();
      } else {
        if (seven) gw_vmwait<2 * PV>(); else gw_vmwait<2 * (PV - 1)>();
      }
      gw_stamp_lds<DBG>(smw, 2, k, 0);
      gw_barrier();  // the partial sums of block k; every first wave's pieces of block k + 1's groups
    };
    for (int k = 0; k < nsub; ++k) step(k);
    gw_barrier();  // step nsub: the second waves finish block nsub - 1
    gw_vmwait<0>();  // (the groups issued past the part land before the workgroup's LDS is released)
    if (wave == 0) {
      gw_stamp_flush<DBG>(a, smw, 1, nsub);
      gw_stamp_flush<DBG>(a, smw, 2, nsub);
    }
  } else {
    // ------------------------------------------------------------------ second waves: K-steps GW_KA..35 + gate epilogue
    // Step k: the MFMAs of block k - 1 (its partial sums come from step k - 1), interleaved with the gate epilogue of
    // block k - 2, whose accumulators this wave kept from step k - 1. In the steady state (2 <= k < nsub) a step is one
    // basic block, so the scheduler can (and the group barriers below make it) spread the epilogue's VALU work and the
    // A-fragment reads among the MFMAs. These waves are the second-dispatched half: static priority 1 for the whole
    // loop (MI355X_MICROARCH.md, two waves per SIMD, item 4).
    const __amdgpu_buffer_rsrc_t rcp =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(a.cp), (short)0, a.M * a.ld_cp * 2, GW_CFG);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(a.y, (short)0, a.M * a.ldy * 2, GW_CFG);
    gw_stamp<DBG>(smw, 0);
    load_w(GW_KA, std::integral_constant<int, GW_KB>());
    const float4 bg = *reinterpret_cast<const float4*>(a.bias + ng + 4 * fk);
    const float4 bfv = *reinterpret_cast<const float4*>(a.bias + nf + 4 * fk);
    // conditioner projection of block j, loaded in step j (two steps before its epilogue) into register set j % 3:
    // fixed roles per set (the steady loop is unrolled by 3), so no register move waits on a load
    auto load_cp = [&](int blk, GwH4* dst) __attribute__((always_inline)) {
      const uint32_t vo = (uint32_t)(r_begin + blk * 16 + fr) * (uint32_t)(a.ld_cp * 2);  // rows past M read 0
      dst[0].u = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rcp, vo + (ng + 4 * fk) * 2, 0, 0));
      dst[1].u = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rcp, vo + (nf + 4 * fk) * 2, 0, 0));
    };
    GwH4 c0[2], c1[2], c2[2];
    floatx4 pg = {0.f, 0.f, 0.f, 0.f}, pf = {0.f, 0.f, 0.f, 0.f};  // accumulators of the block awaiting its epilogue
    GwRow row;
    row.init(a, tvt, r_begin + fr);
    gw_stamp<DBG>(smw, 1);
    gw_barrier();  // (pairs with the first waves' prologue barrier)
    // (priority 1 on the first waves instead, or on neither: 903.2 / 900.5 / 902.6 and 902.4 / 902.1 / 904.0 against
    // 908.1 / 908.0 / 907.3 audio-s/s, r04s)
    __builtin_amdgcn_s_setprio(1);
    gw_stamp<DBG>(smw, 2);
    // gate of the lane's element i (conv_gemm4's DIRECT epilogue arithmetic, same order), and the block's store (rows
    // past the part are dropped)
    auto gate_el = [&](int i, const GwH4* cp, const floatx4& ag, const floatx4& af) __attribute__((always_inline)) {
      if constexpr ((DBG & 4) != 0) {
        return (f16)(ag[i] + af[(i + 1) & 3]);
      } else {
        const float b_g = i == 0 ? bg.x : (i == 1 ? bg.y : (i == 2 ? bg.z : bg.w));
        const float b_f = i == 0 ? bfv.x : (i == 1 ? bfv.y : (i == 2 ? bfv.z : bfv.w));
        return O::enc_lo(gate_act(ag[i] + b_g + O::dec(cp[0].h[i]), af[i] + b_f + O::dec(cp[1].h[i])));
      }
    };
    auto store_blk = [&](int blk, const GwH4& pk) __attribute__((always_inline)) {
      const int m = r_begin + blk * 16 + fr;
      const uint32_t vo = m < r_end ? (uint32_t)m * (uint32_t)(a.ldy * 2) + (uint32_t)ch * 2 : GW_OOR;
      buffer_store_b64(pk.u, ry, vo);
    };
    auto epilogue = [&](int blk, const GwH4* cp, const floatx4& ag, const floatx4& af) __attribute__((always_inline)) {
      GwH4 pk;
#pragma unroll
      for (int i = 0; i < 4; ++i) pk.h[i] = gate_el(i, cp, ag, af);
      store_blk(blk, pk);
    };
    // the MFMAs of block blk on its partial sums (K-steps GW_KA..23: the rest of tap 1; 24..35: tap 2)
    auto mfma_blk = [&](int blk, floatx4& ag, floatx4& af, auto&& hook) __attribute__((always_inline)) {
      int base[3];
      row.bases(a, blk, fr, fk, base);
      const unsigned char* pb = part_buf + (blk & 1) * 8192 + lane * 16;
      ag = *reinterpret_cast<const floatx4*>(pb);
      af = *reinterpret_cast<const floatx4*>(pb + 1024);
      kloop(base, GW_KA, std::integral_constant<int, GW_KB>(), ag, af, hook);
      row.next(a, tvt);
    };
    auto end_step = [&](int k) __attribute__((always_inline)) {
      gw_stamp_lds<DBG>(smw, 3, k, 256);
      gw_barrier();
      gw_stamp<DBG>(smw, 3 + k);
    };
    // steady step k (2 <= k < nsub): cp(k) into LS, MFMAs of block k - 1 with the epilogue of block k - 2 (cp from ES)
    // in their K-step segments: element i at the end of segment (i + 1) GW_KB / 4 - 1 (every element, for any split),
    // the store after the last
    auto steady = [&](int k, GwH4* ls, const GwH4* es) __attribute__((always_inline)) {
      load_cp(k, ls);
      floatx4 ag, af;
      const floatx4 eg = pg, ef = pf;
      GwH4 pk;
      auto hook = [&](int s) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (s == (i + 1) * GW_KB / 4 - 1) pk.h[i] = gate_el(i, es, eg, ef);
        if (s == GW_KB - 1) store_blk(k - 2, pk);
      };
      mfma_blk(k - 1, ag, af, hook);
      pg = ag;
      pf = af;
      end_step(k);
    };
    // step 0: cp(0); step 1: cp(1), MFMAs of block 0 (round 6 tried issuing a steady step's vector-memory operations here
    // as well, a dropped store and an unconditional cp(1), so that the compiler's waits in the unrolled loop are exact:
    // the period-3 slow step stayed and the kernel was 0.5 % slower, profiles/r06_ab/r06h_r05_vs_head.txt, r06i_gate_preamble_revert.txt)
    load_cp(0, c0);
    end_step(0);
    if (nsub >= 2) load_cp(1, c1);
    mfma_blk(0, pg, pf, no_hook);
    end_step(1);
    int k = 2;
    for (; k + 3 <= nsub; k += 3) {  // k = 2 mod 3: loads into c2, c0, c1; epilogues from c0, c1, c2
      steady(k, c2, c0);
      steady(k + 1, c0, c1);
      steady(k + 2, c1, c2);
    }
    if (k < nsub) steady(k++, c2, c0);
    if (k < nsub) steady(k++, c0, c1);
    // step nsub (>= 2): MFMAs of block nsub - 1, epilogue of block nsub - 2 (cp set (nsub - 2) % 3)
    auto epi_set = [&](int blk) __attribute__((always_inline)) {  // epilogue of blk from its set blk % 3
      switch (blk % 3) {
        case 0: epilogue(blk, c0, pg, pf); break;
        case 1: epilogue(blk, c1, pg, pf); break;
        default: epilogue(blk, c2, pg, pf); break;
      }
    };
    if (nsub >= 2) {
      floatx4 ag, af;
      mfma_blk(nsub - 1, ag, af, no_hook);
      epi_set(nsub - 2);
      pg = ag;
      pf = af;
      end_step(nsub);
    }
    epi_set(nsub - 1);  // the last block's epilogue
    if (wave == 4) {
      gw_stamp_flush<DBG>(a, smw, 3, nsub + 1);
      gw_stamp_flush<DBG>(a, smw, 0, nsub + 4);
    }
  }
}

// W (packed [768][1152], W[n][k]) -> gate_ws fragment order (gw_frag_index): 16 B per thread
__global__ void gate_ws_pack_kernel(const f16* __restrict__ W, f16* __restrict__ Wf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // 16-B unit
  if (i >= GW_N * GW_K / 8) return;
  const int lane = i & 63;
  int r = i >> 6;
  const int g = r & 1;
  r >>= 1;
  const int ks = r % GW_KS;
  r /= GW_KS;
  const int p = r & 3, c = r >> 2;
  const int n = 64 * (2 * c + (p >> 1)) + 16 * (p & 1) + 32 * g + (lane & 15);
  const int k = 32 * ks + 8 * (lane >> 4);
  *reinterpret_cast<uint4*>(Wf + (size_t)i * 8) = *reinterpret_cast<const uint4*>(W + (size_t)n * GW_K + k);
}

int gate_ws_pack(const f16* W, int ldw, f16* Wf, hipStream_t s) {
  SVC_REQUIRE(ldw == GW_K && ((uintptr_t)W & 15) == 0 && ((uintptr_t)Wf & 15) == 0, "gate_ws_pack: ldw %d", ldw);
  hipLaunchKernelGGL(gate_ws_pack_kernel, dim3(cdiv(GW_N * GW_K / 8, 256)), dim3(256), 0, s, W, Wf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}
size_t gate_ws_pack_elems() { return (size_t)GW_N * GW_K; }

// diagnostics (svc_gemm_bench with SVC_GWS_STAMPS): a [256][GW_NSTAMP] s_memtime buffer, else NULL
unsigned long long* gate_ws_stamps = nullptr;
int gate_ws_nstamp() { return 4 * GW_NSTAMP; }  // per workgroup

static bool gate_ws_fits_shape(const ConvGemmArgs& a, const EpiArgs& e) {
  const int d = a.tap_mul;
  return e.kind == EPI_GATE && e.cp && e.y16 && e.bias && a.Cp == GW_C && a.Cvalid == GW_C && a.ldx == GW_C &&
         a.K == GW_K && a.Kpad == GW_K && a.N == GW_N && (d == 1 || d == 2 || d == 4 || d == 8) && a.tap_add == -d &&
         a.istride == 1 && a.T_in == a.T_out && a.T_out >= 16 && a.B <= GW_MAXB && e.ld_cp % 4 == 0 && e.ldy16 % 4 == 0 &&
         (int64_t)a.B * a.T_out * std::max(e.ld_cp, std::max(e.ldy16, GW_C)) * 2 < (1ll << 30);
}

bool gate_ws_fits(const ConvGemmArgs& a, const EpiArgs& e) { return a.Wfrag && gate_ws_fits_shape(a, e); }

int gate_ws(const ConvGemmArgs& a, const EpiArgs& e, hipStream_t s) {
  SVC_REQUIRE(gate_ws_fits(a, e), "gate_ws: not the DiffSVC dilated-conv gate shape");
  SVC_REQUIRE(((uintptr_t)a.X & 15) == 0 && ((uintptr_t)a.Wfrag & 15) == 0 && ((uintptr_t)e.cp & 7) == 0 &&
                  ((uintptr_t)e.y16 & 7) == 0 && ((uintptr_t)e.bias & 15) == 0,
              "gate_ws: alignment");
  const int M = a.B * a.T_out;
  if (M == 0) return SVC_OK;
  static const int dbg = getenv("SVC_GWS_DBG") ? atoi(getenv("SVC_GWS_DBG")) : 0;  // (diagnostics, read once)
  GateWsArgs g{a.X, a.Wfrag, e.bias, e.cp, e.ld_cp, e.y16, e.ldy16, M, a.T_out, a.tap_mul, a.tv, a.tv_mul, a.B,
               1.0f / (float)a.T_out, gate_ws_stamps};
  // diagnostics instances (fp16 only): 2 no MFMAs, 4 no gate arithmetic, 8 step stamps (SVC_GWS_STAMPS)
  static const int ka = getenv("SVC_GWS_KA") ? atoi(getenv("SVC_GWS_KA")) : GW_KA_DEF;  // (A/B runs, read once)
  const void* fn = a.bf16 ? (const void*)gate_ws_kernel<true, 0> : (const void*)gate_ws_kernel<false, 0>;
  if (!a.bf16 && gate_ws_stamps) fn = (const void*)gate_ws_kernel<false, 8>;
  else if (!a.bf16 && dbg == 2) fn = (const void*)gate_ws_kernel<false, 2>;
  else if (!a.bf16 && dbg == 4) fn = (const void*)gate_ws_kernel<false, 4>;
  else if (!a.bf16 && ka == 18) fn = (const void*)gate_ws_kernel<false, 0, 18>;
  else if (!a.bf16 && ka == 22) fn = (const void*)gate_ws_kernel<false, 0, 22>;
  const int lds = fn == (const void*)gate_ws_kernel<false, 8> ? GW_LDS_STAMPS : GW_LDS;
  if (int st = ensure_dyn_lds(fn, lds)) return st;
  const int tok = prof_begin("gate_ws<16x128>", 2.0 * M * (double)GW_N * GW_K, 0.0, s);
  void* args[] = {&g};
  SVC_HIP_CHECK(hipLaunchKernel(fn, dim3(GW_GRID), dim3(GW_NT), args, lds, s));
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}



}  // namespace svc
