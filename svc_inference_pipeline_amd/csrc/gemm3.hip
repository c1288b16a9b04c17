// Third-generation implicit-GEMM Conv1d / Linear for gfx950: 8-wave ping-pong, v_mfma_f32_16x16x32_f16 (or _bf16 for
// bfloat16 operands, ConvGemmArgs::bf16).
//
// Same operands and epilogues as conv_gemm2 (A = time-major f16 activations read through per-tap row
// shifts, B = weights packed [Npad][Kpad], LDS images of 128-B rows with the 16-B chunk XOR swizzle
// kv ^ (row & 6) applied on the DMA source address), different schedule:
//
//   * 8 waves = 2 (M) x 4 (N); wave tile (BM/2) x (BN/4), split into 4 quadrants (m half, n half).
//     A K-tile (BK = 64) is 4 phases, one quadrant each: phase p reads its quadrant's fragments
//     (L section), then barrier, then 16 MFMAs (M section, s_setprio 1), then barrier.
//   * The two wave groups run one barrier apart (group 1 takes an extra barrier first), so on every
//     SIMD one wave's M section overlaps the other wave's L section: LDS-read latency and DMA issue
//     hide behind the partner's MFMAs instead of stalling the matrix pipe.
//   * B fragments of both quadrant halves stay in registers for the whole K-tile (as A's do for two phases), so
//     every half-tile image is read in one phase only: A-lo and B-lo in phase 0, B-hi in 1, A-hi in 2, none in 3.
//   * Global -> LDS by LDS-DMA into 2 K-tile buffers, one half-tile (A-lo, A-hi, B-lo or B-hi: the rows one quadrant
//     half needs) per phase with a counted vmcnt:
//         phase 0: B-hi(k+1)  1: A-hi(k+1)  2: A-lo(k+2)  3: B-lo(k+2)
//     An LDS-DMA instruction costs its wave 60-185 issue cycles (MI355X_MICROARCH.md), so the pieces are spread evenly
//     over the phases. Each half-tile is restaged >= 2 phases after its only read of the previous use of that buffer
//     (write-after-read across the staggered groups) and retired (vmcnt + barrier) 1 phase before its first read: 4
//     phases in flight for every half-tile. Tiles past the end are dummy DMAs from the zero page so the counts stay
//     uniform.
//   * When Cp % 64 == 0 (and X / W fit 32-bit offsets) a K-tile lies inside one conv tap: the DMAs go through buffer
//     descriptors, each lane's 32-bit voffset fixed per tap (A; padding rows out of the descriptor's range, which the
//     hardware bounds check turns into zeros) or per launch (B), the K-tile's channel offset the scalar soffset: no
//     per-lane address arithmetic in the K-loop.
//   (A tap-reuse form that staged a 64-channel chunk's A rows once for every tap moved ~40 % fewer operand bytes on
//    the multi-tap convs yet ran 5-10 % slower; it was removed in round 3, DESIGN.md.)
#include <cstdio>
#include <cstdlib>
#include "common.h"
#include "epilogue.h"

namespace svc {

template <int BM, int BN>
struct G3 {
  static constexpr int NT = 512;
  // waves: WMW (M) x WNW (N) = 2 x 4, or 4 x 2 for BN = 192 (the BigVGAN C = 192 convs without idle columns: a quadrant
  // of 48 columns = 3 fragments). (A 256 x 96 tile on 8 x 1 waves for the C = 96 convs ran no faster than 128 x 128 with
  // its idle quarter: 815.7 / 606.0 / 388.3 against 811.3 / 602.5 / 371.1 us at k = 11 / 7 / 3, r05ah.)
  static constexpr int WNW = BN % 128 == 0 ? 4 : 2, WMW = 8 / WNW;
  static constexpr int WTM = BM / WMW, WTN = BN / WNW;  // wave tile
  static constexpr int QM = WTM / 2, QN = WTN / 2;   // quadrant (one phase)
  static constexpr int FQM = QM / 16, FQN = QN / 16; // 16x16 fragments per quadrant
  static constexpr int TILE = (BM + BN) * 128;       // bytes of one K-tile image (A rows, then B rows)
  static constexpr int RING = 2 * TILE;
  static constexpr int AH = BM / 128;                // DMA instructions per wave per A half-tile
  // B half-tile: BN / 16 DMA instructions over the 8 waves: BH per wave, or BH on waves 0 .. BW - 1 and BHL = BH - 1
  // on the others (BN = 192: two on waves 0-3, one on 4-7); each wave's vmcnt counts use its own number
  static constexpr int BH = (BN / 16 + 7) / 8, BW = BN / 16 - 8 * (BH - 1), BHL = BW == 8 ? BH : BH - 1;
  static constexpr int EP = (BM * (BN + 4) * 4 <= 163840) ? 1 : 2;
  static constexpr int LDC = BN / EP + 4;
  static constexpr int C_BYTES = BM * LDC * 4;
  static constexpr int LDS = RING > C_BYTES ? RING : C_BYTES;
  static_assert(LDS <= 163840, "LDS budget");
  static_assert(QM % 16 == 0 && QN % 16 == 0 && QM % 8 == 0 && QN % 8 == 0 && AH >= 1 && BH >= 1 &&
                    BM % 128 == 0 && BN % 16 == 0, "tile shape");
};

// 16-B chunk swizzle of the 128-B-row LDS images: conflict-free ds_read_b128 fragment reads (16 consecutive
// rows per lane group) for every starting row.
__device__ __forceinline__ int sw3(int row, int kv) { return kv ^ (row & 6); }

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void g3_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void g3_dma(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

constexpr uint32_t G3_OOR = 0x7ffffff0u;  // a voffset past every descriptor's range: the DMA lands zeros
__device__ __forceinline__ void g3_bdma(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, unsigned char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, (int)voff, (int)soff,
                                           0, 0);
}

// row (within the A or B image) of element i of half-tile h, for a half made of blocks of Q rows
// every W rows: rows w*W + h*Q + [0, Q)
__device__ __forceinline__ int half_row(int i, int h, int Q, int W) { return (i / Q) * W + h * Q + (i % Q); }

// Register epilogue forms (FORM > 0, !PAIR): the MFMAs run with A and B swapped, so a lane's accumulator holds
// 4 consecutive columns of one output row and the epilogue reads and writes HBM straight from registers (no C tile
// through LDS, no extra barriers). Each form is the epilogue_pass arithmetic, in the same order, for one family:
//   G3_F16  : act(acc + bias) (* col_scale for n < scale_cols) -> out16 (+ split16 lo / hi copies)
//   G3_RES32: acc + bias (+ add_row) ((acc32 + v) / acc_div) -> out32 and / or out16 (+ add16)
//   G3_SPLIT: acc + bias, ((acc16_hi + acc16_lo) - acc_sub + v) / acc_div -> out16 = hi(v + add16), lo16 = lo
enum { G3_LDS = 0, G3_F16 = 1, G3_RES32 = 2, G3_SPLIT = 3 };

template <int BM, int BN, bool CP64, bool PAIR, int FORM = G3_LDS, bool BF = false>
__global__ __launch_bounds__(512, 1) void conv_gemm3_kernel(ConvGemmArgs a, EpiArgs e, const f16* zpage,
                                                           float inv_cp) {
  static_assert(FORM == G3_LDS || !PAIR, "register epilogues: generic epilogues only");
  using CF = G3<BM, BN>;
  // the paired gate epilogue (epilogue_pass<PAIR>) walks 64-column gate | filter blocks: every LDS pass must hold whole
  // blocks (the 256 x 192 tile's two 96-column passes do not)
  static_assert(!PAIR || (BN / CF::EP) % 64 == 0, "paired epilogue: pass width must be a multiple of 64 columns");
  using O = Op16<BF>;  // operand format (binary16 or bfloat16)
  extern __shared__ __align__(16) unsigned char sm3[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / CF::WNW, wn = wave % CF::WNW;
  const int grp = wave >> 2;  // stagger group: one wave of each per SIMD
  const bool bfull = CF::BH == CF::BHL || wave < CF::BW;  // this wave issues BH (else BHL) B pieces per half-tile

  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tile_n = wgid % a.ntiles_n, tile_m = wgid / a.ntiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int M = a.B * a.T_out;
  const int nk = a.Kpad / 64;
  const f16* zsrc = zpage + lane * 8;

  // ---- DMA slots. A half h, instruction v: image rows rb .. rb+7, lane -> row rb + (lane >> 3),
  // LDS chunk lane & 7 holding logical k-chunk kv = sw3(row, lane & 7).
  int a_rb[2][CF::AH], a_kv[2][CF::AH], a_t[2][CF::AH], a_tin[2][CF::AH];
  const f16* a_p[2][CF::AH];
  uint32_t a_row[2][CF::AH], a_voff[2][CF::AH];  // CP64: byte offset of the lane's A row at tap shift 0 / this tap
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int v = 0; v < CF::AH; ++v) {
      const int u = wave + 8 * v;
      const int rb = half_row(8 * u, h, CF::QM, CF::WTM);
      const int row = rb + (lane >> 3);
      const int kv = sw3(row, lane & 7);
      a_rb[h][v] = rb;
      a_kv[h][v] = kv;
      const int m = m0 + row;
      if (m < M) {
        const int b = m / a.T_out, t = m - b * a.T_out;
        a_t[h][v] = t * a.istride;
        a_tin[h][v] = valid_in_rows(a, b);
        a_p[h][v] = a.X + (int64_t)b * a.T_in * a.ldx + kv * 8;
        a_row[h][v] = (uint32_t)(((b * a.T_in + a_t[h][v]) * a.ldx + kv * 8) * 2);
      } else {
        a_t[h][v] = -(1 << 29);
        a_tin[h][v] = 0;
        a_p[h][v] = a.X;
        a_row[h][v] = 0u;
      }
      a_voff[h][v] = G3_OOR;
    }
  int b_rb[2][CF::BH];
  const f16* b_p[2][CF::BH];
  uint32_t b_voff[2][CF::BH];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int v = 0; v < CF::BH; ++v) {
      const int u = min(wave + 8 * v, BN / 16 - 1);  // (u past the half-tile: a wave with BHL pieces, never issued)
      const int rb = half_row(8 * u, h, CF::QN, CF::WTN);
      const int row = rb + (lane >> 3);
      b_rb[h][v] = rb;
      b_p[h][v] = a.W + (int64_t)(n0 + row) * a.Kpad + sw3(row, lane & 7) * 8;
      b_voff[h][v] = (uint32_t)(((n0 + row) * a.Kpad + sw3(row, lane & 7) * 8) * 2);
    }
  // CP64 descriptors (unused otherwise); extents checked on the host (< 1 GiB: no voffset + soffset wraps)
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(a.X), (short)0, a.B * a.T_in * a.ldx * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(a.W), (short)0, a.ntiles_n * BN * a.Kpad * 2, 0x00020000);

  auto a_img = [&](int kt) { return sm3 + (kt & 1) * CF::TILE; };
  auto b_img = [&](int kt) { return sm3 + (kt & 1) * CF::TILE + BM * 128; };
  auto issue_a = [&](int h, int kt) {
    unsigned char* dst = a_img(kt);
    if constexpr (CP64) {
      // the whole K-tile lies in tap `tap`; columns c0 .. c0+63 of it. Each half sees kt = 0, 1, 2, ... in order, so
      // its voffsets are recomputed at the first K-tile of every tap; past the end (kt >= nk) the DMAs land zeros
      const int kg = kt * 64;
      const int tap = kg / a.Cp;  // wave-uniform
      const int c0 = kg - tap * a.Cp;
      if (kt < nk) {
        if (c0 == 0) {
          const int shift = tap * a.tap_mul + a.tap_add;
#pragma unroll
          for (int v = 0; v < CF::AH; ++v) {
            const int st = a_t[h][v] + shift;
            a_voff[h][v] = st >= 0 && st < a_tin[h][v] ? a_row[h][v] + (uint32_t)(shift * a.ldx * 2) : G3_OOR;
          }
        }
#pragma unroll
        for (int v = 0; v < CF::AH; ++v) g3_bdma(rx, a_voff[h][v], (uint32_t)(c0 * 2), dst + a_rb[h][v] * 128);
      } else {
#pragma unroll
        for (int v = 0; v < CF::AH; ++v) g3_bdma(rx, G3_OOR, 0u, dst + a_rb[h][v] * 128);
      }
    } else {
#pragma unroll
      for (int v = 0; v < CF::AH; ++v) {
        const int kg = kt * 64 + a_kv[h][v] * 8;
        int tap = (int)((float)kg * inv_cp);
        if ((tap + 1) * a.Cp <= kg) ++tap;
        if (tap * a.Cp > kg) --tap;
        const int c = kg - tap * a.Cp;
        const int st = a_t[h][v] + tap * a.tap_mul + a.tap_add;
        const bool ok = kt < nk && kg < a.K && st >= 0 && st < a_tin[h][v];
        // a_p already carries the lane's kv * 8 column offset: add the tap-local column base only
        const f16* src = ok ? a_p[h][v] + (int64_t)st * a.ldx + (c - a_kv[h][v] * 8) : zsrc;
        g3_dma(src, dst + a_rb[h][v] * 128);
      }
    }
  };
  auto issue_b = [&](int h, int kt) {
    unsigned char* dst = b_img(kt);
    if constexpr (CP64) {
#pragma unroll
      for (int v = 0; v < CF::BH; ++v)
        if (v < CF::BHL || bfull)
          g3_bdma(rw, kt < nk ? b_voff[h][v] : G3_OOR, (uint32_t)(kt * 128), dst + b_rb[h][v] * 128);
    } else {
      const int koff = kt * 64;
#pragma unroll
      for (int v = 0; v < CF::BH; ++v)
        if (v < CF::BHL || bfull)
          g3_dma(kt < nk ? (const void*)(b_p[h][v] + koff) : (const void*)zsrc, dst + b_rb[h][v] * 128);
    }
  };

  // a phase's wait: this wave's pieces of the two half-tiles issued after the ones to retire (2 AH + 2 B pieces)
  auto g3_wait = [&]() __attribute__((always_inline)) {
    if (bfull) vm_wait<2 * CF::AH + 2 * CF::BH>();
    else vm_wait<2 * CF::AH + 2 * CF::BHL>();
  };
  floatx4 acc[2][2][CF::FQM][CF::FQN];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int i = 0; i < CF::FQM; ++i)
#pragma unroll
        for (int j = 0; j < CF::FQN; ++j) acc[x][y][i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  half8 af[CF::FQM][2], bfl[CF::FQN][2], bfh[CF::FQN][2];
  const int fr = lane & 15, fk = lane >> 4;

  // one phase: quadrant (QMI, QNI) of K-tile kt
  auto phase = [&](auto QMI_, auto QNI_, int kt) {
    constexpr int QMI = decltype(QMI_)::value, QNI = decltype(QNI_)::value;
    constexpr int P = QMI * 2 + QNI;
    const unsigned char* Ab = a_img(kt);
    const unsigned char* Bb = b_img(kt);
    // ---- L section: A-lo + B-lo (phase 0), B-hi (1), A-hi (2); phase 3 reuses A-hi and B-hi
    if constexpr (QNI == 0) {
#pragma unroll
      for (int i = 0; i < CF::FQM; ++i) {
        const int row = wm * CF::WTM + QMI * CF::QM + i * 16 + fr;
#pragma unroll
        for (int s = 0; s < 2; ++s)
          af[i][s] = *reinterpret_cast<const half8*>(Ab + row * 128 + (sw3(row, s * 4 + fk) << 4));
      }
    }
    if constexpr (QMI == 0) {
#pragma unroll
      for (int j = 0; j < CF::FQN; ++j) {
        const int row = wn * CF::WTN + QNI * CF::QN + j * 16 + fr;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const half8 v = *reinterpret_cast<const half8*>(Bb + row * 128 + (sw3(row, s * 4 + fk) << 4));
          if constexpr (QNI == 0)
            bfl[j][s] = v;
          else
            bfh[j][s] = v;
        }
      }
    }
    // restage one half-tile; each wait retires the half-tiles the next phase reads (3 phases read; phase 3 none)
    if constexpr (P == 0) {
      issue_b(1, kt + 1);
      g3_wait();
    } else if constexpr (P == 1) {
      issue_a(1, kt + 1);
      g3_wait();
    } else if constexpr (P == 2) {
      issue_a(0, kt + 2);
    } else {
      issue_b(0, kt + 2);
      g3_wait();
    }
    g3_barrier();
    // ---- M section
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < CF::FQM; ++i)
#pragma unroll
        for (int j = 0; j < CF::FQN; ++j) {
          const half8& b = QNI == 0 ? bfl[j][s] : bfh[j][s];
          if constexpr (FORM != G3_LDS)  // C^T fragment: acc[..][i][j][r] = C[row fr of block i][col fk*4 + r of j]
            acc[QMI][QNI][i][j] = O::mfma(b, af[i][s], acc[QMI][QNI][i][j]);
          else
            acc[QMI][QNI][i][j] = O::mfma(af[i][s], b, acc[QMI][QNI][i][j]);
        }
    __builtin_amdgcn_s_setprio(0);
    g3_barrier();
  };

  // ---- prologue: A-lo(0), B-lo(0), B-hi(0), A-hi(0), A-lo(1), B-lo(1) in flight; retire the first two (the state
  // phase 3 of K-tile -1 would leave)
  issue_a(0, 0);
  issue_b(0, 0);
  issue_b(1, 0);
  issue_a(1, 0);
  issue_a(0, 1);
  issue_b(0, 1);
  g3_wait();
  g3_barrier();
  if (grp == 1) g3_barrier();  // stagger: group 1 runs one barrier behind group 0
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  for (int kt = 0; kt < nk; ++kt) {
    phase(I0{}, I0{}, kt);
    phase(I0{}, I1{}, kt);
    phase(I1{}, I0{}, kt);
    phase(I1{}, I1{}, kt);
  }
  if (grp == 0) g3_barrier();
  vm_wait<0>();  // trailing dummy DMAs land before the ring is reused for C staging (or the workgroup ends)
  if constexpr (FORM != G3_LDS) {
    union H4 { uint2 u; f16 h[4]; };
    // column groups (y, j): packed columns nq .. nq + 3; their bias (and per-column vectors) loaded once
    float4 cb[2][CF::FQN], cs[2][CF::FQN], ca[2][CF::FQN];
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int j = 0; j < CF::FQN; ++j) {
        const int n = min(n0 + wn * CF::WTN + y * CF::QN + j * 16 + fk * 4, a.N - 4);
        cb[y][j] = *reinterpret_cast<const float4*>(e.bias + n);
        if constexpr (FORM == G3_SPLIT) cs[y][j] = *reinterpret_cast<const float4*>(e.acc_sub + n);
        if constexpr (FORM != G3_F16) {
          if (e.add16) ca[y][j] = *reinterpret_cast<const float4*>(e.add16 + n);
        }
      }
    // G3_F16: wait for the bias here, once. Waited for inside the per-row / per-lane branches below, the compiler's
    // wait insertion (conservative where those branches join) drains every store issued before, in every row: Whisper
    // fc1 / qkv 1-2 % faster (r05ai). (The same for the residual forms' row operands measured 2-4 % slower.)
    if constexpr (FORM == G3_F16) {
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int j = 0; j < CF::FQN; ++j)
          asm volatile("" : "+v"(cb[y][j].x), "+v"(cb[y][j].y), "+v"(cb[y][j].z), "+v"(cb[y][j].w));
    }
    // RES32: add_row / acc32; SPLIT: acc16_hi / acc16_lo (host: every operand's extent < 2 GiB, 32-bit offsets)
    const void* opa = FORM == G3_SPLIT ? (const void*)e.acc16_hi : (const void*)e.add_row;
    const void* opb = FORM == G3_SPLIT ? (const void*)e.acc16_lo : (const void*)e.acc32;
    const __amdgpu_buffer_rsrc_t rs_a = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(opa ? opa : (const void*)e.bias), (short)0, opa ? 0x7fffffff : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_b = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void*>(opb ? opb : (const void*)e.bias), (short)0, opb ? 0x7fffffff : 0, 0x00020000);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < CF::FQM; ++i) {
        const int m = m0 + wm * CF::WTM + x * CF::QM + i * 16 + fr;
        if (m >= M) continue;
        const int b = m / a.T_out, t = m - b * a.T_out;
        const int64_t orow = (int64_t)b * e.T_ostore + (int64_t)t * e.ostride + e.ophase;
        // this row's residual operands for every column group, loaded before any of its stores (which may alias
        // them, so the compiler cannot move a later group's loads above an earlier group's stores)
        float4 pr[2][CF::FQN], pq[2][CF::FQN];  // RES32: add_row, acc32; SPLIT: the hi / lo halves as raw bits
        if constexpr (FORM != G3_F16) {
          // loaded through the buffer descriptors rs_a / rs_b (a missing operand's range is empty and reads 0) with no
          // branch, then waited for here, once. Loaded under `if (e.add_row)` / `if (e.acc32)` and waited for at their
          // uses, the compiler's wait insertion (its state merged at those joins and at each column group's per-lane
          // branch) put a vmcnt(0) before every column group's arithmetic, each draining the stores of the column
          // group before it (assembly, r06)
#pragma unroll
          for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int j = 0; j < CF::FQN; ++j) {
              const int n = min(n0 + wn * CF::WTN + y * CF::QN + j * 16 + fk * 4, a.N - 4);
              if constexpr (FORM == G3_SPLIT) {
                const uint32_t vo = (uint32_t)((orow * e.ld_acc + n) * 2);
                const uint2 h = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs_a, vo, 0, 0));
                const uint2 l = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs_b, vo, 0, 0));
                pq[y][j] = make_float4(__uint_as_float(h.x), __uint_as_float(h.y), __uint_as_float(l.x),
                                       __uint_as_float(l.y));
                pr[y][j] = make_float4(0.f, 0.f, 0.f, 0.f);
              } else {
                pr[y][j] = __builtin_bit_cast(
                    float4, __builtin_amdgcn_raw_buffer_load_b128(rs_a, (uint32_t)((orow * e.ld_add_row + n) * 4), 0, 0));
                pq[y][j] = __builtin_bit_cast(
                    float4, __builtin_amdgcn_raw_buffer_load_b128(rs_b, (uint32_t)((orow * e.ld_acc + n) * 4), 0, 0));
              }
            }
#pragma unroll
          for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int j = 0; j < CF::FQN; ++j) {
              asm volatile("" : "+v"(pr[y][j].x), "+v"(pr[y][j].y), "+v"(pr[y][j].z), "+v"(pr[y][j].w));
              asm volatile("" : "+v"(pq[y][j].x), "+v"(pq[y][j].y), "+v"(pq[y][j].z), "+v"(pq[y][j].w));
            }
        }
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
          for (int j = 0; j < CF::FQN; ++j) {
            const int n = n0 + wn * CF::WTN + y * CF::QN + j * 16 + fk * 4;
            if (n >= a.N) continue;
            const floatx4& c = acc[x][y][i][j];
            float4 v = make_float4(c[0] + cb[y][j].x, c[1] + cb[y][j].y, c[2] + cb[y][j].z, c[3] + cb[y][j].w);
            if constexpr (FORM == G3_F16) {
              if (e.act == ACT_GELU) {  // on value pairs (packed VALU), bit for bit gelu_erf
                const f32x2 g0 = gelu_erf2(f32x2{v.x, v.y}), g1 = gelu_erf2(f32x2{v.z, v.w});
                v = make_float4(g0.x, g0.y, g1.x, g1.y);
              } else if (e.act == ACT_RELU) {
                v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
              }
              if (n < e.scale_cols) {
                const float cs = n < e.scale_cols2 ? e.col_scale2 : e.col_scale;
                v.x *= cs; v.y *= cs; v.z *= cs; v.w *= cs;
              }
              H4 pk;
              pk.h[0] = O::enc(v.x); pk.h[1] = O::enc(v.y); pk.h[2] = O::enc(v.z); pk.h[3] = O::enc(v.w);
              f16* o = e.out16 + orow * e.ld16 + n;
              *reinterpret_cast<uint2*>(o) = pk.u;
              if (e.split16) {
                H4 lo;
                lo.h[0] = O::enc_lo(v.x - O::dec(pk.h[0])); lo.h[1] = O::enc_lo(v.y - O::dec(pk.h[1]));
                lo.h[2] = O::enc_lo(v.z - O::dec(pk.h[2])); lo.h[3] = O::enc_lo(v.w - O::dec(pk.h[3]));
                *reinterpret_cast<uint2*>(o + e.split16) = lo.u;
                *reinterpret_cast<uint2*>(o + 2 * e.split16) = pk.u;
              }
            } else {
              if constexpr (FORM == G3_RES32) {
                if (e.add_row) {
                  const float4 ar = pr[y][j];
                  v.x += ar.x; v.y += ar.y; v.z += ar.z; v.w += ar.w;
                }
              }
              float4 ac;
              bool has_acc = true;
              if constexpr (FORM == G3_SPLIT) {
                H4 hi, lo;
                hi.u = make_uint2(__float_as_uint(pq[y][j].x), __float_as_uint(pq[y][j].y));
                lo.u = make_uint2(__float_as_uint(pq[y][j].z), __float_as_uint(pq[y][j].w));
                ac.x = (O::dec(hi.h[0]) + O::dec(lo.h[0])) - cs[y][j].x;
                ac.y = (O::dec(hi.h[1]) + O::dec(lo.h[1])) - cs[y][j].y;
                ac.z = (O::dec(hi.h[2]) + O::dec(lo.h[2])) - cs[y][j].z;
                ac.w = (O::dec(hi.h[3]) + O::dec(lo.h[3])) - cs[y][j].w;
              } else {
                has_acc = e.acc32 != nullptr;
                if (has_acc) ac = pq[y][j];
              }
              if (has_acc) {
                v.x = ac.x + v.x; v.y = ac.y + v.y; v.z = ac.z + v.z; v.w = ac.w + v.w;
                if (e.acc_div != 1.0f) {
                  v.x = v.x / e.acc_div; v.y = v.y / e.acc_div; v.z = v.z / e.acc_div; v.w = v.w / e.acc_div;
                }
              }
              if constexpr (FORM == G3_RES32) {
                if (e.out32) *reinterpret_cast<float4*>(e.out32 + orow * e.ld32 + n) = v;  // may alias add_row / acc32
              }
              if (e.out16) {
                float4 w = v;
                if (e.add16) {
                  w.x += ca[y][j].x; w.y += ca[y][j].y; w.z += ca[y][j].z; w.w += ca[y][j].w;
                }
                H4 pk;
                pk.h[0] = O::enc(w.x); pk.h[1] = O::enc(w.y); pk.h[2] = O::enc(w.z); pk.h[3] = O::enc(w.w);
                *reinterpret_cast<uint2*>(e.out16 + orow * e.ld16 + n) = pk.u;
                if constexpr (FORM == G3_SPLIT) {
                  H4 lo;
                  lo.h[0] = O::enc_lo(w.x - O::dec(pk.h[0])); lo.h[1] = O::enc_lo(w.y - O::dec(pk.h[1]));
                  lo.h[2] = O::enc_lo(w.z - O::dec(pk.h[2])); lo.h[3] = O::enc_lo(w.w - O::dec(pk.h[3]));
                  *reinterpret_cast<uint2*>(e.lo16 + orow * e.ld16 + n) = lo.u;
                }
              }
            }
          }
      }
    return;
  }
  __syncthreads();

  // ---- epilogue: stage C through LDS in EP column passes, then the shared vector epilogue
  // acc[x][y][i][j][r] = C[wm*WTM + x*QM + i*16 + fk*4 + r][wn*WTN + y*QN + j*16 + fr]
  constexpr int EP = CF::EP, BNP = BN / EP, LDC = CF::LDC;
  float* Cs = reinterpret_cast<float*>(sm3);
#pragma unroll
  for (int pass = 0; pass < EP; ++pass) {
    if (wn / (CF::WNW / EP) == pass) {
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
          for (int i = 0; i < CF::FQM; ++i)
#pragma unroll
            for (int j = 0; j < CF::FQN; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                Cs[(wm * CF::WTM + x * CF::QM + i * 16 + fk * 4 + r) * LDC + wn * CF::WTN - pass * BNP + y * CF::QN +
                   j * 16 + fr] = acc[x][y][i][j][r];
    }
    __syncthreads();
    epilogue_pass<BM, BNP, LDC, CF::NT, PAIR, BF>(Cs, m0, n0 + pass * BNP, M, a, e, tid);
    __syncthreads();
  }
}

// Register epilogue form of a generic epilogue (G3_LDS when it has none). tuning gemm3_direct is a mask of the forms in
// use: 1 = G3_F16, 2 = G3_RES32, 4 = G3_SPLIT, 8 = also inside the DiffSVC sampler (run_gemm sets no_reg_epi there
// otherwise); default 3, 0 = the LDS epilogue everywhere. Alone every form is as fast or faster (Whisper fc1 12 %,
// the DiffSVC 3-tap store 12 %, skip sum 3 %); inside the 3-stream sampler the gate GEMMs beside them ran slower.
static int direct_form3(const ConvGemmArgs& a, const EpiArgs& e) {
  const int mask = tuning().gemm3_direct;
  if (e.no_reg_epi || e.col_block || e.kind != EPI_GENERIC || e.add_t) return G3_LDS;
  const bool acc16 = e.acc16_hi || e.acc16_lo || e.acc_sub || e.lo16;
  if (e.out16 && !e.out32 && !e.add_row && !e.acc32 && !acc16 && !e.add16) return (mask & 1) ? G3_F16 : G3_LDS;
  if (e.act != ACT_NONE || e.scale_cols > 0 || e.split16) return G3_LDS;
  // the residual forms read their row operands through buffer descriptors with 32-bit byte offsets
  const int64_t orows = (int64_t)a.B * e.T_ostore;
  if ((e.add_row && orows * e.ld_add_row * 4 >= (1ll << 31) - 64) ||
      ((e.acc32 || e.acc16_hi) && orows * e.ld_acc * 4 >= (1ll << 31) - 64))
    return G3_LDS;
  if (!acc16 && (e.out32 || e.out16)) return (mask & 2) ? G3_RES32 : G3_LDS;
  if (e.acc16_hi && e.acc16_lo && e.acc_sub && e.lo16 && e.out16 && !e.out32 && !e.add_row && !e.acc32)
    return (mask & 4) ? G3_SPLIT : G3_LDS;
  return G3_LDS;
}

template <int BM, int BN, bool PAIR>
static int launch3(const ConvGemmArgs& a0, const EpiArgs& e, const f16* zpage, hipStream_t s, const char* tag) {
  ConvGemmArgs a = a0;
  using CF = G3<BM, BN>;
  const int M = a.B * a.T_out;
  const int form = PAIR ? G3_LDS : direct_form3(a, e);
  a.ntiles_n = cdiv(a.N, BN);
  const int64_t grid = (int64_t)cdiv(M, BM) * a.ntiles_n;
  SVC_REQUIRE(grid > 0 && grid < (1ll << 31), "conv_gemm3: bad grid");
  SVC_REQUIRE((int64_t)a.ntiles_n * BN <= std::max(round_up(a.N, 256), round_up(a.N, 384)),
              "conv_gemm3: weights not padded for BN=%d", BN);
  // the buffer-descriptor (CP64) form: one tap per K-tile, and X / W extents addressable by 32-bit offsets
  const bool cp64 = a.Cp % 64 == 0 && a.K == a.Kpad && (int64_t)a.B * a.T_in * a.ldx * 2 < (1ll << 30) &&
                    (int64_t)a.ntiles_n * BN * a.Kpad * 2 < (1ll << 30);
  const int bf = a.bf16 ? 1 : 0;
#define G3_FORMS(BFV)                                                                                    \
  {{(const void*)conv_gemm3_kernel<BM, BN, false, PAIR, G3_LDS, BFV>,                                    \
    (const void*)conv_gemm3_kernel<BM, BN, false, false, G3_F16, BFV>,                                   \
    (const void*)conv_gemm3_kernel<BM, BN, false, false, G3_RES32, BFV>,                                 \
    (const void*)conv_gemm3_kernel<BM, BN, false, false, G3_SPLIT, BFV>},                                \
   {(const void*)conv_gemm3_kernel<BM, BN, true, PAIR, G3_LDS, BFV>,                                     \
    (const void*)conv_gemm3_kernel<BM, BN, true, false, G3_F16, BFV>,                                    \
    (const void*)conv_gemm3_kernel<BM, BN, true, false, G3_RES32, BFV>,                                  \
    (const void*)conv_gemm3_kernel<BM, BN, true, false, G3_SPLIT, BFV>}}
  const void* fns[2][2][4] = {G3_FORMS(false), G3_FORMS(true)};
#undef G3_FORMS
  const void* fn = fns[bf][cp64][form];
  // the register forms need only the operand ring (no C staging)
  const int lds = form == G3_LDS ? CF::LDS : CF::RING;
  if (int st = ensure_dyn_lds(fn, lds)) return st;
  const double kreal = (double)(a.K / a.Cp) * a.Cvalid;
  const int tok = prof_begin(tag, 2.0 * M * (double)a.N * kreal, 0.0, s);
  const float inv = 1.0f / (float)a.Cp;
  void* args[] = {&a, const_cast<EpiArgs*>(&e), const_cast<const f16**>(&zpage), const_cast<float*>(&inv)};
  SVC_HIP_CHECK(hipLaunchKernel(fn, dim3((unsigned)grid), dim3(CF::NT), args, lds, s));
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// Tile choice: estimated time = rounds of workgroups over the CUs x cost of one round, in units of a
// 256x256 round, fitted to tools/gemm_bench.py on MI355X (profiles/r01_gemm_bench.txt):
//   256x128 / 128x256 0.62; 128x384 0.87 (N = 384 without the 256-wide tile's idle half);
//   128x128 0.6, or 0.4 when K <= 512 where the fixed prologue/epilogue share dominates. 128x128 needs
//   68 KiB of LDS, so two workgroups share a CU (512 slots). 256x192 (index 6, 4 x 2 waves): only where N is
//   a multiple of 192 and of neither 256 nor 384 (the BigVGAN C = 192 convs: k = 11 977 -> 885-893 us against the
//   256x256 tile's 64 idle columns; at N = 384 it ran 5 % behind 128x384, r05af)
static int pick3(int M, int N, int Kpad) {
  const int bms[6] = {256, 128, 256, 128, 128, 256}, bns[6] = {256, 256, 128, 128, 384, 192};
  const double cost[6] = {1.0, 0.62, 0.62, Kpad <= 512 ? 0.4 : 0.6, 0.87, 0.78};
  const int slots[6] = {256, 256, 256, 512, 256, 256};
  const int nv = (N % 192 == 0 && N % 256 != 0 && N % 384 != 0) ? 6 : 5;
  int best = 0;
  double best_t = 1e300;
  for (int v = 0; v < nv; ++v) {
    const int64_t tiles = (int64_t)cdiv(M, bms[v]) * cdiv(N, bns[v]);
    const double t = (double)cdiv64(tiles, slots[v]) * cost[v];
    if (t < best_t - 1e-9) {
      best_t = t;
      best = v;
    }
  }
  return best == 5 ? 6 : best;
}

int conv_gemm3(const ConvGemmArgs& a, const EpiArgs& e, const f16* zpage, int variant, hipStream_t s) {
  SVC_REQUIRE(a.Cp % 8 == 0 && a.ldx % 8 == 0 && a.Kpad % 64 == 0 && a.N % 4 == 0, "conv_gemm3: layout");
  SVC_REQUIRE(e.ld32 % 4 == 0 && e.ld16 % 4 == 0 && e.ld_add_row % 4 == 0 && e.ld_acc % 4 == 0 && e.ld_add_t % 4 == 0 &&
                  e.ld_cp % 4 == 0 && e.ldy16 % 4 == 0 && e.ld_emb % 4 == 0,
              "conv_gemm3: epilogue leading dimensions must be multiples of 4 (vector epilogue)");
  SVC_REQUIRE(((uintptr_t)a.X & 15) == 0 && ((uintptr_t)a.W & 15) == 0, "conv_gemm3: 16-B alignment");
  // column blocks (EpiArgs::col_block) re-address the out16 high-half store only
  SVC_REQUIRE(!e.col_block || (!e.lo16 && !e.split16 && !e.out32), "conv_gemm3: col_block with lo16 / split16 / out32");
  const int M = a.B * a.T_out;
  const int v = ((variant >= 0 && variant < 5) || variant == 6) ? variant : pick3(M, a.N, a.Kpad);
  if (e.kind == EPI_GATE) {
    SVC_REQUIRE(a.N % 64 == 0, "conv_gemm3: paired epilogue needs N %% 64 == 0");
    switch (v) {
      case 6:  // (the 256 x 192 tile's epilogue passes split the 64-column gate | filter blocks: the 256 x 256 tile)
      case 0: return launch3<256, 256, true>(a, e, zpage, s, "conv_gemm3<256,256,pair>");
      case 1: return launch3<128, 256, true>(a, e, zpage, s, "conv_gemm3<128,256,pair>");
      case 2: return launch3<256, 128, true>(a, e, zpage, s, "conv_gemm3<256,128,pair>");
      case 4: return launch3<128, 384, true>(a, e, zpage, s, "conv_gemm3<128,384,pair>");
      default: return launch3<128, 128, true>(a, e, zpage, s, "conv_gemm3<128,128,pair>");
    }
  }
  switch (v) {
    case 0: return launch3<256, 256, false>(a, e, zpage, s, "conv_gemm3<256,256>");
    case 1: return launch3<128, 256, false>(a, e, zpage, s, "conv_gemm3<128,256>");
    case 2: return launch3<256, 128, false>(a, e, zpage, s, "conv_gemm3<256,128>");
    case 4: return launch3<128, 384, false>(a, e, zpage, s, "conv_gemm3<128,384>");
    case 6: return launch3<256, 192, false>(a, e, zpage, s, "conv_gemm3<256,192>");
    default: return launch3<128, 128, false>(a, e, zpage, s, "conv_gemm3<128,128>");
  }
}

}  // namespace svc
