// DiffSVC residual layer with the rows held still (modules/diffsvc.py:212-232, ResidualBlock.forward), round 5.
//
// gate_ws.hip keeps the dilated conv's weights still (in VGPRs, 6 column groups x 42 row parts) and streams the rows;
// the residual projection then needs a second launch, because a row's 384 gate outputs come from six workgroups. Here a
// workgroup owns a tile of 8 row blocks (128 rows) for the whole layer and streams the weights instead:
//   * prologue: the tile's input rows (the split residual stream's high half, x + dproj_l) plus 8 halo rows each side go
//     to LDS once (LDS-DMA, 144 rows at an 800-B stride: conflict-free 16-row fragment reads at any tap shift);
//   * gate GEMM in 3 passes of 256 packed columns: in pass P wave w owns one gate / filter column pair (16 + 16 columns
//     of packed block q = 4 P + w / 2) for all 128 rows: 8 row blocks x 2 accumulators; per 32-deep K-step it reads the
//     8 A fragments of the step's tap from the image and its two 1-KiB weight fragments from L2 (gate_ws_pack order,
//     loaded three K-steps ahead), and issues 16 v_mfma_f32_16x16x32 with the operands swapped (a lane holds 4
//     consecutive channels of one row, gate and filter of a channel in the same lane). The K order (K-steps 0..35 on
//     one accumulator) and the gate arithmetic are gate_ws's / conv_gemm4's, so g is bit-identical;
//   * the pass's gate epilogue: the conditioner projection (loaded during the last K-steps), the gate, f16 g stores.
// Per CU and layer the weights cross L2 -> L1 once (1.77 MB; the 8 waves read disjoint fragments) while each input row is
// read from HBM once plus the halo: 768 B of A per row against gate_ws's 6 column-group re-reads from L2.
// Zero padding: an (output row, tap) whose input frame lies outside its utterance (or past a ragged utterance's valid
// rows, tv) reads its fragments from a zero row (per-lane address select at each tap change).
#include <type_traits>

#include "common.h"

namespace svc {

constexpr int DL_C = 384;
constexpr int DL_KS = 36;                   // K-steps of 32 (3 taps x 12 channel chunks)
constexpr int DL_NB = 8;                    // 16-row blocks per tile
constexpr int DL_HALO = 8;                  // largest tap shift (dilation 8)
constexpr int DL_IROWS = DL_NB * 16 + 2 * DL_HALO;  // 144 image rows
constexpr int DL_STRIDE = 800;              // 768 B + 32 B: 16-row fragment reads conflict-free at any row offset
constexpr int DL_UNITS = DL_IROWS * 50;     // 16-B units of the image (48 data + 2 pad per row)
constexpr int DL_PIECES = (DL_UNITS + 63) / 64;  // 113 LDS-DMA wave-instructions
constexpr int DL_ZERO = DL_PIECES * 1024;   // 800 B of zeros (past the last piece)
constexpr int DL_TVT = DL_ZERO + DL_STRIDE;
constexpr int DL_MAXB = 1024;
constexpr int DL_SLAB_STRIDE = 288;        // g slab row: 128 channels (256 B) + 32 B, conflict-free fragment reads
constexpr int DL_SLAB = DL_NB * 16 * DL_SLAB_STRIDE;  // 36,864 B per 128-channel slab
constexpr int DL_SLAB0 = DL_TVT + DL_MAXB * 4;         // slab 0 past the image (written during the gate passes)
constexpr int DL_LDS_GATE = DL_SLAB0;
constexpr int DL_LDS = DL_SLAB0 + DL_SLAB;             // with the projection: slabs 1 and 2 reuse the image
constexpr int DL_NT = 512;
constexpr int DL_PF = 3;                    // weight fragments loaded this many K-steps ahead
static_assert(DL_KS % (DL_PF + 1) == 0, "the weight ring slot of K-step s of every pass is s % (DL_PF + 1)");
constexpr uint32_t DL_OOR = 0x80000000u;    // past every descriptor's range: loads return 0, stores drop
constexpr uint32_t DL_CFG = 0x00020000u;

struct DLayerArgs {
  const f16* X;       // [M][384] layer input: the split residual stream's high half
  const f16* W;       // dilated conv weights in gate_ws_pack fragment order
  const float* bias;  // [768] packed
  const f16* cp;      // [M][ld_cp] conditioner projection (packed order)
  int ld_cp;
  f16* y;             // [M][ldy] gate output g
  int ldy;
  int M, T, dil;
  const int* tv;      // ragged: utterance b has min(T, tv[b] * tv_mul) valid input rows (NULL = T)
  int tv_mul, B;
  float invT;
  // the residual half of output_projection (PROJ): x' = (((hi + lo) - sub) + g W_res^T + b_res) / sqrt(2),
  // hi_out = f16(x' + add), lo = f16((x' + add) - hi_out) (res_proj.hip's arithmetic); hi_out is not X (neighbouring
  // tiles read X's rows as their halo), lo is updated in place (only its own tile reads it)
  const f16* Wr;      // W_res in res_proj_pack fragment order
  const float* br;    // [384]
  const float* sub;   // dproj_i
  const float* add;   // dproj_{i+1}
  f16* hi_out;
  f16* lo;
};

// W fragment (gate_ws_pack): column group c, pair p, K-step ks, gate / filter g; 512 halves = 1 KiB per wave
__device__ __forceinline__ size_t dl_frag(int c, int p, int ks, int g) {
  return (size_t)(((c * 4 + p) * DL_KS + ks) * 2 + g) * 512;
}

template <bool BF, bool PROJ>
__global__ __launch_bounds__(DL_NT, 1) void dlayer_kernel(DLayerArgs a) {
  using O = Op16<BF>;
  extern __shared__ __align__(16) unsigned char sm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fk = lane >> 4;
  const int nblk = (a.M + 15) >> 4;
  const int blk0 = blockIdx.x * DL_NB;
  if (blk0 >= nblk) return;
  const int r_begin = blk0 * 16, r_end = min(a.M, r_begin + DL_NB * 16);

  int* tvt = reinterpret_cast<int*>(sm + DL_TVT);
  for (int i = tid; i < a.B; i += DL_NT) tvt[i] = a.tv ? min(a.T, a.tv[i] * a.tv_mul) : a.T;
  for (int i = tid; i < DL_STRIDE / 16; i += DL_NT) *reinterpret_cast<uint4*>(sm + DL_ZERO + i * 16) = make_uint4(0, 0, 0, 0);
  {
    // image unit u (16 B) = image row u / 50, chunk u % 50 (48, 49: the row's padding) of input row r_begin - 8 + row;
    // rows outside [0, M) fall outside the descriptor's range and land as zeros
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(a.X), (short)0, a.M * DL_C * 2, DL_CFG);
    for (int p = wave; p < DL_PIECES; p += DL_NT / 64) {
      const int u = p * 64 + lane, ir = u / 50, ch = u - ir * 50;
      const int src = r_begin - DL_HALO + ir;
      const uint32_t vo = (ch < 48 && u < DL_UNITS && src >= 0) ? (uint32_t)src * (DL_C * 2) + ch * 16 : DL_OOR;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(sm + p * 1024), 16,
                                               (int)vo, 0, 0, 0);
    }
  }
  // valid-tap bits of the lane's 8 rows: bit 3 i + tap <=> input frame t_i + (tap - 1) dil lies in [0, tvb_i)
  uint32_t vmask = 0;
  __syncthreads();  // (the length table)
  {
    int m = r_begin + fr;
    int bb = (int)((float)m * a.invT);
    int t = m - bb * a.T;
    if (t < 0) {
      --bb;
      t += a.T;
    } else if (t >= a.T) {
      ++bb;
      t -= a.T;
    }
#pragma unroll
    for (int i = 0; i < DL_NB; ++i) {
      const int tvb = tvt[min(bb, a.B - 1)];
#pragma unroll
      for (int tap = 0; tap < 3; ++tap) {
        const int tp = t + (tap - 1) * a.dil;
        if (m < a.M && tp >= 0 && tp < tvb) vmask |= 1u << (3 * i + tap);
      }
      m += 16;
      t += 16;
      if (t >= a.T) {  // T >= 16: at most one utterance boundary per block
        t -= a.T;
        ++bb;
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): this wave's image pieces have landed
  __syncthreads();                      // ... and every wave's

  const int lane_base = (fr + DL_HALO) * DL_STRIDE + fk * 16;  // image bytes of block 0, row fr, the lane's 16-B chunk
  const int zero_base = DL_ZERO + fk * 16;
  const __amdgpu_buffer_rsrc_t rcp =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(a.cp), (short)0, a.M * a.ld_cp * 2, DL_CFG);
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(a.y, (short)0, a.M * a.ldy * 2, DL_CFG);

  union H4 { uint2 u; f16 h[4]; };
  H4 gk[2][DL_NB];  // (PROJ) the lane's g of passes 1 and 2, for the projection's slabs 1 and 2
  // the wave's weight fragments as one stream over the 3 passes (global K-step 36 P + s, ring slot s % 4): the first
  // K-steps of pass P + 1 are loaded during pass P's last ones
  const auto wbase = [&](int P) { return a.W + dl_frag(2 * P + (wave >> 2), wave & 3, 0, 0) + lane * 8; };
  // pass order rotated by workgroup: the CUs of an XCD then stream three different weight slices at a time instead of
  // all requesting the same 16 KiB per K-step from the same L2 channels
  const int rot = blockIdx.x % 3;
  half8 wg[DL_PF + 1], wf[DL_PF + 1];
  {
    const f16* wb0 = wbase(rot);
#pragma unroll
    for (int s = 0; s < DL_PF; ++s) {
      wg[s] = *reinterpret_cast<const half8*>(wb0 + (size_t)(2 * s) * 512);
      wf[s] = *reinterpret_cast<const half8*>(wb0 + (size_t)(2 * s + 1) * 512);
    }
  }
  for (int n = 0; n < 3; ++n) {
    const int P = n + rot < 3 ? n + rot : n + rot - 3;
    const int c = 2 * P + (wave >> 2), pr = wave & 3;
    const int q = 2 * c + (pr >> 1), h = pr & 1;
    const int ng = 64 * q + 16 * h, nf = ng + 32;
    const int chn = 32 * q + 16 * h + 4 * fk;  // the lane's 4 output channels
    const f16* wb = wbase(P);
    const f16* wbn = wbase(P < 2 ? P + 1 : 0);
    floatx4 ag[DL_NB], af[DL_NB];
#pragma unroll
    for (int i = 0; i < DL_NB; ++i) {
      ag[i] = floatx4{0.f, 0.f, 0.f, 0.f};
      af[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    H4 cpg[DL_NB], cpf[DL_NB];
    int addr[DL_NB];
    const auto set_addr = [&](int tap) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < DL_NB; ++i)
        addr[i] = (vmask >> (3 * i + tap)) & 1u ? lane_base + (i * 16 + (tap - 1) * a.dil) * DL_STRIDE : zero_base;
    };
    // A fragments double-buffered: K-step s + 1's reads are issued in step s's scheduling segment, ahead of its MFMAs
    half8 av[2][DL_NB];
    const auto read_a = [&](int s, half8* dst) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < DL_NB; ++i) dst[i] = *reinterpret_cast<const half8*>(sm + addr[i] + (s % 12) * 64);
    };
    set_addr(0);
    read_a(0, av[0]);
#pragma unroll
    for (int s = 0; s < DL_KS; ++s) {
      // one scheduling segment per K-step (left alone the compiler hoisted the weight loads of many K-steps and spilled)
      __builtin_amdgcn_sched_barrier(0);
      if (s + DL_PF < DL_KS) {
        wg[(s + DL_PF) % (DL_PF + 1)] = *reinterpret_cast<const half8*>(wb + (size_t)(2 * (s + DL_PF)) * 512);
        wf[(s + DL_PF) % (DL_PF + 1)] = *reinterpret_cast<const half8*>(wb + (size_t)(2 * (s + DL_PF) + 1) * 512);
      } else if (n < 2) {
        const int sn = s + DL_PF - DL_KS;
        wg[(s + DL_PF) % (DL_PF + 1)] = *reinterpret_cast<const half8*>(wbn + (size_t)(2 * sn) * 512);
        wf[(s + DL_PF) % (DL_PF + 1)] = *reinterpret_cast<const half8*>(wbn + (size_t)(2 * sn + 1) * 512);
      }
      // the conditioner projection of the pass's rows, for the epilogue (rows past M read 0), right after the pass's
      // last weight fragments: vmcnt retires in issue order, so a weight load issued behind these HBM loads would wait
      // for them (only the next pass's first fragments, which the epilogue precedes anyway, come later)
      if (s == DL_KS - DL_PF - 1) {
#pragma unroll
        for (int i = 0; i < DL_NB; ++i) {
          const uint32_t vo = (uint32_t)(r_begin + i * 16 + fr) * (uint32_t)(a.ld_cp * 2);
          cpg[i].u = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rcp, vo + (ng + 4 * fk) * 2, 0, 0));
          cpf[i].u = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rcp, vo + (nf + 4 * fk) * 2, 0, 0));
        }
      }
      if (s + 1 < DL_KS) {
        if ((s + 1) % 12 == 0) set_addr((s + 1) / 12);
        read_a(s + 1, av[(s + 1) & 1]);
      }
      const half8 g0 = wg[s % (DL_PF + 1)], f0 = wf[s % (DL_PF + 1)];
#pragma unroll
      for (int i = 0; i < DL_NB; ++i) {
        ag[i] = O::mfma(g0, av[s & 1][i], ag[i]);
        af[i] = O::mfma(f0, av[s & 1][i], af[i]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // gate epilogue (gate_ws's / conv_gemm4's DIRECT arithmetic, same order); rows past the tile are not stored
    const float4 bg = *reinterpret_cast<const float4*>(a.bias + ng + 4 * fk);
    const float4 bfv = *reinterpret_cast<const float4*>(a.bias + nf + 4 * fk);
    const float bga[4] = {bg.x, bg.y, bg.z, bg.w}, bfa[4] = {bfv.x, bfv.y, bfv.z, bfv.w};
#pragma unroll
    for (int i = 0; i < DL_NB; ++i) {
      H4 pk;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        pk.h[e] = O::enc_lo(gate_act(ag[i][e] + bga[e] + O::dec(cpg[i].h[e]), af[i][e] + bfa[e] + O::dec(cpf[i].h[e])));
      const int m = r_begin + i * 16 + fr;
      const uint32_t vo = m < r_end ? (uint32_t)m * (uint32_t)(a.ldy * 2) + (uint32_t)chn * 2 : DL_OOR;
      buffer_store_b64(pk.u, ry, vo);
      if constexpr (PROJ) {
        // g of pass P = K-steps 4P .. 4P + 3 of the projection, row 16 i + fr, channels chn - 128 P: the first pass's
        // slab goes past the image now, the others' after the gate passes (over the image)
        if (n == 0)
          *reinterpret_cast<uint2*>(sm + DL_SLAB0 + (i * 16 + fr) * DL_SLAB_STRIDE + (chn - 128 * P) * 2) = pk.u;
        else
          gk[n - 1][i] = pk;
      }
    }
  }
  if constexpr (PROJ) {
    // ---- residual projection of the tile's rows: out = g W_res^T (K = 384 = 12 K-steps, slab kc / 4), wave w owns
    // output columns 48 w .. 48 w + 47 (res_proj_pack blocks nb = 3 w + j); two halves of 4 row blocks each
    H4 hv[DL_NB][3];  // the lane's hi (x + dproj_i, high half) at its output columns, from the image before it is reused
#pragma unroll
    for (int i = 0; i < DL_NB; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        hv[i][j].u = *reinterpret_cast<const uint2*>(sm + (DL_HALO + i * 16 + fr) * DL_STRIDE +
                                                     (48 * wave + 16 * j + 4 * fk) * 2);
    __syncthreads();  // every wave is done with the image: slabs 1 and 2 go over it
#pragma unroll
    for (int n = 1; n < 3; ++n) {
      const int P = n + rot < 3 ? n + rot : n + rot - 3;
      const int chn = 32 * (4 * P + (wave >> 1)) + 16 * (wave & 1) + 4 * fk;
#pragma unroll
      for (int i = 0; i < DL_NB; ++i)
        *reinterpret_cast<uint2*>(sm + (n - 1) * DL_SLAB + (i * 16 + fr) * DL_SLAB_STRIDE + (chn - 128 * P) * 2) =
            gk[n - 1][i].u;
    }
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rhi = __builtin_amdgcn_make_buffer_rsrc(a.hi_out, (short)0, a.M * DL_C * 2, DL_CFG);
    const __amdgpu_buffer_rsrc_t rlo = __builtin_amdgcn_make_buffer_rsrc(a.lo, (short)0, a.M * DL_C * 2, DL_CFG);
    const auto slab = [rot](int kc) {  // the slab of pass kc / 4 (processed n-th)
      const int n = (kc / 4 - rot + 3) % 3;
      return n == 0 ? DL_SLAB0 : (n - 1) * DL_SLAB;
    };
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      __builtin_amdgcn_sched_barrier(0);
      H4 lv[4][3];  // lo of the half's rows at the lane's columns (HBM), loaded under the K-loop
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const uint32_t row = (uint32_t)(r_begin + (4 * hf + ii) * 16 + fr) * (DL_C * 2);
#pragma unroll
        for (int j = 0; j < 3; ++j)
          lv[ii][j].u = __builtin_bit_cast(
              uint2, __builtin_amdgcn_raw_buffer_load_b64(rlo, row + (48 * wave + 16 * j + 4 * fk) * 2, 0, 0));
      }
      floatx4 acc[4][3];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[ii][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < 12; ++kc) {
        __builtin_amdgcn_sched_barrier(0);
        half8 wr[3], am[4];
#pragma unroll
        for (int j = 0; j < 3; ++j)
          wr[j] = *reinterpret_cast<const half8*>(a.Wr + (size_t)((3 * wave + j) * 12 + kc) * 512 + lane * 8);
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
          am[ii] = *reinterpret_cast<const half8*>(sm + slab(kc) + ((4 * hf + ii) * 16 + fr) * DL_SLAB_STRIDE +
                                                  (kc % 4) * 64 + fk * 16);
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int j = 0; j < 3; ++j) acc[ii][j] = O::mfma(wr[j], am[ii], acc[ii][j]);
      }
      __builtin_amdgcn_sched_barrier(0);
      // split-residual update (res_proj.hip's arithmetic, same order)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int n0 = 48 * wave + 16 * j + 4 * fk;
        const float4 bi = *reinterpret_cast<const float4*>(a.br + n0);
        const float4 sb = *reinterpret_cast<const float4*>(a.sub + n0);
        const float4 ad = *reinterpret_cast<const float4*>(a.add + n0);
        const float b4[4] = {bi.x, bi.y, bi.z, bi.w}, s4[4] = {sb.x, sb.y, sb.z, sb.w}, a4[4] = {ad.x, ad.y, ad.z, ad.w};
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          const int i = 4 * hf + ii;
          H4 ph, pl;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = acc[ii][j][r] + b4[r];
            const float x = div_sqrt2_exact(((O::dec(hv[i][j].h[r]) + O::dec(lv[ii][j].h[r])) - s4[r]) + v);
            const float wv = x + a4[r];
            ph.h[r] = O::enc(wv);
            pl.h[r] = O::enc_lo(wv - O::dec(ph.h[r]));
          }
          const int m = r_begin + i * 16 + fr;
          const uint32_t vo = m < r_end ? (uint32_t)m * (DL_C * 2) + (uint32_t)n0 * 2 : DL_OOR;
          buffer_store_b64(ph.u, rhi, vo);
          buffer_store_b64(pl.u, rlo, vo);
        }
      }
    }
  }
}

bool dlayer_fits(const ConvGemmArgs& a, const EpiArgs& e) {
  const int d = a.tap_mul;
  return a.Wfrag && e.kind == EPI_GATE && e.cp && e.y16 && e.bias && a.Cp == DL_C && a.Cvalid == DL_C &&
         a.ldx == DL_C && a.K == 3 * DL_C && a.Kpad == 3 * DL_C && a.N == 2 * DL_C &&
         (d == 1 || d == 2 || d == 4 || d == 8) && a.tap_add == -d && a.istride == 1 && a.T_in == a.T_out &&
         a.T_out >= 16 && a.B <= DL_MAXB && e.ld_cp % 4 == 0 && e.ldy16 % 4 == 0 &&
         (int64_t)a.B * a.T_out * std::max(e.ld_cp, std::max(e.ldy16, DL_C)) * 2 < (1ll << 30);
}

// the gate alone (the last layer, or run_gemm's dispatch) or, with pr (PROJ), the whole residual layer
int dlayer(const ConvGemmArgs& a, const EpiArgs& e, hipStream_t s, const DLayerProj* pr) {
  SVC_REQUIRE(dlayer_fits(a, e), "dlayer: not the DiffSVC dilated-conv gate shape");
  SVC_REQUIRE(((uintptr_t)a.X & 15) == 0 && ((uintptr_t)a.Wfrag & 15) == 0 && ((uintptr_t)e.cp & 7) == 0 &&
                  ((uintptr_t)e.y16 & 7) == 0 && ((uintptr_t)e.bias & 15) == 0,
              "dlayer: alignment");
  SVC_REQUIRE(!pr || (pr->Wr && pr->br && pr->sub && pr->add && pr->hi_out && pr->lo && pr->hi_out != a.X &&
                      ((uintptr_t)pr->hi_out & 7) == 0 && ((uintptr_t)pr->lo & 7) == 0 && ((uintptr_t)pr->Wr & 15) == 0),
              "dlayer: projection arguments (hi_out must not be the layer input)");
  const int M = a.B * a.T_out;
  if (M == 0) return SVC_OK;
  DLayerArgs g{a.X, a.Wfrag, e.bias, e.cp, e.ld_cp, e.y16, e.ldy16, M, a.T_out, a.tap_mul, a.tv, a.tv_mul, a.B,
               1.0f / (float)a.T_out};
  if (pr) {
    g.Wr = pr->Wr; g.br = pr->br; g.sub = pr->sub; g.add = pr->add; g.hi_out = pr->hi_out; g.lo = pr->lo;
  }
  const void* fn = pr ? (a.bf16 ? (const void*)dlayer_kernel<true, true> : (const void*)dlayer_kernel<false, true>)
                      : (a.bf16 ? (const void*)dlayer_kernel<true, false> : (const void*)dlayer_kernel<false, false>);
  const int lds = pr ? DL_LDS : DL_LDS_GATE;
  if (int st = ensure_dyn_lds(fn, lds)) return st;
  const int grid = cdiv(cdiv(M, 16), DL_NB);
  const double flops = 2.0 * M * (double)(2 * DL_C) * (3 * DL_C) + (pr ? 2.0 * M * DL_C * DL_C : 0.0);
  const int tok = prof_begin(pr ? "dlayer<128x768+proj>" : "dlayer<128x768>", flops, 0.0, s);
  void* args[] = {&g};
  SVC_HIP_CHECK(hipLaunchKernel(fn, dim3(grid), dim3(DL_NT), args, lds, s));
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
