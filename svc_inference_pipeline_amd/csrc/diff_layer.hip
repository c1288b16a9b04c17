// Fused DiffSVC residual layer for gfx950 (modules/diffsvc.py:192-232, ResidualBlock.forward), one launch per layer:
//
//   y  = sigmoid(gate) * tanh(filter),  [gate | filter] = dilated_conv_k3,d(x + dproj_l) + conditioner_proj(cond)
//   x' = (x + output_projection_residual(y)) / sqrt(2),   next input = x' + dproj_{l+1},   y -> skip operand
//
// One workgroup owns 64 time rows and ALL 768 gate/filter columns, so the gate, the 384x384 residual projection and
// the residual update happen on chip: the gate output never makes an HBM round trip before the projection, and the
// two GEMMs of a layer share one launch (the unfused path is conv_gemm3 GATE + conv_gemm3 residual epilogue).
//
//   GEMM1  [64 x 1152] x [1152 x 768]: 36 K-steps of 32. LDS stage = A image (64 rows x 64 B) + B image (768 rows x
//          64 B), 2 stages filled by LDS-DMA (global_load_lds_dwordx4; 16-B chunk swizzle kc ^ ((row >> 2) & 3) on the
//          source address makes the fragment ds_read_b128s conflict-free). 8 waves = 1 (M) x 8 (N): wave tile 64 x 96 =
//          4 x 6 fragments of v_mfma_f32_16x16x32_f16. Weights are packed in "pair16" order: packed column n is the
//          gate (n & 16 == 0) or filter half of channel (n >> 5) * 16 + (n & 15), so a lane's gate accumulator and its
//          filter accumulator sit in fragments 2jp and 2jp+1 at the same (row, channel): the gate is applied in
//          registers. The conditioner projection (+ dilated bias) comes in a fragment-major layout (16 B per lane).
//   y tile 64 x 384 f16 in LDS (chunk swizzle kc ^ (row & 15)), copied to the skip buffer with 16-B stores.
//   GEMM2  [64 x 384] x [384 x 384] (residual half of output_projection): A = y tile from LDS, B streamed by LDS-DMA
//          in 12 K-steps; wave tile 64 x 48. Epilogue: x' = (x + z + b) / sqrt(2) in place (f32), next input
//          f16(x' + dproj_{l+1}) staged through LDS and stored as 16-B row vectors.
#include "common.h"

namespace svc {

struct DiffLayerArgs {
  const f16* x16;    // [M][C] layer input x + dproj_l (row-major; A operand, read through tap shifts)
  const f16* Wd;     // [2C][3C] pair16-packed dilated conv (K index tap * C + c)
  const f16* cpF;    // fragment-major conditioner projection + dilated bias of this layer
  const f16* Wo;     // [C][C] residual half of output_projection (row = out channel)
  const float* bo;   // [C]
  const float* dpn;  // [C] next layer's diffusion projection
  float* x32;        // [M][C] residual stream (read + written when OUT)
  f16* x16n;         // [M][C] next layer input (OUT)
  f16* g16;          // gate output rows (skip-GEMM operand), row stride ldg
  int ldg;
  int B, T, dil;
  const f16* zpage;  // >= 1 KiB of zeros (DMA source of padded rows)
};

constexpr int DL_C = 384, DL_BM = 64;
constexpr int DL_N = 2 * DL_C;
constexpr int DL_K1 = 3 * DL_C;                    // 1152
constexpr int DL_A_BYTES = DL_BM * 64;             // 4 KiB
constexpr int DL_B_BYTES = DL_N * 64;              // 48 KiB
constexpr int DL_STAGE = DL_A_BYTES + DL_B_BYTES;  // 52 KiB
constexpr int DL_RING = 2 * DL_STAGE;              // 104 KiB
constexpr int DL_DUMMY = 4096;                     // sink of waves 4..7's A-slot DMAs (uniform vmcnt)
constexpr int DL_Y_OFF = DL_RING + DL_DUMMY;
constexpr int DL_Y_BYTES = DL_BM * DL_C * 2;       // 48 KiB
constexpr int DL_LDS = DL_Y_OFF + DL_Y_BYTES;      // 156 KiB
static_assert(DL_LDS <= 163840, "LDS budget");

__device__ __forceinline__ void dl_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void dl_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void dl_dma(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// byte offset of 16-B chunk kc of row `row` in a 64-B-row image
__device__ __forceinline__ int img64(int row, int kc) { return row * 64 + ((kc ^ ((row >> 2) & 3)) << 4); }
// byte offset of 16-B chunk kc (0..47) of row `row` in the 64 x 384 f16 y / output tile
__device__ __forceinline__ int ytile(int row, int kc) { return row * (DL_C * 2) + ((kc ^ (row & 15)) << 4); }

template <bool OUT>
__global__ __launch_bounds__(512, 1) void diff_layer_kernel(DiffLayerArgs p) {
  extern __shared__ __align__(16) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fk = lane >> 4;
  const int M = p.B * p.T;
  const int m0 = blockIdx.x * DL_BM;
  const f16* zsrc = p.zpage + (lane & 63) * 8;

  // ---- GEMM1 DMA slots: A (waves 0..3 own image rows 16w..16w+15), B (6 instructions per wave)
  const int a_row = (w & 3) * 16 + (lane >> 2);
  const int a_kc = (lane & 3) ^ ((a_row >> 2) & 3);
  int a_t = -(1 << 29);
  const f16* a_base = p.x16;
  {
    const int m = m0 + a_row;
    if (w < 4 && m < M) {
      const int b = m / p.T;
      a_t = m - b * p.T;
      a_base = p.x16 + (int64_t)b * p.T * DL_C + a_kc * 8;
    }
  }
  unsigned char* a_dst0 = lds + (w < 4 ? w * 1024 : DL_Y_OFF - DL_DUMMY);  // waves 4..7: dummy sink
  const f16* b_src[6];
#pragma unroll
  for (int v = 0; v < 6; ++v) {
    const int n = (w * 6 + v) * 16 + (lane >> 2);
    b_src[v] = p.Wd + (int64_t)n * DL_K1 + (((lane & 3) ^ ((n >> 2) & 3)) * 8);
  }
  auto issue1 = [&](int k) {
    unsigned char* st = lds + (k & 1) * DL_STAGE;
    const int tap = k / (DL_C / 32), c0 = (k - tap * (DL_C / 32)) * 32;
    const int t = a_t + (tap - 1) * p.dil;
    const bool ok = t >= 0 && t < p.T;
    dl_dma(ok ? (const void*)(a_base + (int64_t)t * DL_C + c0) : (const void*)zsrc,
           w < 4 ? st + w * 1024 : a_dst0);
    unsigned char* bst = st + DL_A_BYTES + w * 6 * 1024;
#pragma unroll
    for (int v = 0; v < 6; ++v) dl_dma(b_src[v] + k * 32, bst + v * 1024);
  };

  floatx4 acc[4][6];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  constexpr int NK1 = DL_K1 / 32;  // 36
  issue1(0);
  for (int k = 0; k < NK1; ++k) {
    if (k + 1 < NK1) {
      issue1(k + 1);
      dl_vmwait<7>();
    } else {
      dl_vmwait<0>();
    }
    dl_barrier();
    const unsigned char* A = lds + (k & 1) * DL_STAGE;
    const unsigned char* Bm = A + DL_A_BYTES;
    half8 af[4], bf[6];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const half8*>(A + img64(i * 16 + fr, fk));
#pragma unroll
    for (int j = 0; j < 6; ++j) bf[j] = *reinterpret_cast<const half8*>(Bm + img64(w * 96 + j * 16 + fr, fk));
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    dl_barrier();
  }

  // ---- gate in registers: acc[i][2jp] = gate, acc[i][2jp+1] = filter of channel w*48 + jp*16 + fr,
  // rows i*16 + fk*4 + r. cpF record (16 B per lane) = {gate, filter} x 4 rows.
  const int rb0 = m0 / 16;
  uint4 cpr[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jp = 0; jp < 3; ++jp)
      cpr[i][jp] = *reinterpret_cast<const uint4*>(
          p.cpF + ((((int64_t)(rb0 + i) * (DL_C / 16) + (w * 3 + jp)) * 64 + lane) * 8));
  float xr[OUT ? 4 : 1][OUT ? 3 : 1][4];  // residual stream values at the GEMM2 accumulator positions
  if constexpr (OUT) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + i * 16 + fk * 4 + r;
#pragma unroll
        for (int j = 0; j < 3; ++j) xr[i][j][r] = m < M ? p.x32[(int64_t)m * DL_C + w * 48 + j * 16 + fr] : 0.f;
      }
  }
  unsigned char* Y = lds + DL_Y_OFF;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jp = 0; jp < 3; ++jp) {
      union { uint4 u; f16 h[8]; } cp;
      cp.u = cpr[i][jp];
      const int ch = w * 48 + jp * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float g = acc[i][2 * jp][r] + (float)cp.h[2 * r];
        const float f = acc[i][2 * jp + 1][r] + (float)cp.h[2 * r + 1];
        const int row = i * 16 + fk * 4 + r;
        *reinterpret_cast<f16*>(Y + ytile(row, ch >> 3) + (ch & 7) * 2) = f16_sat(fast_sigmoid(g) * fast_tanh(f));
      }
    }
  __syncthreads();
  // y tile -> skip operand rows (16-B vectors)
  for (int idx = tid; idx < DL_BM * (DL_C / 8); idx += 512) {
    const int row = idx / (DL_C / 8), kc = idx - row * (DL_C / 8);
    const int m = m0 + row;
    if (m < M)
      *reinterpret_cast<uint4*>(p.g16 + (int64_t)m * p.ldg + kc * 8) = *reinterpret_cast<const uint4*>(Y + ytile(row, kc));
  }
  if constexpr (OUT) {
    // ---- GEMM2: z = y Wo^T over 12 K-steps; B (384 rows x 64 B = 24 instructions) through the ring
    const f16* o_src[3];
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      const int n = (w * 3 + v) * 16 + (lane >> 2);
      o_src[v] = p.Wo + (int64_t)n * DL_C + (((lane & 3) ^ ((n >> 2) & 3)) * 8);
    }
    auto issue2 = [&](int k) {
      unsigned char* bst = lds + (k & 1) * DL_STAGE + w * 3 * 1024;
#pragma unroll
      for (int v = 0; v < 3; ++v) dl_dma(o_src[v] + k * 32, bst + v * 1024);
    };
    floatx4 z[4][3];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) z[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    constexpr int NK2 = DL_C / 32;  // 12
    issue2(0);
    for (int k = 0; k < NK2; ++k) {
      if (k + 1 < NK2) {
        issue2(k + 1);
        dl_vmwait<3>();
      } else {
        dl_vmwait<0>();
      }
      dl_barrier();
      const unsigned char* Bm = lds + (k & 1) * DL_STAGE;
      half8 af[4], bf[3];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const half8*>(Y + ytile(i * 16 + fr, k * 4 + fk));
#pragma unroll
      for (int j = 0; j < 3; ++j) bf[j] = *reinterpret_cast<const half8*>(Bm + img64(w * 48 + j * 16 + fr, fk));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) z[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], z[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      dl_barrier();
    }
    // ---- residual update; next input staged in the (now idle) ring as a swizzled 64 x 384 f16 tile
    unsigned char* O = lds;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int col = w * 48 + j * 16 + fr;
      const float bo = p.bo[col], dn = p.dpn[col];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = i * 16 + fk * 4 + r, m = m0 + row;
          const float xn = (xr[i][j][r] + (z[i][j][r] + bo)) / 1.41421356237309515f;
          if (m < M) p.x32[(int64_t)m * DL_C + col] = xn;
          *reinterpret_cast<f16*>(O + ytile(row, col >> 3) + (col & 7) * 2) = f16_sat(xn + dn);
        }
    }
    __syncthreads();
    for (int idx = tid; idx < DL_BM * (DL_C / 8); idx += 512) {
      const int row = idx / (DL_C / 8), kc = idx - row * (DL_C / 8);
      const int m = m0 + row;
      if (m < M)
        *reinterpret_cast<uint4*>(p.x16n + (int64_t)m * DL_C + kc * 8) = *reinterpret_cast<const uint4*>(O + ytile(row, kc));
    }
  }
}

int diff_layer(const DiffLayerArgs& a, bool out, hipStream_t s) {
  SVC_REQUIRE(a.x16 && a.Wd && a.cpF && a.g16 && a.zpage && a.B > 0 && a.T > 0 && a.dil >= 1,
              "diff_layer: bad args");
  SVC_REQUIRE(!out || (a.Wo && a.bo && a.dpn && a.x32 && a.x16n), "diff_layer: residual operands missing");
  SVC_REQUIRE(a.ldg % 8 == 0 && ((uintptr_t)a.g16 & 15) == 0 && ((uintptr_t)a.x16 & 15) == 0, "diff_layer: alignment");
  const int M = a.B * a.T;
  static bool attr[2] = {false, false};
  if (!attr[out]) {
    const void* fn = out ? (const void*)diff_layer_kernel<true> : (const void*)diff_layer_kernel<false>;
    SVC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, DL_LDS));
    attr[out] = true;
  }
  const double flops = 2.0 * M * DL_N * DL_K1 + (out ? 2.0 * M * DL_C * DL_C : 0.0);
  const int tok = prof_begin(out ? "diff_layer<out>" : "diff_layer<last>", flops, 0.0, s);
  if (out)
    hipLaunchKernelGGL(diff_layer_kernel<true>, dim3(cdiv(M, DL_BM)), dim3(512), DL_LDS, s, a);
  else
    hipLaunchKernelGGL(diff_layer_kernel<false>, dim3(cdiv(M, DL_BM)), dim3(512), DL_LDS, s, a);
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// cp16 [rows][ldcp] (layer l's 2C columns at l*2C in conv_gemm "pair32" order: packed n -> channel
// (n >> 6) * 32 + (n & 31), filter half when n & 32) + dilated bias (original order [2C]) -> cpF record
// [rows_pad/16][C/16][64 lanes][4 rows][gate, filter] f16. Rows >= rows are zero.
__global__ void cp_fragment_kernel(const f16* __restrict__ cp16, int ldcp, const float* __restrict__ bdil, int rows,
                                   int rows_pad, f16* __restrict__ cpF) {
  const int64_t rec = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one 16-B record
  const int64_t nrec = (int64_t)rows_pad / 16 * (DL_C / 16) * 64;
  if (rec >= nrec) return;
  const int lane = (int)(rec & 63);
  const int64_t blk = rec >> 6;
  const int cb = (int)(blk % (DL_C / 16));
  const int rb = (int)(blk / (DL_C / 16));
  const int fr = lane & 15, fk = lane >> 4;
  const int ch = cb * 16 + fr;
  const int ng = (ch >> 5) * 64 + (ch & 31), nf = ng + 32;
  union { uint4 u; f16 h[8]; } o;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = rb * 16 + fk * 4 + r;
    float g = 0.f, f = 0.f;
    if (row < rows) {
      g = (float)cp16[(int64_t)row * ldcp + ng] + bdil[ch];
      f = (float)cp16[(int64_t)row * ldcp + nf] + bdil[DL_C + ch];
    }
    o.h[2 * r] = f16_sat(g);
    o.h[2 * r + 1] = f16_sat(f);
  }
  *reinterpret_cast<uint4*>(cpF + rec * 8) = o.u;
}

int cp_fragment(const f16* cp16, int ldcp, const float* bdil, int rows, int rows_pad, f16* cpF, hipStream_t s) {
  SVC_REQUIRE(rows_pad % 64 == 0 && rows_pad >= rows, "cp_fragment: rows_pad %d", rows_pad);
  const int64_t nrec = (int64_t)rows_pad / 16 * (DL_C / 16) * 64;
  hipLaunchKernelGGL(cp_fragment_kernel, dim3((unsigned)cdiv64(nrec, 256)), dim3(256), 0, s, cp16, ldcp, bdil, rows,
                     rows_pad, cpF);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
