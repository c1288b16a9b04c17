// DiffSVC residual projection as a weight-stationary row stream (modules/diffsvc.py:228-232), round 3.
//
// Per layer i < 19 of every denoiser call the split residual stream x + dproj_i = hi + lo (two fp16 halves, engine.hip
// denoise) is updated in place from the layer's gate output g (f16 [M][384]):
//   v  = g W_res^T + b_res                                    (residual half of output_projection, K = N = 384)
//   x' = (((hi + lo) - dproj_i) + v) / sqrt(2)                (modules/diffsvc.py:232)
//   hi = f16(x' + dproj_{i+1}),  lo = f16((x' + dproj_{i+1}) - hi)
// The GEMM is small (0.3 MFLOP per row) and the row's bytes are large (768 B of g in, 1536 B of hi / lo in and out), so
// the kernel is an HBM stream: 57.6 MB per 15 k-row sampler sub-batch. conv_gemm3's 128 x 128 tiles ran it as six
// dependent K-tile DMA round trips plus an epilogue read-modify-write per tile (latency-bound: 0.18 of HBM in situ).
// Here instead:
//   * W_res lives in VGPRs for the whole launch: a workgroup owns one half of the output columns (192), and each of its
//     12 waves holds one 16-column block's 384 x 16 f16 weights as 12 MFMA fragments (48 VGPRs), loaded once;
//   * the two workgroups of a row lane (one per half) walk the lane's 16-row tiles and LDS-DMA each tile's g rows and
//     their half of the hi / lo rows (24 KiB) into a ring of RP_D slots, RP_D - 1 tiles ahead of the tile being
//     computed: the loop issues no per-lane address arithmetic (a per-tile buffer descriptor carries the row base;
//     rows past M fall outside its range and read as 0);
//   * per tile a wave runs 12 v_mfma_f32_16x16x32 (operands swapped, so a lane's accumulator holds 4 consecutive
//     columns of one row) and applies the split-residual update in registers, storing hi / lo with range-checked buffer
//     stores (rows past M are dropped by the hardware), 8 B per lane and half.
// (A first form held all 384 columns per workgroup, 144 VGPRs of W per wave: loading 288 KiB of W into every CU took
// ~10 us per launch, longer than the sampler sub-batch's whole stream; measured 35 vs 23 us full batch.)
// K order (k = 0..383 in 32-deep MFMA steps into one accumulator) and the epilogue's arithmetic are conv_gemm3's, so the
// result is bit-identical to the tiled GEMM with its LDS-staged split epilogue (tests/test_gpu_ops.py).
#include "common.h"

// rp_dma clobbers m0 (reserved for the compiler's own LDS-DMA and indexing uses, which all set it right before use)
#pragma clang diagnostic ignored "-Winline-asm"

namespace svc {

constexpr int RP_C = 384;                 // channels: K = N = 384
constexpr int RP_H = 192;                 // output columns per workgroup (one half of N)
constexpr int RP_ROWS = 16;               // rows per tile (one MFMA block)
constexpr int RP_NW = 12;                 // waves per workgroup, one 16-column MFMA block each
constexpr int RP_NT = 64 * RP_NW;
constexpr int RP_GB = RP_ROWS * RP_C * 2;  // g image of a tile: 12 KiB = 12 DMA wave-instructions
constexpr int RP_HB = RP_ROWS * RP_H * 2;  // hi (or lo) image of a tile's half: 6 KiB = 6
constexpr int RP_SLOT = RP_GB + 2 * RP_HB;  // 24 KiB: 24 DMA wave-instructions, 2 per wave
constexpr int RP_ND = 2, RP_NS = 2;       // per wave and tile: DMA wave-instructions, stores
constexpr uint32_t RP_CFG = 0x00020000u;  // buffer descriptor dword 3 (raw, 32-bit data format)

struct ResProjArgs {
  const f16* g;       // [M][384] gate outputs of the layer
  const f16* Wf;      // W_res in fragment order (res_proj_pack)
  const float* bias;  // [384]
  const float* sub;   // dproj_i [384]
  const float* add;   // dproj_{i+1} [384]
  float div;          // sqrt(2)
  f16* hi;            // [M][384] split residual stream, updated in place
  f16* lo;
  int M;
  int lanes;          // row lanes = gridDim.x / 2 (each lane's two workgroups take the two halves of N)
  int iters;          // tiles per workgroup: ceil(ceil(M / 16) / lanes)
};

// LDS images, 16-B chunks: g row r (< 16) chunk q (< 48) at r * 48 + (q ^ r); hi / lo row r chunk q (< 24) at
// r * 24 + (q ^ ((r >> 1) & 7)). The MFMA operand reads (16 rows x one chunk per lane quarter, ds_read_b128) and the
// epilogue's 8-B hi / lo reads (16 rows x 2 halves of one chunk per half-wave, ds_read_b64) are then conflict-free.
__device__ __forceinline__ int rp_gchunk(int r, int q) { return r * 48 + (q ^ r); }
__device__ __forceinline__ int rp_hchunk(int r, int q) { return r * 24 + (q ^ ((r >> 1) & 7)); }

// LDS-DMA of 16 B per lane (lane i's bytes land at lds + 16 i) through a buffer descriptor, in inline asm: the compiler
// does not see it, so it neither drains it before every LDS read it cannot prove disjoint (it did, for the hi / lo
// reads of the ring) nor counts it; the loop's own vmcnt waits (rp_wait_tile) order the ring
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 rp_desc(const f16* base, int64_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return u32x4{(uint32_t)a, (uint32_t)(a >> 32) & 0xffffu, (uint32_t)(bytes > 0 ? bytes : 0), RP_CFG};
}
__device__ __forceinline__ void rp_dma(u32x4 d, uint32_t voff, unsigned char* lds) {
  const uint32_t m0 =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               ::"s"(m0), "v"(voff), "s"(d) : "memory", "m0");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rp_rsrc(const f16* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<f16*>(base), (short)0, (int)(bytes > 0 ? bytes : 0), RP_CFG);
}

// wait until at most N of this wave's vector-memory operations are outstanding (loads, LDS-DMAs and stores count
// together, in issue order)
template <int N>
__device__ __forceinline__ void rp_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Every wave issues RP_ND DMA wave-instructions and RP_NS buffer stores per iteration, whatever the rows (tiles past
// the end DMA zeros, stores past M are dropped by the range check), so the number of its vector-memory operations
// younger than its DMAs of tile t is a compile-time count:
//   t < D - 1 (DMA(t) issued in the prologue): (D - 2 - t) ND + t (ND + NS);  t >= D - 1: NS + (D - 2) (ND + NS)
template <int D, int T>
__device__ __forceinline__ void rp_wait_case() {
  constexpr int n = T < D - 1 ? (D - 2 - T) * RP_ND + T * (RP_ND + RP_NS) : RP_NS + (D - 2) * (RP_ND + RP_NS);
  rp_vmwait<n>();
}
template <int D>
__device__ __forceinline__ void rp_wait_tile(int t) {
  static_assert(D >= 2 && D <= 5, "ring depth");
  if (t == 0) rp_wait_case<D, 0>();
  else if (t == 1) rp_wait_case<D, 1>();
  else if (D >= 4 && t == 2) rp_wait_case<D, (D >= 4 ? 2 : D - 1)>();
  else if (D >= 5 && t == 3) rp_wait_case<D, (D >= 5 ? 3 : D - 1)>();
  else rp_wait_case<D, D - 1>();
}

// RP_D: ring slots (tiles); DMAs run RP_D - 1 tiles ahead
constexpr float RP_SQRT2 = SQRT2_F;
__device__ __forceinline__ float rp_div_sqrt2(float x) { return div_sqrt2_exact(x); }

// 101-104 VGPRs as built (keep it at or under 104): three waves per SIMD (312 registers) then fit beside one gate GEMM
// workgroup (184), which is what
// lets the other sampler stream's gate GEMM and this stream share a CU (r03o / r03p)
template <bool BF, int RP_D>
__global__ __launch_bounds__(RP_NT, 1) void res_proj_kernel(ResProjArgs p) {
  using O = Op16<BF>;
  extern __shared__ __align__(16) unsigned char smr[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fk = lane >> 4;
  // workgroups b and b + 8 (one XCD under round-robin placement) take the two halves of the same row tiles, so the
  // second read of each g tile is an L2 hit (speed only)
  const int b = blockIdx.x;
  const int half = (b >> 3) & 1, rlane = (b & 7) | ((b >> 4) << 3);
  const int n0 = half * RP_H + 16 * wave;  // this wave's output columns n0 .. n0 + 15; the lane's: n0 + 4 fk .. + 3

  // W fragments of the swapped MFMA (its A operand): w[kc] = W[n0 + fr][kc * 32 + fk * 8 .. + 8], stored in fragment
  // order by res_proj_pack so that each of the 12 loads is one contiguous KiB per wave
  half8 w[12];
  const f16* wf = p.Wf + (size_t)(half * RP_NW + wave) * 12 * 64 * 8 + lane * 8;
#pragma unroll
  for (int kc = 0; kc < 12; ++kc) w[kc] = *reinterpret_cast<const half8*>(wf + kc * 64 * 8);
  const float4 bi = *reinterpret_cast<const float4*>(p.bias + n0 + 4 * fk);
  const float4 sb = *reinterpret_cast<const float4*>(p.sub + n0 + 4 * fk);
  const float4 ad = *reinterpret_cast<const float4*>(p.add + n0 + 4 * fk);

  // this wave's DMA wave-instructions f = wave and wave + 12: f < 12 g piece f; 12..17 hi piece f - 12; 18..23 lo
  uint32_t voff[2];
  int dst[2], img[2];
  const f16* src[2];  // image base (row 0 of this half)
  int hoff[2];        // bytes of that base past the row start
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int f = wave + 12 * v;
    img[v] = f < 12 ? 0 : (f < 18 ? 1 : 2);
    const int piece = f < 12 ? f : (f < 18 ? f - 12 : f - 18);
    const int c = 64 * piece + lane;
    if (img[v] == 0) {
      const int r = c / 48, q = (c % 48) ^ r;
      voff[v] = (uint32_t)(r * RP_C * 2 + q * 16);
      dst[v] = piece * 1024;
      src[v] = p.g;
      hoff[v] = 0;
    } else {
      const int r = c / 24, q = (c % 24) ^ ((r >> 1) & 7);
      voff[v] = (uint32_t)(r * RP_C * 2 + q * 16);
      dst[v] = RP_GB + (img[v] - 1) * RP_HB + piece * 1024;
      src[v] = (img[v] == 1 ? p.hi : p.lo) + half * RP_H;
      hoff[v] = half * RP_H * 2;
    }
  }
  auto issue = [&](int t) {  // tile t of this workgroup into slot t % RP_D (tiles past the end read zeros)
    const int row0 = (rlane + t * p.lanes) * RP_ROWS;
    const bool live = row0 < p.M;
    const int64_t bytes = live ? (int64_t)(p.M - row0) * RP_C * 2 : 0;
    const int64_t off = live ? (int64_t)row0 * RP_C : 0;
    unsigned char* slot = smr + (t % RP_D) * RP_SLOT;
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      rp_dma(rp_desc(src[v] + off, bytes - hoff[v]), voff[v], slot + dst[v]);
    }
  };
  const __amdgpu_buffer_rsrc_t sh = rp_rsrc(p.hi, (int64_t)p.M * RP_C * 2), sl = rp_rsrc(p.lo, (int64_t)p.M * RP_C * 2);

#pragma unroll
  for (int t = 0; t < RP_D - 1; ++t) issue(t);
  for (int t = 0; t < p.iters; ++t) {
    rp_wait_tile<RP_D>(t);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // every wave's DMAs of tile t have landed; slot (t - 1) % RP_D is free
    __builtin_amdgcn_sched_barrier(0);
    issue(t + RP_D - 1);
    __builtin_amdgcn_sched_barrier(0);
    const unsigned char* slot = smr + (t % RP_D) * RP_SLOT;

    // this lane's hi / lo: row fr, columns n0 + 4 fk .. + 3 = chunk 2 wave + (fk >> 1) of the half, 8-B half fk & 1
    const int hb = rp_hchunk(fr, 2 * wave + (fk >> 1)) * 16 + (fk & 1) * 8;
    union { uint2 u; f16 h[4]; } hi, lo, ph, pl;
    hi.u = *reinterpret_cast<const uint2*>(slot + RP_GB + hb);
    lo.u = *reinterpret_cast<const uint2*>(slot + RP_GB + RP_HB + hb);
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < 12; ++kc)  // acc[r] = C[row fr][n0 + 4 fk + r]
      acc = O::mfma(w[kc], *reinterpret_cast<const half8*>(slot + rp_gchunk(fr, kc * 4 + fk) * 16), acc);
    // split-residual update (engine.hip epilogue_pass arithmetic, same order)
    const float v[4] = {acc[0] + bi.x, acc[1] + bi.y, acc[2] + bi.z, acc[3] + bi.w};
    const float s4[4] = {sb.x, sb.y, sb.z, sb.w}, a4[4] = {ad.x, ad.y, ad.z, ad.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float x = rp_div_sqrt2(((O::dec(hi.h[r]) + O::dec(lo.h[r])) - s4[r]) + v[r]);
      const float wv = x + a4[r];
      ph.h[r] = O::enc(wv);
      pl.h[r] = O::enc_lo(wv - O::dec(ph.h[r]));
    }
    const int row = (rlane + t * p.lanes) * RP_ROWS + fr;
    const uint32_t vo = (uint32_t)row * (RP_C * 2) + (uint32_t)(n0 + 4 * fk) * 2;
    buffer_store_b64(ph.u, sh, vo);
    buffer_store_b64(pl.u, sl, vo);
    __builtin_amdgcn_sched_barrier(0);
  }
  rp_vmwait<0>();  // (the remaining DMAs of tiles past the end land before the workgroup's LDS is released)
}

// W_res (packed [>= 384][ldw], W[n][k]) -> fragment order Wf[half][wave][kc][lane][8]: 16 B per thread
__global__ void res_proj_pack_kernel(const f16* __restrict__ W, int ldw, f16* __restrict__ Wf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= RP_C * RP_C / 8) return;
  const int lane = i & 63, kc = (i >> 6) % 12, hw = (i >> 6) / 12, wave = hw % RP_NW, half = hw / RP_NW;
  const int n = half * RP_H + 16 * wave + (lane & 15), k = kc * 32 + (lane >> 4) * 8;
  *reinterpret_cast<uint4*>(Wf + (size_t)i * 8) = *reinterpret_cast<const uint4*>(W + (size_t)n * ldw + k);
}

int res_proj_pack(const f16* W, int ldw, f16* Wf, hipStream_t s) {
  SVC_REQUIRE(ldw >= RP_C && ldw % 8 == 0 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)Wf & 15) == 0,
              "res_proj_pack: ldw %d", ldw);
  hipLaunchKernelGGL(res_proj_pack_kernel, dim3(cdiv(RP_C * RP_C / 8, 256)), dim3(256), 0, s, W, ldw, Wf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}
size_t res_proj_pack_elems() { return (size_t)RP_C * RP_C; }

// M rows of the split residual update for one layer; Wf: W_res in fragment order (res_proj_pack).
// lanes_cap > 0: that many row lanes (2 workgroups each); 0: 3/8 of the CU count (beside another sampler stream);
// -2: half the CU count (the projection alone on the chip: one workgroup per CU)
int res_proj(const f16* g, const f16* Wf, const float* bias, const float* sub, const float* add, float div, f16* hi,
             f16* lo, int M, bool bf16, int lanes_cap, hipStream_t s) {
  SVC_REQUIRE(M >= 0 && Wf, "res_proj: M %d, packed weights %p", M, (const void*)Wf);
  SVC_REQUIRE(div == RP_SQRT2, "res_proj: the residual divisor is sqrt(2) (modules/diffsvc.py:232)");
  if (M == 0) return SVC_OK;
  SVC_REQUIRE((int64_t)M * RP_C * 2 < (1ll << 31) - (1 << 20), "res_proj: %d rows exceed the 32-bit buffer range", M);
  SVC_REQUIRE(((uintptr_t)g & 15) == 0 && ((uintptr_t)Wf & 15) == 0 && ((uintptr_t)hi & 15) == 0 &&
                  ((uintptr_t)lo & 15) == 0,
              "res_proj: 16-B alignment");
  // the CU count (it sizes the row-lane grid) per device
  static int ncu_dev[16] = {};
  int dev = 0;
  SVC_HIP_CHECK(hipGetDevice(&dev));
  SVC_REQUIRE(dev >= 0 && dev < 16, "res_proj: device %d", dev);
  int& ncu = ncu_dev[dev];
  if (!ncu) SVC_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int tiles = cdiv(M, RP_ROWS);
  // row lanes in groups of 8 (the b / b + 8 pairing above). Default: 3/8 of the CU count (96 lanes = 192 workgroups
  // on 256 CUs): end to end 810.4-810.8 audio-s/s against 800.6-806.1 with one workgroup per CU, 804-805 with 80 lanes
  // and 807-808 with 112 (r03p, three alternating rounds): the CUs it leaves free run the other sampler stream's gate
  // GEMM, and fewer workgroups load W fewer times
  // One sampler stream (the round-4 default): half the CU count, 128 lanes = 256 workgroups, one per CU. Alone on the
  // chip 850.7 / 850.0 / 849.9 audio-s/s against 843.3 / 843.5 / 841.0 with 112 lanes (r04j, alternating); 160 lanes
  // (320 workgroups: a second round) 816 (r04i)
  int lanes = lanes_cap > 0 ? lanes_cap : (lanes_cap == -2 ? ncu / 2 : ncu * 3 / 8);
  lanes = std::max(8, std::min(lanes, (int)round_up(tiles, 8)));
  lanes = (int)round_up(lanes, 8);
  ResProjArgs a{g, Wf, bias, sub, add, div, hi, lo, M, lanes, cdiv(tiles, lanes)};
  // ring depth 3 (two tiles in flight): 4 / 5 slots measured no faster alone or in the sampler (r03k, two sampler
  // streams; r04n, one stream: 882.3 / 880.9 and 876.8 / 878.3 against 879.6 / 881.3 audio-s/s), 2 slots 4 % slower end
  // to end (r03o)
  constexpr int depth = 3;
  const void* fn = bf16 ? (const void*)res_proj_kernel<true, depth> : (const void*)res_proj_kernel<false, depth>;
  const int lds = depth * RP_SLOT;
  if (int st = ensure_dyn_lds(fn, lds)) return st;
  const int tok = prof_begin("res_proj<16x192>", 2.0 * M * RP_C * RP_C, (double)M * RP_C * 10.0, s);
  void* args[] = {&a};
  SVC_HIP_CHECK(hipLaunchKernel(fn, dim3(2 * lanes), dim3(RP_NT), args, lds, s));
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// ---------------------------------------------------------------------------- input projection (round 5)
// The denoiser's first step (modules/diffsvc.py:299-300, mel_preprocess: Conv1d(n_mel -> 384, 1) then ReLU) writes
// the split residual stream's first value: h = relu(x W_mel^T + b), hi = f16(h + dproj_0), lo = f16((h + dproj_0) - hi)
// (engine.hip denoise). K = 100 against 1536 B of hi / lo out per row: a store stream of 52 MB per sampler call, which
// conv_gemm3's 128 x 128 tiles ran at MFMA busy 0.04 with 36 VALU per MFMA (24 us per launch).
// Here one workgroup per CU walks 16-row tiles:
//   * W_mel (384 x 128 f16, zero past k = 100) lives in VGPRs: each of 12 compute waves holds its 32 output columns as
//     2 x 4 MFMA fragments (32 VGPRs), loaded once;
//   * a 13th wave only loads: each tile's x rows (16 x ldx f16) by LDS-DMA as four 1-KiB pieces into a ring of MP_D
//     slots, MP_D - 1 tiles ahead (rows past M read 0). Its own counted vmcnt retires a tile before the barrier the
//     compute waves pass to read it, and the compute waves' vmcnt holds only their stores, which so never delay a load
//     wait. In LDS a row takes MP_RS = 14 16-B chunks (rows of up to 13 chunks, ldx <= 104, then padded; the lane of
//     each LDS chunk picks its source chunk): the fragment reads (16 rows x one chunk, ds_read_b128 lane groups mixing
//     rows of two chunk columns) are conflict-free at that stride, where the unpadded 13-chunk rows (ldx 104) put 2-way
//     conflicts into every group (LDS-conflict share 0.47);
//   * per tile a compute wave runs 8 swapped v_mfma_f32_16x16x32 (a lane's accumulator holds 4 consecutive columns of
//     one row; k chunks past the row's ldx / 8 read as zero, as the padded tile does), swaps its two column blocks'
//     values between lane rows (8 consecutive columns per lane) and stores hi / lo, 16 B per lane and half.
// (A first form gave each workgroup one 64-row span and no ring: 21.1 us against conv_gemm3's 25.3, r05p.)
// Same 32-deep K order and epilogue arithmetic as conv_gemm3 with its LDS-staged epilogue: bit-identical
// (tests/test_gpu_stages.py test_res_proj_bit_identical, switch res_proj).
constexpr int MP_NW = 12, MP_NT = 64 * (MP_NW + 1);  // compute waves (32 output columns each) + the loader wave
constexpr int MP_D = 4;                              // ring slots (16-row tiles)
constexpr int MP_SLOT = 4096;                        // 16 rows x ldx f16 (ldx <= 128): four 1-KiB DMA pieces
constexpr int MP_RS = 14;                            // LDS row stride in 16-B chunks when ldx <= 104 (else ldx / 8)

struct MelProjArgs {
  const f16* x;       // [M][ldx] sampler input in the 16-bit operand format
  const f16* Wf;      // W_mel in fragment order (mel_proj_pack)
  const float* bias;  // [384]
  const float* add;   // dproj_0 [384]
  f16* hi;            // [M][384] split residual stream, written
  f16* lo;
  int M, ldx;
  int iters;          // tiles per workgroup: ceil(ceil(M / 16) / gridDim.x)
};

template <bool BF>
__global__ __launch_bounds__(MP_NT, 1) void mel_proj_kernel(MelProjArgs p) {
  using O = Op16<BF>;
  extern __shared__ __align__(16) unsigned char smm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;
  const int rowb = p.ldx * 2;  // bytes per x row
  const int qmax = p.ldx / 8;  // 16-B chunks per x row
  const int rs = qmax <= MP_RS - 1 ? MP_RS : qmax;  // LDS row stride (chunks)
  if (wave == MP_NW) {         // ---- loader
    // LDS chunk u = 64 v + lane of a slot holds x row u / rs, chunk u % rs (the padding chunks and those past the
    // 16 rows read nothing: out of the descriptor's range, zeros)
    uint32_t src[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int u = 64 * v + lane, r = u / rs, c = u - r * rs;
      src[v] = r < 16 && c < qmax ? (uint32_t)(r * rowb + c * 16) : 0x80000000u;
    }
    auto issue = [&](int t) {  // tile t of this workgroup into slot t % MP_D (tiles past the end read zeros)
      const int row0 = (blockIdx.x + t * G) * 16;
      const bool live = row0 < p.M;
      const u32x4 d = rp_desc(p.x + (live ? (int64_t)row0 * p.ldx : 0), live ? (int64_t)(p.M - row0) * rowb : 0);
      unsigned char* slot = smm + (t % MP_D) * MP_SLOT;
#pragma unroll
      for (int v = 0; v < 4; ++v) rp_dma(d, src[v], slot + v * 1024);
    };
#pragma unroll
    for (int t = 0; t < MP_D - 1; ++t) issue(t);
    for (int t = 0; t < p.iters; ++t) {
      rp_vmwait<(MP_D - 2) * 4>();  // tile t landed (tiles t + 1 .. t + MP_D - 2 may be in flight)
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();  // every compute wave finished tile t - 1: slot (t - 1) % MP_D is free
      __builtin_amdgcn_sched_barrier(0);
      issue(t + MP_D - 1);
    }
    rp_vmwait<0>();  // (the DMAs of tiles past the end land before the workgroup's LDS is released)
    return;
  }
  // ---- compute waves
  const int fr = lane & 15, fk = lane >> 4;
  half8 w[2][4];
  const f16* wf = p.Wf + (size_t)wave * 8 * 512 + lane * 8;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) w[j][kc] = *reinterpret_cast<const half8*>(wf + (j * 4 + kc) * 512);
  float4 bi[2], ad[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = 32 * wave + 16 * j + 4 * fk;
    bi[j] = *reinterpret_cast<const float4*>(p.bias + n);
    ad[j] = *reinterpret_cast<const float4*>(p.add + n);
  }
  const __amdgpu_buffer_rsrc_t sh = rp_rsrc(p.hi, (int64_t)p.M * RP_C * 2), sl = rp_rsrc(p.lo, (int64_t)p.M * RP_C * 2);
  const half8 zero = {};
  for (int t = 0; t < p.iters; ++t) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // the loader retired tile t
    __builtin_amdgcn_sched_barrier(0);
    const unsigned char* slot = smm + (t % MP_D) * MP_SLOT;
    floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) {
      const int q = kc * 4 + fk;
      half8 a = *reinterpret_cast<const half8*>(slot + (fr * rs + (q < qmax ? q : 0)) * 16);
      if (q >= qmax) a = zero;
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j] = O::mfma(w[j][kc], a, acc[j]);  // acc[r] = C[row fr][n + r]
    }
    const uint32_t rowo = (uint32_t)((blockIdx.x + t * G) * 16 + fr) * (RP_C * 2);
    union { uint2 u; f16 h[4]; } ph[2], pl[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float b4[4] = {bi[j].x, bi[j].y, bi[j].z, bi[j].w}, a4[4] = {ad[j].x, ad[j].y, ad[j].z, ad[j].w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // conv_gemm3's LDS-staged epilogue: relu(acc + bias) + add16, split
        const float wv = fmaxf(acc[j][r] + b4[r], 0.f) + a4[r];
        ph[j].h[r] = O::enc(wv);
        pl[j].h[r] = O::enc_lo(wv - O::dec(ph[j].h[r]));
      }
    }
    // the two 16-column blocks' values swapped between lane rows fk and fk ^ 1 (same output row): each lane then holds
    // 8 consecutive columns, and a store covers 16 rows x 64 B (conv_gemm3's block-pair epilogue)
    const auto hx = __builtin_amdgcn_permlane16_swap(ph[0].u.x, ph[1].u.x, false, false);
    const auto hy = __builtin_amdgcn_permlane16_swap(ph[0].u.y, ph[1].u.y, false, false);
    const auto lx = __builtin_amdgcn_permlane16_swap(pl[0].u.x, pl[1].u.x, false, false);
    const auto ly = __builtin_amdgcn_permlane16_swap(pl[0].u.y, pl[1].u.y, false, false);
    const uint32_t vo = rowo + (uint32_t)(32 * wave + 8 * (2 * (fk & 1) + (fk >> 1))) * 2;
    // rows past M fall outside the descriptor's range and are dropped
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{hx[0], hy[0], hx[1], hy[1]}, sh, vo, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{lx[0], ly[0], lx[1], ly[1]}, sl, vo, 0, 0);
  }
}

// W_mel (packed [>= 384][ldw], W[n][k], zero for k >= K) -> fragment order Wf[wave][j][kc][lane][8]
__global__ void mel_proj_pack_kernel(const f16* __restrict__ W, int ldw, f16* __restrict__ Wf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= RP_C * 128 / 8) return;
  const int lane = i & 63, kc = (i >> 6) & 3, j = (i >> 8) & 1, wave = i >> 9;
  const int n = 32 * wave + 16 * j + (lane & 15), k = kc * 32 + (lane >> 4) * 8;
  *reinterpret_cast<uint4*>(Wf + (size_t)i * 8) = *reinterpret_cast<const uint4*>(W + (size_t)n * ldw + k);
}

int mel_proj_pack(const f16* W, int ldw, f16* Wf, hipStream_t s) {
  SVC_REQUIRE(ldw >= 128 && ldw % 8 == 0 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)Wf & 15) == 0,
              "mel_proj_pack: ldw %d", ldw);
  hipLaunchKernelGGL(mel_proj_pack_kernel, dim3(cdiv(RP_C * 128 / 8, 256)), dim3(256), 0, s, W, ldw, Wf);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}
size_t mel_proj_pack_elems() { return (size_t)RP_C * 128; }

// M rows of the input projection (K = n_mel <= 128 channels of x at row stride ldx, ldx % 8 == 0, ldx <= 128; the
// columns K .. ldx - 1 of x hold zeros and W is zero past K) into the split residual stream hi / lo [M][384]
int mel_proj(const f16* x, int ldx, const f16* Wf, const float* bias, const float* add, f16* hi, f16* lo, int M,
             bool bf16, hipStream_t s) {
  SVC_REQUIRE(M >= 0 && Wf && ldx >= 8 && ldx <= 128 && ldx % 8 == 0, "mel_proj: M %d ldx %d", M, ldx);
  if (M == 0) return SVC_OK;
  SVC_REQUIRE((int64_t)M * RP_C * 2 < (1ll << 31) - (1 << 20), "mel_proj: %d rows exceed the 32-bit buffer range", M);
  SVC_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)Wf & 15) == 0 && ((uintptr_t)hi & 15) == 0 &&
                  ((uintptr_t)lo & 15) == 0,
              "mel_proj: 16-B alignment");
  static int ncu_dev[16] = {};  // the CU count (one workgroup per CU) per device
  int dev = 0;
  SVC_HIP_CHECK(hipGetDevice(&dev));
  SVC_REQUIRE(dev >= 0 && dev < 16, "mel_proj: device %d", dev);
  int& ncu = ncu_dev[dev];
  if (!ncu) SVC_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int tiles = cdiv(M, 16), grid = std::min(tiles, ncu);
  MelProjArgs a{x, Wf, bias, add, hi, lo, M, ldx, cdiv(tiles, grid)};
  const void* fn = bf16 ? (const void*)mel_proj_kernel<true> : (const void*)mel_proj_kernel<false>;
  const int lds = MP_D * MP_SLOT;
  if (int st = ensure_dyn_lds(fn, lds)) return st;
  const int tok = prof_begin("mel_proj<16x384>", 2.0 * M * RP_C * ldx, (double)M * (ldx * 2 + RP_C * 4), s);
  void* args[] = {&a};
  SVC_HIP_CHECK(hipLaunchKernel(fn, dim3(grid), dim3(MP_NT), args, lds, s));
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
