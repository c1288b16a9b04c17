// Shared definitions for the gfx950 (MI355X / CDNA4) SVC kernels.
// Layout convention for every activation tensor on the device: TIME-MAJOR ("channels-last"),
// row = b * T + t, channels contiguous. This makes every Conv1d an implicit GEMM whose A-operand
// rows are contiguous channel vectors (see gemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>

typedef _Float16 f16;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

#define SVC_OK 0
#define SVC_ERR_INVALID 1
#define SVC_ERR_HIP 2
#define SVC_ERR_STATE 3

namespace svc {

void set_error(const char* fmt, ...);
const char* get_error();

#define SVC_HIP_CHECK(expr)                                                              \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) {                                                              \
      ::svc::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr, hipGetErrorString(_e)); \
      return SVC_ERR_HIP;                                                                \
    }                                                                                    \
  } while (0)

#define SVC_REQUIRE(cond, ...)        \
  do {                                \
    if (!(cond)) {                    \
      ::svc::set_error(__VA_ARGS__);  \
      return SVC_ERR_INVALID;         \
    }                                 \
  } while (0)

#define SVC_LAUNCH_CHECK()                                                          \
  do {                                                                              \
    hipError_t _e = hipGetLastError();                                              \
    if (_e != hipSuccess) {                                                         \
      ::svc::set_error("%s:%d launch failed: %s", __FILE__, __LINE__, hipGetErrorString(_e)); \
      return SVC_ERR_HIP;                                                           \
    }                                                                               \
  } while (0)

static inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
static inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }
static inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

// exact-form GELU, x * Phi(x) (torch F.gelu default). erf by Abramowitz & Stegun 7.1.26 on the native
// v_exp_f32 / v_rcp_f32 (|error| <= 1.5e-7 absolute, ~14 VALU instead of libm erff's branchy ~30): every
// caller stores the result as fp16 or adds it to an fp32 stream whose other terms carry fp16 operand error.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(-1.4426950408889634f * ax * ax);
  return copysignf(fmaf(-p * t, e, 1.0f), x);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }
// gelu_erf on a pair of values with the packed f32 VALU (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two values per
// issue): erf_fast's and gelu_erf's operations per element, in the same order, so bit for bit gelu_erf's results.
// For VALU-only epilogue stretches (the Whisper fc1 GELU of conv_gemm3's register epilogue).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  const f32x2 z = x * 0.70710678118654752f;
  const f32x2 az = __builtin_elementwise_abs(z);
  f32x2 t = __builtin_elementwise_fma(f32x2{0.3275911f, 0.3275911f}, az, f32x2{1.0f, 1.0f});
  t = f32x2{__builtin_amdgcn_rcpf(t.x), __builtin_amdgcn_rcpf(t.y)};
  f32x2 p = __builtin_elementwise_fma(f32x2{1.061405429f, 1.061405429f}, t, f32x2{-1.453152027f, -1.453152027f});
  p = __builtin_elementwise_fma(p, t, f32x2{1.421413741f, 1.421413741f});
  p = __builtin_elementwise_fma(p, t, f32x2{-0.284496736f, -0.284496736f});
  p = __builtin_elementwise_fma(p, t, f32x2{0.254829592f, 0.254829592f});
  const f32x2 q = (-1.4426950408889634f * az) * az;
  const f32x2 e = f32x2{__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
  const f32x2 r = __builtin_elementwise_fma(-p * t, e, f32x2{1.0f, 1.0f});
  const f32x2 erf = f32x2{copysignf(r.x, z.x), copysignf(r.y, z.y)};
  return (0.5f * x) * (1.0f + erf);
}
// saturating fp32 -> fp16 store (NaN stays NaN): random-weight regimes can exceed the fp16 range
__device__ __forceinline__ f16 f16_sat(float v) { return (f16)(v > 65504.f ? 65504.f : (v < -65504.f ? -65504.f : v)); }
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
// Gate math on the native v_exp_f32 / v_rcp_f32 (~1 ulp each): the products feed an fp16 store, so these
// replace libm's expf / tanhf / IEEE division (~60 VALU per gate pair) in the MFMA kernels' epilogues.
__device__ __forceinline__ float fast_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
__device__ __forceinline__ float fast_tanh(float x) {  // 1 - 2 / (1 + e^{2x}): +-1 at the saturated ends
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(2.8853900817779268f * x));
}
// The DiffSVC gate sigmoid(a) * tanh(b) (modules/diffsvc.py:226-227) on two v_exp_f32 and ONE v_rcp_f32:
// tanh(b) = sign(b) (1 - E2) / (1 + E2) with E2 = e^{-2|b|} in [0, 1], sigmoid(a) = 1 / (1 + E1), E1 = e^{-a}, so the
// product is sign(b) (1 - E2) / ((1 + E1)(1 + E2)). E1's exponent is capped at 2^64 (a < -44: sigmoid < 6e-20, returned
// as ~5e-20): an infinite E1 times an underflowed E2 would make the denominator NaN, which the PLMS-100 trajectory of
// random weights reaches. The select keeps a NaN argument NaN; |result| <= 1, so its f16 store needs no saturation.
// Within 1-2 ulp of sigmoid * tanh (the fp32 oracle with this form tracks the reference's PLMS-100 to 2.4e-7).
__device__ __forceinline__ float gate_act(float a, float b) {
  float t1 = -1.4426950408889634f * a;
  t1 = t1 > 64.0f ? 64.0f : t1;
  const float e1 = __builtin_amdgcn_exp2f(t1);
  const float e2 = __builtin_amdgcn_exp2f(-2.8853900817779268f * fabsf(b));
  const float d1 = 1.0f + e1;
  float r = (1.0f - e2) * __builtin_amdgcn_rcpf(fmaf(d1, e2, d1));
  // the product is rounded to f32 here, then to f16 by the caller's store: the empty asm keeps hipcc from fusing the
  // multiply with that conversion into one v_fma_mixlo_f16 (one rounding), which it did in some kernels and not in
  // others (the last f16 bit differed in ~1e-5 of the outputs and broke gate_ws / conv_gemm4 bit identity, r04f)
  asm("" : "+v"(r));
  return copysignf(r, b);
}

// 8-byte buffer store (range-checked: a voffset past the descriptor's range is dropped). Write-through (cache policy
// sc1), so that the kernel-end release would find the outputs clean, measured slower for the row-stream kernels
// (r04n: 855.8 / 857.1 against 879.6 / 881.3 audio-s/s): plain write-back
// x / sqrt(2) (f32 sqrt(2)) exactly as the IEEE division rounds it, in one multiply and two FMAs (q0 = x r,
// e = x - q0 sqrt(2) exactly, q0 + e r): equal to the division bit for bit for every float x with 2^-100 <= |x| < inf
// (all 2^32 inputs checked against x86 fmaf / division; the differing inputs are |x| <= 2.2e-32 and +-inf). Those
// lanes take the division, behind a branch no wave takes in practice. Replaces the ~10-instruction division sequence
// (v_div_scale x2, v_rcp, 4 FMAs, v_div_fmas, v_div_fixup) of the DiffSVC residual epilogues (res_proj).
constexpr float SQRT2_F = 1.41421356237309515f;
__device__ __forceinline__ float div_sqrt2_exact(float x) {
  constexpr float r = 1.0f / SQRT2_F;
  float q;
  if (__builtin_expect(fabsf(x) >= 0x1p-100f && fabsf(x) <= 3.402823466e38f, 1)) {
    const float q0 = x * r;
    q = fmaf(fmaf(-q0, SQRT2_F, x), r, q0);
  } else {
    q = x / SQRT2_F;  // (NaN too) the IEEE division for this lane
  }
  return q;
}

__device__ __forceinline__ void buffer_store_b64(uint2 v, __amdgpu_buffer_rsrc_t r, uint32_t vo) {
  typedef unsigned int u32x2v __attribute__((vector_size(8)));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, v), r, vo, 0, 0);
}

// ------------------------------------------------------------------ 16-bit MFMA operand formats
// GEMM operands (activations and packed weights) are 16-bit values in f16-typed buffers: IEEE binary16 by default, or
// bfloat16 bit patterns when a context runs its DiffSVC / content-encoder GEMMs in the bf16 operand variant (config
// "operands.bf16", BASELINE configs[4]'s fp16-vs-bf16 sweep). Op16<BF> encodes / decodes them and picks the MFMA.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
template <bool BF>
struct Op16;
template <>
struct Op16<false> {
  static __device__ __forceinline__ float dec(f16 h) { return (float)h; }
  static __device__ __forceinline__ f16 enc(float v) { return f16_sat(v); }  // saturating, NaN stays NaN
  static __device__ __forceinline__ f16 enc_lo(float v) { return (f16)v; }  // low half of a split value
  static __device__ __forceinline__ floatx4 mfma(half8 a, half8 b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
template <>
struct Op16<true> {
  static __device__ __forceinline__ float dec(f16 h) {
    return __uint_as_float((uint32_t)__builtin_bit_cast(uint16_t, h) << 16);
  }
  static __device__ __forceinline__ f16 enc(float v) { return __builtin_bit_cast(f16, (__bf16)v); }  // RNE
  static __device__ __forceinline__ f16 enc_lo(float v) { return __builtin_bit_cast(f16, (__bf16)v); }
  static __device__ __forceinline__ floatx4 mfma(half8 a, half8 b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
};
// runtime-format forms for the element-wise producers (a wave-uniform flag)
__device__ __forceinline__ f16 enc16(float v, bool bf) { return bf ? Op16<true>::enc(v) : Op16<false>::enc(v); }
__device__ __forceinline__ f16 enc16_lo(float v, bool bf) {
  return bf ? Op16<true>::enc_lo(v) : Op16<false>::enc_lo(v);
}
__device__ __forceinline__ float dec16(f16 h, bool bf) { return bf ? Op16<true>::dec(h) : Op16<false>::dec(h); }

// ------------------------------------------------------------------ implicit-GEMM descriptors
// Y[m, n] = epilogue( sum_{tap, c} X[in_row(m, tap), c] * Wp[n, tap*Cp + c] )
//   m = b*T_out + t  (b < B, t < T_out);   in_row = b*T_in + t*istride + tap*tap_mul + tap_add
//   rows outside [0, T_in) of utterance b read as zero (Conv1d zero padding, per utterance).
struct ConvGemmArgs {
  const f16* X;  // [B*T_in rows][ldx] f16
  int ldx;       // row stride (elements), multiple of 8
  int T_in;
  int Cp;        // channels per tap in the K index (multiple of 8)
  int Cvalid;    // channels >= Cvalid read as zero
  const f16* W;  // packed [Npad][Kpad]
  int K;         // ntaps * Cp
  int Kpad;      // multiple of 64
  int tap_mul, tap_add, istride;
  int B, T_out;
  int N;         // valid (packed) output columns
  int ntiles_n;
  // ragged batches: utterance b has min(T_in, tv[b] * tv_mul) valid input rows (NULL = all T_in); rows past it read
  // as zero, exactly the Conv1d zero padding of a clip of that length (its own rows keep the batch stride T_in)
  const int* tv;
  int tv_mul;
  int bf16;      // operands (X, W) are bfloat16 (Op16<true>); the epilogue's 16-bit inputs / outputs too
  const f16* Wfrag;  // W once more in a kernel's own fragment order (gate_ws; NULL: none)
};

__device__ __forceinline__ int valid_in_rows(const ConvGemmArgs& a, int b) {
  return a.tv ? min(a.T_in, a.tv[b] * a.tv_mul) : a.T_in;
}

// Epilogue kinds (runtime-selected inside one kernel family)
enum EpiKind : int {
  EPI_GENERIC = 0,  // v = act(acc + bias[n]) (*col_scale) (+add_t) (+add_row) ((acc32+v)/acc_div)
  EPI_GATE = 1,     // DiffSVC: sigmoid(gate+cp) * tanh(filter+cp)          (paired columns)
  EPI_COND = 3,     // conditioner: acc + bias + emb_m[idx_m] + emb_l[idx_l] + emb_s[singer]
};

enum ActKind : int { ACT_NONE = 0, ACT_GELU = 1, ACT_RELU = 2 };

// The attention kernel takes q pre-multiplied by log2(e) (with its dh^-1/4 share of the score scale, in the QKV GEMM
// epilogue), so its scores come out of the MFMAs in exp2 units
constexpr float ATT_LOG2E = 1.4426950408889634f;

struct EpiArgs {
  int kind;
  const float* bias;  // [Npad] packed order
  int act;
  // output row mapping: orow = b*T_ostore + t*ostride + ophase
  int T_ostore, ostride, ophase;
  float* out32; int ld32;                   // f32 output (may alias acc32 / add_row element-wise)
  const float* acc32; int ld_acc; float acc_div;  // v = (acc32[orow][n] + v) / acc_div   (resblock mean)
  f16* out16; int ld16; const float* add16; // out16 = f16(v + add16[n])  (next-layer input)
  const float* add_t; int ld_add_t;         // added after act, indexed by t (positional embedding)
  const float* add_row; int ld_add_row;     // added after act, indexed by orow (residual input)
  int scale_cols; float col_scale;          // columns < scale_cols multiplied by col_scale (q/k scaling) ...
  int scale_cols2; float col_scale2;        // ... except columns < scale_cols2 (<= scale_cols): by col_scale2 (q)
  // DiffSVC gate
  const f16* cp; int ld_cp;                 // conditioner projection (packed order, bias folded)
  f16* y16; int ldy16;                      // gate output sigmoid(gate) * tanh(filter), f16
  // conditioner
  const int* idx_m; const int* idx_l; const int* singer;
  const float* emb_m; const float* emb_l; const float* emb_s; int ld_emb;
  // split-fp16 operand output ("fp16x3", elementwise.hip f32_to_f16x3): when > 0, out16 also receives the
  // residual lo = f16(v - hi) at column split16 + n and hi again at 2 * split16 + n
  int split16;
  // column blocks (LDS-staged generic epilogue, out16 only): when > 0, output column n goes to block n / col_block,
  // which starts col_block_stride elements after the previous one (the layer-major conditioner projections of all
  // DiffSVC layers as one GEMM); a tile's columns lie in one block
  int col_block;
  int64_t col_block_stride;
  // split residual stream (the DiffSVC x): x + add16 is held as hi (out16 / acc16_hi, the next GEMM's operand) plus
  // lo16 = f16((x + add16) - hi), ~22 significand bits in 4 bytes. acc16_hi / acc16_lo / acc_sub: the residual read
  // as acc = (hi + lo) - acc_sub (the add16 it was stored with), in place of acc32; lo16: also write the lo half
  const f16* acc16_hi; const f16* acc16_lo; const float* acc_sub;
  f16* lo16;
  // host-side launch hint: keep conv_gemm3's LDS-staged epilogue for this call (set by run_gemm, see gemm3.hip)
  int no_reg_epi;
};

// Per-call host tables (ragged-batch lengths) staged to the device, stream-ordered: a ring of pinned host + device
// slots, so a table is never rewritten while an earlier copy, or a kernel reading an earlier table, may still be in
// flight. put() records the slot's event after the copy; the entry point that consumed the table re-records it with
// retire() on its stream after its last launch (RingRetire below), so a slot is reused only after every kernel of
// the call that read it has finished, whichever stream the next call of another entry point runs on.
struct StageRing {
  static constexpr int kRing = 8;
  void* h[kRing] = {};
  void* d[kRing] = {};
  size_t cap[kRing] = {};
  hipEvent_t ev[kRing] = {};
  int next = 0;
  int last = -1;  // slot handed out by the latest put(), until retire()
  // copies `bytes` from `src` to device memory owned by the ring; *dev receives it
  int put(const void* src, size_t bytes, hipStream_t s, void** dev) {
    const int k = next;
    next = (next + 1) % kRing;
    if (ev[k]) SVC_HIP_CHECK(hipEventSynchronize(ev[k]));
    else SVC_HIP_CHECK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
    if (cap[k] < bytes) {
      if (h[k]) SVC_HIP_CHECK(hipHostFree(h[k]));
      if (d[k]) SVC_HIP_CHECK(hipFree(d[k]));
      const size_t want = std::max<size_t>(bytes, 4096);
      SVC_HIP_CHECK(hipHostMalloc(&h[k], want, hipHostMallocDefault));
      SVC_HIP_CHECK(hipMalloc(&d[k], want));
      cap[k] = want;
    }
    memcpy(h[k], src, bytes);
    SVC_HIP_CHECK(hipMemcpyAsync(d[k], h[k], bytes, hipMemcpyHostToDevice, s));
    SVC_HIP_CHECK(hipEventRecord(ev[k], s));
    last = k;
    *dev = d[k];
    return SVC_OK;
  }
  // the latest table's readers are all enqueued on s (sub-streams joined back): its slot waits for them
  void retire(hipStream_t s) {
    if (last >= 0) (void)hipEventRecord(ev[last], s);
    last = -1;
  }
  void release() {
    for (int k = 0; k < kRing; ++k) {
      if (ev[k]) (void)hipEventSynchronize(ev[k]), (void)hipEventDestroy(ev[k]);
      if (h[k]) (void)hipHostFree(h[k]);
      if (d[k]) (void)hipFree(d[k]);
    }
  }
};
// scope guard of an entry point that stages a table: retires it on the entry point's stream when the call returns
// (after its last launch, on every return path)
struct RingRetire {
  StageRing& r;
  hipStream_t s;
  RingRetire(StageRing& ring, hipStream_t stream) : r(ring), s(stream) { r.last = -1; }
  ~RingRetire() { r.retire(s); }
};


// One PLMS update x' = x + d (A x - Bc e'), e' = (sum_k c_k e_k) / div (modules/diffsvcrepo_inference.py:91-130;
// engine.hip svc_diffsvc_sample, elementwise.hip plms_update).
struct PlmsArgs {
  const float* e[4]; float c[4]; int ne; float div;
  float d, A, Bc;
  const float* xin;  // x the update is applied to
  float* xout; f16* x16; int ld16;
  float* e_avg_out;  // optional: store e' (used for the first PLMS step's x_pred path)
  int bf16;          // x16 holds bfloat16 operands (the bf16 variant)
};
// The PLMS update of 4 consecutive channels of one row, e_k = ev[k] (k < p.ne), x the row's current values:
// e' = (c_0 e_0 + c_1 e_1 + ...) / div in the reference's left-to-right order, x' = x + d (A x - Bc e') (the x16 copy is
// the caller's; plms4_kernel).
__device__ __forceinline__ void plms_math4(const PlmsArgs& p, const float4* ev, float4 x, float4& e_out, float4& x_out) {
  float e[4] = {p.c[0] * ev[0].x, p.c[0] * ev[0].y, p.c[0] * ev[0].z, p.c[0] * ev[0].w};
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    if (p.ne > k) {
      e[0] = e[0] + p.c[k] * ev[k].x;
      e[1] = e[1] + p.c[k] * ev[k].y;
      e[2] = e[2] + p.c[k] * ev[k].z;
      e[3] = e[3] + p.c[k] * ev[k].w;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) e[k] = e[k] / p.div;
  e_out = make_float4(e[0], e[1], e[2], e[3]);
  x_out = make_float4(x.x + p.d * (p.A * x.x - p.Bc * e[0]), x.y + p.d * (p.A * x.y - p.Bc * e[1]),
                      x.z + p.d * (p.A * x.z - p.Bc * e[2]), x.w + p.d * (p.A * x.w - p.Bc * e[3]));
}
// Kernel-selection switches: the measured production choices by default, other values select the earlier or
// alternative kernel forms that the parity tests cover and the A/B benches compare (DESIGN.md records each result).
// A context copies the defaults at creation, where an SVC_<NAME> environment variable overrides each (so a whole
// benchmark can be A/B-run from the shell); svc_ctx_set_config(ctx, "tune.<name>", v) changes one for that context
// (ctx NULL: the op-level entry points' context). Launchers read the switches of the context whose entry point is
// running (tuning(), set per call by TuningScope) instead of the environment.
struct Tuning {
  int gemm_variant = 15;    // GEMM kernel: 15 fitted choice (conv_gemm3 tile by pick3; the DiffSVC gate GEMM on
                            // conv_gemm4 with its register gate epilogue), 10..14 / 16 a fixed conv_gemm3 tile (16: 256 x 192), 20 / 24
                            // conv_gemm4 with the LDS-staged / register epilogue where N > 64
  int gemm3_direct = 3;     // conv_gemm3 register-epilogue forms in use (mask, gemm3.hip direct_form3)
  int whisper_streams = 1;  // Whisper encoder sub-batch streams
  int sampler_streams = 1;  // DiffSVC sampler sub-batch streams (round 4: 1 with gate_ws; 2 was the conv_gemm4 default)
  int vocoder_streams = 1;  // BigVGAN sub-batch streams
  int diff_head = 1;        // DiffSVC skip_projection + output_projection as one launch (diff_head.hip)
  int amp_maxc = 192;       // widest BigVGAN channel count on the fused activation + conv kernel (0: none). C = 96 on
                            // the 256-row 2 x 2-wave tiles: BigVGAN -1.0 ms per step against activation1d + the plain
                            // conv (profiles/r06_ab/r06x_amp_fused_c96.txt); C = 192 on 2 x 4 waves: -0.6 ms against
                            // activation1d + conv_gemm3<256,192> (r06z_amp_c192.txt)
  int amp_ups = 1;          // BigVGAN rate-2 ConvTranspose with cin 48 / 96 / 192 as one amp_conv plain conv (VStage::upc;
                            // 0: phase GEMMs): those stages 1.93 -> 0.89 ms per step (profiles/r06_ab/r06zc_amp_ups.txt)
  int res_proj = 1;         // DiffSVC residual and input projections on the weight-stationary streams (res_proj.hip
                            // res_proj / mel_proj; 0: conv_gemm3;
                            // > 1: that many row lanes of 2 workgroups instead of 1/2 (one sampler stream) or 3/8
                            // (several) of the CU count)
  int gate_ws = 1;          // DiffSVC dilated conv + gate: 1 the weight-stationary row stream (gate_ws.hip), 0 conv_gemm4
                            // (the A-stationary dlayer.hip of round 5, gate alone or the whole layer, measured no
                            // faster and was removed: DESIGN.md, r05k)
  std::string site_variant;  // "site=variant,...": per-call-site GEMM kernel override (environment only, A/B runs)
  void from_env();
  bool set(const char* name, double v);  // false: unknown name ("reset" restores the creation-time values)
  bool get(const char* name, double* v) const;
};
const Tuning& tuning();
struct TuningScope {
  explicit TuningScope(const Tuning* t);
  ~TuningScope();
  const Tuning* prev;
};

// The dynamic-LDS limit of a kernel (hipFuncSetAttribute) is a per-device function attribute: set it once per (kernel,
// device) on the current device before launching with more than 64 KiB (engine.hip)
int ensure_dyn_lds(const void* fn, int bytes);

// live per-kernel timing (bench roofline): when enabled, launches are bracketed by hipEvents and
// aggregated by kernel name together with their algorithmic FLOPs / bytes.
int prof_begin(const char* name, double flops, double bytes, hipStream_t s);  // returns token or -1
void prof_end(int token, hipStream_t s);
void prof_site(const char* site);  // label attached to the next launches ("kernel@site")

}  // namespace svc
