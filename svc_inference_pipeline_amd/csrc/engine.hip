// Native runtime of the SVC hot path: context, weight packing (weight_norm fold, MFMA layouts),
// device workspace arena and the stage orchestration behind the C-ABI (include/svc_hip.h).
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <ctype.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/svc_hip.h"
#include <cstring>

#include "common.h"
#include "amp_conv.h"
#include "spectral.h"

namespace svc {

// ---------------------------------------------------------------------------- errors
static thread_local char g_err[1024] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const char* get_error() { return g_err; }

// ---------------------------------------------------------------------------- live profiling
struct ProfRec {
  std::string name;
  hipEvent_t a, b;
  double flops, bytes;
};
static bool g_prof = false;
static std::string g_prof_filter;  // when non-empty, only kernels whose name starts with it are recorded
static std::vector<ProfRec> g_prof_recs;
static std::vector<hipEvent_t> g_ev_pool;

static hipEvent_t ev_get() {
  if (!g_ev_pool.empty()) {
    hipEvent_t e = g_ev_pool.back();
    g_ev_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

static thread_local const char* g_site = "";
void prof_site(const char* site) { g_site = site ? site : ""; }

int prof_begin(const char* name, double flops, double bytes, hipStream_t s) {
  if (!g_prof) return -1;
  if (!g_prof_filter.empty() && strncmp(name, g_prof_filter.c_str(), g_prof_filter.size()) != 0) return -1;
  std::string full = std::string(name) + (g_site[0] ? std::string("@") + g_site : std::string());
  ProfRec r{full, ev_get(), ev_get(), flops, bytes};
  if (!r.a || !r.b) return -1;
  (void)hipEventRecord(r.a, s);
  g_prof_recs.push_back(r);
  return (int)g_prof_recs.size() - 1;
}

void prof_end(int tok, hipStream_t s) {
  if (tok >= 0 && tok < (int)g_prof_recs.size()) (void)hipEventRecord(g_prof_recs[tok].b, s);
}

// kernels in other translation units
int attention(const f16* qkv, f16* out, int B, int L, int D, hipStream_t s, bool bf16);
int layernorm_f16(const float* x, const float* g, const float* b, f16* y, int rows, int D, int ldy, hipStream_t s,
                  bool bf);
int layernorm_f32(const float* x, const float* g, const float* b, float* y, int rows, int D, int ldy, hipStream_t s);
int activation1d(const float* x, f16* y, int B, int L, int C, int ldy, const float* alpha_log, const float* beta_log,
                 const float* filt, hipStream_t s, const int* tv = nullptr, int tv_mul = 1, const f16* x16 = nullptr);
int f32_to_f16(const float* x, int ldx, f16* y, int ldy, int rows, int C, int Cpad, hipStream_t s, bool bf);
int denorm_mel(const float* x, f16* y, float* y32, int ldy, int rows, int C, const float* mn, const float* mx,
               hipStream_t s);
int content_map(const float* src, int B, int src_rows, int ld_src, int T, int D, f16* dst, int ld_dst, hipStream_t s,
                bool bf);
int bucketize(const double* f0, const float* en, const float* mbins, const float* ebins, int nb, int* im, int* ie,
              int n, hipStream_t s);
int plms_update(const PlmsArgs& p, int rows, int C, hipStream_t s);
struct DdpmArgs {
  float sra, srm1, c1, c2, sigma;
  const float* z; uint64_t seed; const int* utt_ids; int step;
  int bf16;  // x16 holds bfloat16 operands
};
int ddpm_update(float* x, const float* eps, f16* x16, int ld16, int B, int T, int C, const DdpmArgs& a, hipStream_t s);
int init_noise(float* x, f16* x16, int ld16, int B, int T, int C, uint64_t seed, const int* utt_ids, float std,
               hipStream_t s, bool bf);
int conv_post(const f16* a, int lda, int B, int L, int C, const float* w, float bias, const float* fade, int nfade,
              float* out, hipStream_t s, const int* tv = nullptr, int tv_mul = 1);
int zero_tail_rows(float* x, int B, int T, int C, const int* Tb, hipStream_t s);
int whisper_normalize(const float* logspec, float* mx_scratch, f16* out, int B, int64_t n_per_utt, hipStream_t s,
                      int split_c, bool bf, int ldo);
int layernorm_f16x3(const float* x, const float* g, const float* b, f16* y, int rows, int D, hipStream_t s, bool bf);
int f32_to_f16x3_grouped(const float* x, f16* y, int rows, int C, int Cg, hipStream_t s, bool bf);
int f16_to_f32(const f16* x, float* y, int64_t n, hipStream_t s);
int f32_to_f16x3(const float* x, int ldx, f16* y, int rows, int C, hipStream_t s, bool bf);
int conv_gemm3(const ConvGemmArgs& a, const EpiArgs& e, const f16* zpage, int variant, hipStream_t s);
int conv_gemm4(const ConvGemmArgs& a, const EpiArgs& e, const f16* zpage, hipStream_t s, bool direct_gate);
bool gate_ws_fits(const ConvGemmArgs& a, const EpiArgs& e);
extern unsigned long long* gate_ws_stamps;
int gate_ws_nstamp();
int gate_ws(const ConvGemmArgs& a, const EpiArgs& e, hipStream_t s);
int gate_ws_pack(const f16* W, int ldw, f16* Wf, hipStream_t s);
size_t gate_ws_pack_elems();
int res_proj(const f16* g, const f16* Wf, const float* bias, const float* sub, const float* add, float div, f16* hi,
             f16* lo, int M, bool bf16, int lanes_cap, hipStream_t s);
int res_proj_pack(const f16* W, int ldw, f16* Wf, hipStream_t s);
size_t res_proj_pack_elems();
int mel_proj(const f16* x, int ldx, const f16* Wf, const float* bias, const float* add, f16* hi, f16* lo, int M,
             bool bf16, hipStream_t s);
int mel_proj_pack(const f16* W, int ldw, f16* Wf, hipStream_t s);
size_t mel_proj_pack_elems();
int diff_head(const f16* s16, const f16* Wsp, const float* bsp, int Nsp, int Ksp, const f16* Wout, const float* bout,
              int Nout, int Kout, int Npad_out, float* eps, int ld_eps, int M, const f16* zpage, hipStream_t s,
              bool bf16);
int pitch_shift(double* f0, int B, int T, double target, hipStream_t s);
int content_map_hubert(const float* src, int B, int src_rows, int ld_src, int T, int D, f16* dst, int ld_dst,
                       hipStream_t s, bool bf);
int hubert_frames5(const float* wav, int B, int64_t n, f16* out, bool split, hipStream_t s, bool bf);
int groupnorm_gelu(const float* x, int B, int T, int C, const float* gamma, const float* beta, double* part,
                   int max_chunks, float2* ss, f16* y, bool split, hipStream_t s, bool bf);
int layernorm_dual(const float* x, const float* g, const float* b, float* y32, f16* y16, int rows, int D, bool split,
                   hipStream_t s, bool bf);
int pack_qkv(const float* q, const float* k, const float* v, f16* qkv, int64_t rows, int D, float scale, hipStream_t s);
int f0_praat_ac(const float* wav, int B, int64_t n_samples, double fs, double time_step, double floor_hz,
                double ceiling_hz, double voicing, int T, double* f0_out, void* workspace, size_t ws_bytes,
                const double* tables, hipStream_t s, const int64_t* n_b = nullptr, const int* T_b = nullptr,
                StageRing* ring = nullptr);
size_t f0_workspace_bytes(int B, int64_t n_samples, double fs, double time_step, double floor_hz);
size_t f0_table_doubles(double fs, double floor_hz);
int f0_tables(double fs, double floor_hz, double* out);
size_t pyin_table_doubles(double sr, double fmin, double fmax, int frame_length, int win_length, int hop);
size_t pyin_workspace_bytes(int B, int F, double sr, double fmin, double fmax, int frame_length, int win_length,
                            int hop);
int pyin_tables(double sr, double fmin, double fmax, int frame_length, int win_length, int hop, double* out);
int f0_pyin(const float* wav, int B, int64_t ld, const int64_t* nvalid_dev, const int64_t* nvalid_host, double sr,
            double fmin, double fmax, int frame_length, int win_length, int hop, int F, double* f0, void* ws,
            size_t ws_bytes, const double* tables_dev, hipStream_t s);

// ---------------------------------------------------------------------------- host helpers
static std::vector<float> slaney_mel(int sr, int n_fft, int n_mels, double f_lo, double f_hi) {
  auto hz2mel = [](double f) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = log(6.4) / 27.0;
    return f >= min_log_hz ? min_log_mel + log(f / min_log_hz) / logstep : f / f_sp;
  };
  auto mel2hz = [](double m) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = log(6.4) / 27.0;
    return m >= min_log_mel ? min_log_hz * exp(logstep * (m - min_log_mel)) : f_sp * m;
  };
  const int nb = 1 + n_fft / 2;
  std::vector<double> fftf(nb), melf(n_mels + 2);
  // np.fft.rfftfreq(n, 1/sr) = k * (1 / (n * (1/sr)))
  const double val = 1.0 / ((double)n_fft * (1.0 / (double)sr));
  for (int k = 0; k < nb; ++k) fftf[k] = k * val;
  const double m0 = hz2mel(f_lo), m1 = hz2mel(f_hi);
  // np.linspace(start, stop, num): step = (stop-start)/(num-1); y = arange*step + start; y[-1] = stop
  const int num = n_mels + 2;
  const double step = (m1 - m0) / (num - 1);
  for (int i = 0; i < num; ++i) melf[i] = mel2hz(i == num - 1 ? m1 : i * step + m0);
  std::vector<float> w((size_t)n_mels * nb);
  for (int i = 0; i < n_mels; ++i) {
    const double fd0 = melf[i + 1] - melf[i], fd1 = melf[i + 2] - melf[i + 1];
    const double enorm = 2.0 / (melf[i + 2] - melf[i]);
    for (int k = 0; k < nb; ++k) {
      double lower = -(melf[i] - fftf[k]) / fd0;
      double upper = (melf[i + 2] - fftf[k]) / fd1;
      double v = fmax(0.0, fmin(lower, upper));
      float vf = (float)v;                      // weights[i] = ... stored in the f32 array
      w[(size_t)i * nb + k] = (float)((double)vf * enorm);  // weights *= enorm (f32 *= f64)
    }
  }
  return w;
}

// W_n^m = exp(-2 pi i m / n) as interleaved (re, im) f64 pairs
static std::vector<double> fft_twiddles(int n) {
  std::vector<double> t(2 * (size_t)n);
  for (int m = 0; m < n; ++m) {
    const double a = 2.0 * M_PI * (double)m / (double)n;
    t[2 * (size_t)m] = cos(a);
    t[2 * (size_t)m + 1] = -sin(a);
  }
  return t;
}

// The nonzero band [lo, hi) of each filter row, packed (the DFT kernel keeps only those weights, in LDS):
// band[3m .. 3m+2] = lo, hi, offset of the band in the packed weights
struct FilterBands {
  std::vector<float> w;
  std::vector<int> band;
};
static FilterBands filter_bands(const std::vector<float>& fb, int n_mels) {
  const int nb = (int)(fb.size() / n_mels);
  FilterBands r;
  r.band.assign(3 * n_mels, 0);
  for (int m = 0; m < n_mels; ++m) {
    int lo = nb, hi = 0;
    for (int k = 0; k < nb; ++k)
      if (fb[(size_t)m * nb + k] != 0.f) {
        lo = std::min(lo, k);
        hi = k + 1;
      }
    if (hi == 0) lo = 0;
    r.band[3 * m] = lo;
    r.band[3 * m + 1] = hi;
    r.band[3 * m + 2] = (int)r.w.size();
    for (int k = lo; k < hi; ++k) r.w.push_back(fb[(size_t)m * nb + k]);
  }
  return r;
}

static std::vector<float> hann_periodic(int n) {
  std::vector<float> w(n);
  for (int j = 0; j < n; ++j) w[j] = (float)(0.5 - 0.5 * cos(2.0 * M_PI * j / n));
  return w;
}

// ---------------------------------------------------------------------------- arena
struct Arena {
  char* base = nullptr;
  size_t cap = 0, off = 0, peak = 0;
  int reserve(size_t bytes) {
    if (bytes <= cap) return SVC_OK;
    if (base) SVC_HIP_CHECK(hipFree(base));
    base = nullptr;
    cap = 0;
    SVC_HIP_CHECK(hipMalloc(&base, bytes));
    cap = bytes;
    return SVC_OK;
  }
  void reset() { off = 0; }
  template <typename T>
  T* get(size_t n) {
    size_t bytes = (n * sizeof(T) + 255) & ~(size_t)255;
    if (off + bytes > cap) return nullptr;
    T* p = reinterpret_cast<T*>(base + off);
    off += bytes;
    if (off > peak) peak = off;
    return p;
  }
};

constexpr int kMaxSubStreams = 8;

struct PackedGemm {
  f16* W = nullptr;
  float* bias = nullptr;
  int N = 0, Npad = 0, K = 0, Kpad = 0, Cp = 0, Cin = 0, taps = 0;
  int tap_mul = 1, tap_add = 0, istride = 1;
  bool bf16 = false;  // W (and so the GEMM's operands) in bfloat16 (the bf16 operand variant, common.h Op16)
  f16* Wfrag = nullptr;  // W in a kernel's fragment order: the DiffSVC residual projections (res_proj.hip), the dilated
                         // convs (gate_ws.hip)
};

// host-side rounding of a weight to the 16-bit operand format: binary16 (default) or bfloat16 (round to nearest even)
static inline uint16_t bf16_bits(float v) {
  uint32_t u;
  memcpy(&u, &v, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static inline f16 enc16_host(float v, bool bf) {
  if (!bf) return (f16)v;
  const uint16_t b = bf16_bits(v);
  f16 h;
  memcpy(&h, &b, 2);
  return h;
}
static inline float round16_host(float v, bool bf) {
  if (!bf) return (float)(f16)v;
  const uint32_t u = (uint32_t)bf16_bits(v) << 16;
  float r;
  memcpy(&r, &u, 4);
  return r;
}

struct Param {
  const float* host = nullptr;
  std::vector<int64_t> shape;
  int64_t numel = 0;
};

struct WBlock {
  float *ln1_g, *ln1_b, *ln2_g, *ln2_b;
  PackedGemm qkv, out, fc1, fc2;
  PackedGemm v;         // value projection as its own GEMM when its weight split differs from q / k's
  bool split_v = false;  // (then qkv holds the q and k columns only)
};

struct HBlock {  // post-LN fairseq TransformerSentenceEncoderLayer
  float *ln1_g, *ln1_b, *ln2_g, *ln2_b;
  PackedGemm qkv, out, fc1, fc2;
};

struct ActP {
  float *alpha, *beta, *filt;
};

struct VStage {
  int cin, cout, rate, k;
  std::vector<PackedGemm> phases;
  // rate-2 ConvTranspose as ONE conv over the input rows (tune.amp_ups): output columns r * cout + n of input row t are
  // output row 2t + r, so [L][2 cout] is the time-major output; 3 taps at offsets +1, 0, -1 (each phase's two taps in
  // its own GEMM's order, zeros for the tap it lacks); run by amp_conv's plain-conv form (cin = 2 cout = 48 / 96 / 192)
  PackedGemm upc;
  bool up_comb = false;
  // resblocks j: convs1[l], convs2[l], acts[2l], acts[2l+1]
  std::vector<std::vector<PackedGemm>> c1, c2;
  std::vector<std::vector<ActP>> acts;
  std::vector<int> rk;
  std::vector<std::vector<int>> rd;
};

// ---------------------------------------------------------------------------- kernel switches
static thread_local const Tuning* t_tuning = nullptr;

// the switches by name: (tune.<name>, SVC_<NAME> environment override at context creation)
template <typename T>
static int* tuning_field(T& t, const char* name) {
  struct {
    const char* name;
    int* v;
  } ints[] = {{"gemm_variant", &t.gemm_variant},       {"gemm3_direct", &t.gemm3_direct},
              {"whisper_streams", &t.whisper_streams}, {"sampler_streams", &t.sampler_streams},
              {"vocoder_streams", &t.vocoder_streams}, {"diff_head", &t.diff_head},
              {"amp_maxc", &t.amp_maxc},               {"res_proj", &t.res_proj},
              {"gate_ws", &t.gate_ws},                 {"amp_ups", &t.amp_ups}};
  for (auto& it : ints)
    if (strcmp(it.name, name) == 0) return it.v;
  return nullptr;
}

void Tuning::from_env() {
  for (const char* name : {"gemm_variant", "gemm3_direct", "whisper_streams", "sampler_streams", "vocoder_streams",
                           "diff_head", "amp_maxc", "res_proj", "gate_ws", "amp_ups"}) {
    std::string env = "SVC_";
    for (const char* q = name; *q; ++q) env += (char)toupper((unsigned char)*q);
    if (const char* v = getenv(env.c_str())) *tuning_field(*this, name) = atoi(v);
  }
  if (const char* v = getenv("SVC_SITE_VARIANT")) site_variant = v;
}

bool Tuning::set(const char* name, double v) {
  int* f = tuning_field(*this, name);
  if (f) *f = (int)v;
  return f != nullptr;
}

bool Tuning::get(const char* name, double* v) const {
  int* f = tuning_field(const_cast<Tuning&>(*this), name);
  if (f) *v = *f;
  return f != nullptr;
}

const Tuning& tuning() {
  static const Tuning env_default = [] {
    Tuning t;
    t.from_env();
    return t;
  }();
  return t_tuning ? *t_tuning : env_default;
}
TuningScope::TuningScope(const Tuning* t) : prev(t_tuning) { t_tuning = t; }
TuningScope::~TuningScope() { t_tuning = prev; }
int ensure_dyn_lds(const void* fn, int bytes) {
  static std::mutex mu;
  static std::set<std::tuple<const void*, int, int>> done;
  int dev = 0;
  SVC_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(mu);
  if (done.count({fn, dev, bytes})) return SVC_OK;
  SVC_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  done.insert({fn, dev, bytes});
  return SVC_OK;
}

}  // namespace svc

using namespace svc;

// Device tables keyed by a parameter set (F0 front ends): an entry is built once and reused by every call with the same
// key, so a server alternating between parameter sets allocates nothing after the first call of each. At most kMax
// entries: beyond that the least recently used one is freed after the device has drained (a call in flight on any
// stream may still read it).
struct TableCache {
  static constexpr int kMax = 8;
  struct Entry {
    std::vector<double> key;
    double* dev;
    uint64_t used;
  };
  std::vector<Entry> e;
  uint64_t clock = 0;
  double* find(const double* key, int nk) {
    for (auto& x : e)
      if ((int)x.key.size() == nk && memcmp(x.key.data(), key, nk * sizeof(double)) == 0) {
        x.used = ++clock;
        return x.dev;
      }
    return nullptr;
  }
  // takes ownership of dev (hipMalloc'd)
  int insert(const double* key, int nk, double* dev) {
    if ((int)e.size() >= kMax) {
      size_t lru = 0;
      for (size_t i = 1; i < e.size(); ++i)
        if (e[i].used < e[lru].used) lru = i;
      SVC_HIP_CHECK(hipDeviceSynchronize());
      (void)hipFree(e[lru].dev);
      e.erase(e.begin() + (long)lru);
    }
    e.push_back(Entry{std::vector<double>(key, key + nk), dev, ++clock});
    return SVC_OK;
  }
  void clear() {
    for (auto& x : e) (void)hipFree(x.dev);
    e.clear();
  }
};

struct svc_ctx {
  int device = 0;
  Tuning tune, tune0;  // kernel switches (tune0: their values at creation, for "tune.reset")
  // ragged-batch length tables, one ring per stage (the feature stages run on their own stream)
  StageRing lens_feat, lens_main;
  std::map<std::string, Param> params;
  std::map<std::string, double> cfg;
  bool finalized = false;
  std::vector<void*> allocs;
  int64_t weight_bytes = 0;
  Arena ws;
  Arena auxws;  // workspace of the 24 kHz feature stages (mel / energy, F0): they may run on a side stream beside
               // the content encoder, which uses ws

  // features
  float *fb24 = nullptr, *fb16 = nullptr, *win_mel = nullptr, *win16 = nullptr;
  int *band24 = nullptr, *band16 = nullptr;  // [n_mels][3] nonzero band of each filter (lo, hi, offset in fb)
  int fb24_len = 0, fb16_len = 0;              // fb24 / fb16 hold only those bands, packed
  double *tw24 = nullptr, *tw16 = nullptr;     // FFT twiddles: [n_fft] (cos, -sin)(2 pi m / n_fft)
  int n_fft = 1024, hop = 256, n_mels = 100, fs = 24000;
  double fmin = 0, fmax = 12000, f0_min = 65, f0_max = 800;
  // content encoders in split-fp16 precision ("content.split" = 1 at finalize): every GEMM operand of Whisper /
  // HuBERT except the attention path is [hi | lo | hi] against [W_hi; W_hi; W_lo] weights (3x MFMA work)
  bool content_split = false;  // content_mode == 1
  int content_mode = 0;         // "content.split": 0 fp16, 1 split-fp16 operands (x3), 2 weight-split (x2, Whisper)
  bool head_split = true;  // DiffSVC skip_projection / output_projection on split-fp16 operands ("mapper.head_split")
  // bf16 operand variant ("operands.bf16" at finalize, BASELINE configs[4]'s fp16-vs-bf16 sweep): the DiffSVC,
  // conditioner and content-encoder GEMMs (and Whisper / HuBERT attention) take bfloat16 operands on
  // v_mfma_f32_16x16x32_bf16; BigVGAN stays binary16. pack_bf16: the weights being packed are for such a GEMM.
  bool bf16 = false;
  bool pack_bf16 = false;
  // whisper
  bool has_whisper = false;
  int wD = 0, wH = 0, wL = 0, wctx = 0, wmels = 80;
  PackedGemm wconv1, wconv2;
  int wstem_ld = 0;  // row stride (halves) of the conv stem's log-mel operand (split: 3 n_mels padded to 64)
  float *wpos = nullptr, *wlnp_g = nullptr, *wlnp_b = nullptr;
  std::vector<WBlock> wblocks;
  // hubert / contentvec (A8)
  bool has_hubert = false;
  int hC = 512, hD = 768, hH = 12, hLayers = 9, hFinal = 256, hPosK = 128, hPosG = 16;
  std::vector<PackedGemm> hconv;    // feature extractor conv_layers 0..6 (layer 0 as a 2-tap GEMM over 5-sample rows)
  std::vector<int> hconv_k, hconv_s;
  float *hgn_g = nullptr, *hgn_b = nullptr, *hln_g = nullptr, *hln_b = nullptr, *henc_ln_g = nullptr, *henc_ln_b = nullptr;
  PackedGemm hproj, hfinal;
  std::vector<PackedGemm> hpos;     // one GEMM per pos_conv group
  std::vector<HBlock> hblocks;
  // mapper
  bool has_mapper = false;
  int C = 384, n_mel = 100, n_layers = 20, dil_cycle = 4, steps = 1000, content_dim = 1024, n_bins = 256;
  PackedGemm content_lin, cp_all, melpre, skipproj, outproj;
  std::vector<PackedGemm> dil, outres;  // per layer: dilated conv (paired), residual half of output_projection
  PackedGemm skip_all;                  // skip halves of all layers' output_projection, K = layers * C
  float *emb_m = nullptr, *emb_l = nullptr, *emb_s = nullptr, *mbins = nullptr, *ebins = nullptr;
  float* dproj = nullptr;  // [steps][layers][C]
  std::vector<float> alphas_cumprod_f32, sra, srm1, pc1, pc2, plogvar;
  float *mel_min = nullptr, *mel_max = nullptr;
  // vocoder
  bool has_vocoder = false;
  int v_in = 100, v_c0 = 1536;
  bool v_rb2 = false;  // vocoder resblocks are AMPBlock2 (config resblock "2")
  PackedGemm vpre;
  std::vector<VStage> vstages;
  ActP vact_post;
  float* vpost_w = nullptr;
  float vpost_b = 0;
  float* fade = nullptr;
  int nfade = 5120;
  // sampler sub-batch streams (svc_diffsvc_sample), created on first use
  hipStream_t sub_streams[kMaxSubStreams] = {};
  hipEvent_t ev_fork = nullptr, ev_join[kMaxSubStreams] = {};
  int n_sub_streams = 0;
  int ensure_sub_streams(int n) {
    if (!ev_fork && hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming) != hipSuccess) return SVC_ERR_HIP;
    for (; n_sub_streams < n; ++n_sub_streams) {
      if (hipStreamCreateWithFlags(&sub_streams[n_sub_streams], hipStreamNonBlocking) != hipSuccess) return SVC_ERR_HIP;
      if (hipEventCreateWithFlags(&ev_join[n_sub_streams], hipEventDisableTiming) != hipSuccess) return SVC_ERR_HIP;
    }
    return SVC_OK;
  }
  int hop_out = 256;
  // pYIN's device tables (beta priors, banded log-transitions, bin frequencies) per (fs, f0_min, f0_max, win, hop), and
  // Praat-AC F0's window / window autocorrelation / FFT twiddle tables per (fs, f0_min) (f0.hip f0_tables): built once per
  // parameter set and reused by every later call with that set (TableCache)
  TableCache pyin_tabs, f0_tabs;
  ~svc_ctx() {
    pyin_tabs.clear();
    f0_tabs.clear();
  }
};

namespace {

int dev_upload(svc_ctx* c, const void* host, size_t bytes, void** out) {
  void* p = nullptr;
  SVC_HIP_CHECK(hipMalloc(&p, bytes > 0 ? bytes : 16));
  if (bytes) SVC_HIP_CHECK(hipMemcpy(p, host, bytes, hipMemcpyHostToDevice));
  c->allocs.push_back(p);
  c->weight_bytes += (int64_t)bytes;
  *out = p;
  return SVC_OK;
}

template <typename T>
int upload_vec(svc_ctx* c, const std::vector<T>& v, T** out) {
  return dev_upload(c, v.data(), v.size() * sizeof(T), reinterpret_cast<void**>(out));
}

const Param* getp(svc_ctx* c, const std::string& name, std::initializer_list<int64_t> shape) {
  auto it = c->params.find(name);
  if (it == c->params.end()) {
    set_error("missing parameter '%s'", name.c_str());
    return nullptr;
  }
  std::vector<int64_t> want(shape);
  if (want.size() != it->second.shape.size()) {
    set_error("parameter '%s': expected %zu dims, got %zu", name.c_str(), want.size(), it->second.shape.size());
    return nullptr;
  }
  for (size_t i = 0; i < want.size(); ++i)
    if (want[i] >= 0 && want[i] != it->second.shape[i]) {
      set_error("parameter '%s': dim %zu expected %lld got %lld", name.c_str(), i, (long long)want[i],
                (long long)it->second.shape[i]);
      return nullptr;
    }
  return &it->second;
}

#define GETP(var, name, ...)                           \
  const Param* var = getp(c, (name), {__VA_ARGS__});   \
  if (!var) return SVC_ERR_INVALID;

int upload_param(svc_ctx* c, const Param* p, float** out) {
  return dev_upload(c, p->host, (size_t)p->numel * sizeof(float), reinterpret_cast<void**>(out));
}

// generic packer: W16[n][tap*Cp + ci] = wget(n, ci, tap), bias[n] = bget(n)
template <typename WG, typename BG>
int pack_gemm(svc_ctx* c, PackedGemm& g, int N, int Cin, int Cp, int taps, WG wget, BG bget) {
  g.N = N;
  g.Cin = Cin;
  g.Cp = Cp;
  g.taps = taps;
  g.K = taps * Cp;
  g.Kpad = (int)round_up(g.K, 64);
  g.Npad = (int)std::max(round_up(N, 256), round_up(N, 384));  // every conv_gemm2/3 tile width fits
  g.bf16 = c->pack_bf16;
  std::vector<f16> w((size_t)g.Npad * g.Kpad, (f16)0.0f);  // +0 in both formats
  std::vector<float> b((size_t)g.Npad, 0.0f);
  for (int n = 0; n < N; ++n) {
    for (int t = 0; t < taps; ++t)
      for (int ci = 0; ci < Cin; ++ci)
        w[(size_t)n * g.Kpad + (size_t)t * Cp + ci] = enc16_host(wget(n, ci, t), g.bf16);
    b[n] = bget(n);
  }
  int st = upload_vec(c, w, &g.W);
  if (st) return st;
  return upload_vec(c, b, &g.bias);
}

// Split-fp16 packing of a 1-tap GEMM for the [x_hi | x_lo | x_hi] operand of f32_to_f16x3:
// W'[n] = [f16(w) | f16(w) | f16(w - f16(w))] over K = 3 * Cin.
// Cp > 3 * Cin: each tap's K segment padded to Cp (zero weights), e.g. to a multiple of 64 for the buffer-descriptor
// K-loop (the Whisper conv stem: 3 x 80 -> 256 per tap, its operand rows padded to match).
template <typename WG, typename BG>
int pack_gemm_split3(svc_ctx* c, PackedGemm& g, int N, int Cin, WG wget, BG bget, int taps = 1, int Cp = 0) {
  return pack_gemm(
      c, g, N, 3 * Cin, Cp > 0 ? Cp : 3 * Cin, taps,
      [&](int n, int ci, int t) {
        const int seg = ci / Cin;
        const float w = wget(n, ci - seg * Cin, t);
        const float hi = round16_host(w, c->pack_bf16);
        return seg < 2 ? hi : w - hi;
      },
      bget);
}

// Weight-split packing of a 1-tap GEMM (plain f16 operand): W'[n] = [f16(w) | f16(w - f16(w))] as TWO taps with a
// zero row shift, so the implicit-GEMM A loader reads the same activation row for both and the product carries the
// weights to ~22 significand bits at 2x the MFMA work, with no extra activation bytes. The weight rounding is the
// larger share of an fp16 linear's error (precision).
template <typename WG, typename BG>
int pack_gemm_wsplit2(svc_ctx* c, PackedGemm& g, int N, int Cin, WG wget, BG bget) {
  int st = pack_gemm(
      c, g, N, Cin, Cin, 2,
      [&](int n, int ci, int t) {
        const float w = wget(n, ci, 0);
        const float hi = round16_host(w, c->pack_bf16);
        return t == 0 ? hi : w - hi;
      },
      bget);
  g.tap_mul = 0;
  g.tap_add = 0;
  g.istride = 1;
  return st;
}

// a content-encoder linear in precision mode `mode` (0 fp16, 1 split-fp16 operands, 2 weight-split)
template <typename WG, typename BG>
int pack_linear_mode(svc_ctx* c, PackedGemm& g, int N, int Cin, int mode, WG wget, BG bget) {
  if (mode == 1) return pack_gemm_split3(c, g, N, Cin, wget, bget);
  if (mode == 2) return pack_gemm_wsplit2(c, g, N, Cin, wget, bget);
  return pack_gemm(c, g, N, Cin, Cin, 1, wget, bget);
}

// Conv1d weight [Cout][Cin][k] (optionally weight-normed along dim 0) into a packed GEMM
int pack_conv1d(svc_ctx* c, PackedGemm& g, const float* w, const float* bias, int Cout, int Cin, int k, int Cp,
                int dil, int pad, int stride, const std::vector<int>* perm = nullptr, const float* wn_g = nullptr) {
  std::vector<double> scale(Cout, 1.0);
  if (wn_g) {
    for (int o = 0; o < Cout; ++o) {
      double s = 0;
      for (int64_t i = 0; i < (int64_t)Cin * k; ++i) {
        double v = w[(int64_t)o * Cin * k + i];
        s += v * v;
      }
      scale[o] = (double)wn_g[o] / sqrt(s);
    }
  }
  auto src = [&](int n) { return perm ? (*perm)[n] : n; };
  int st = pack_gemm(
      c, g, Cout, Cin, Cp, k,
      [&](int n, int ci, int t) {
        int o = src(n);
        return (float)((double)w[((int64_t)o * Cin + ci) * k + t] * scale[o]);
      },
      [&](int n) { return bias ? bias[src(n)] : 0.0f; });
  g.tap_mul = dil;
  g.tap_add = -pad;
  g.istride = stride;
  return st;
}

// Conv1d [Cout][Cin][k] (+ bias) packed for a split-fp16 operand when `split`, else as pack_conv1d
int pack_conv1d_opt(svc_ctx* c, PackedGemm& g, const float* w, const float* bias, int Cout, int Cin, int k, int Cp,
                    int dil, int pad, int stride, bool split) {
  if (!split) return pack_conv1d(c, g, w, bias, Cout, Cin, k, Cp, dil, pad, stride);
  int st = pack_gemm_split3(
      c, g, Cout, Cin, [&](int n, int ci, int t) { return w[((int64_t)n * Cin + ci) * k + t]; },
      [&](int n) { return bias ? bias[n] : 0.0f; }, k);
  g.tap_mul = dil;
  g.tap_add = -pad;
  g.istride = stride;
  return st;
}

// ConvTranspose1d weight [Cin][Cout][k] (weight-normed along dim 0 = Cin) into `stride` phase GEMMs
int pack_conv_transpose(svc_ctx* c, std::vector<PackedGemm>& phases, const float* v, const float* wn_g,
                        const float* bias, int Cin, int Cout, int k, int s, int pad) {
  std::vector<double> scale(Cin, 1.0);
  if (wn_g) {
    for (int i = 0; i < Cin; ++i) {
      double acc = 0;
      for (int64_t j = 0; j < (int64_t)Cout * k; ++j) {
        double x = v[(int64_t)i * Cout * k + j];
        acc += x * x;
      }
      scale[i] = (double)wn_g[i] / sqrt(acc);
    }
  }
  if (k % s != 0) {
    set_error("conv_transpose: kernel %d not a multiple of stride %d", k, s);
    return SVC_ERR_INVALID;
  }
  phases.assign(s, PackedGemm());
  for (int r = 0; r < s; ++r) {
    const int base = (r + pad) % s, add = (r + pad) / s;
    int st = pack_gemm(
        c, phases[r], Cout, Cin, Cin, k / s,
        [&](int n, int ci, int j) {
          int kk = base + s * j;
          return (float)((double)v[((int64_t)ci * Cout + n) * k + kk] * scale[ci]);
        },
        [&](int n) { return bias ? bias[n] : 0.0f; });
    if (st) return st;
    phases[r].tap_mul = -1;
    phases[r].tap_add = add;
    phases[r].istride = 1;
  }
  return SVC_OK;
}

// The combined form of a rate-2 ConvTranspose (VStage::upc): phase r's tap j reads input row t + add_r - j with weight
// tap base_r + 2j (pack_conv_transpose); here tap q reads row t + 1 - q (amp_conv with k = 3, d = -1), so q = 1 - add_r + j.
// Built only where each phase's taps lie within offsets -1..1 and cin = 2 cout is an amp_conv plain-conv width. At cin 96 /
// 192 every 32-deep MFMA step lies within one tap, so each phase sums exactly its GEMM's products in its GEMM's order;
// at cin 48 the steps straddle taps and the zero tap shifts phase 0's grouping (fp32 summation order only).
int pack_conv_transpose_comb(svc_ctx* c, VStage& S, const float* v, const float* wn_g, const float* bias) {
  const int Cin = S.cin, Cout = S.cout, k = S.k, s = S.rate, pad = (S.k - S.rate) / 2;
  S.up_comb = false;
  if (s != 2 || k % s != 0 || Cin != 2 * Cout || !(Cin == 48 || Cin == 96 || Cin == 192)) return SVC_OK;
  for (int r = 0; r < s; ++r) {
    const int add = (r + pad) / s;
    if (add > 1 || add - (k / s - 1) < -1) return SVC_OK;
  }
  std::vector<double> scale(Cin, 1.0);
  if (wn_g) {
    for (int i = 0; i < Cin; ++i) {
      double acc = 0;
      for (int64_t j = 0; j < (int64_t)Cout * k; ++j) {
        double x = v[(int64_t)i * Cout * k + j];
        acc += x * x;
      }
      scale[i] = (double)wn_g[i] / sqrt(acc);
    }
  }
  int st = pack_gemm(
      c, S.upc, 2 * Cout, Cin, Cin, 3,
      [&](int n, int ci, int q) {
        const int r = n / Cout, o = n - r * Cout;
        const int base = (r + pad) % s, add = (r + pad) / s;
        const int j = q - 1 + add;
        if (j < 0 || j >= k / s) return 0.0f;
        return (float)((double)v[((int64_t)ci * Cout + o) * k + base + s * j] * scale[ci]);
      },
      [&](int n) { return bias ? bias[n % Cout] : 0.0f; });
  if (st) return st;
  S.up_comb = true;
  return SVC_OK;
}

// paired packing order (conv_gemm2 epilogue): packed n -> original channel ((n & 32) ? C : 0) + (n >> 6) * 32 + (n & 31)
std::vector<int> pair_perm(int C) {
  std::vector<int> p(2 * C);
  for (int n = 0; n < 2 * C; ++n) p[n] = ((n & 32) ? C : 0) + (n >> 6) * 32 + (n & 31);
  return p;
}

double cfgv(svc_ctx* c, const char* k, double d) {
  auto it = c->cfg.find(k);
  return it == c->cfg.end() ? d : it->second;
}

// 4 KiB of zeros: the LDS-DMA source of padded / out-of-range conv rows (conv_gemm2)
const f16* zero_page() {
  static f16* z = nullptr;
  if (!z) {
    if (hipMalloc(&z, 4096) != hipSuccess) return nullptr;
    if (hipMemset(z, 0, 4096) != hipSuccess) return nullptr;
  }
  return z;
}

// the kernel arguments of one implicit-GEMM launch over the packed weights g (run_gemm, the dual launches)
static ConvGemmArgs gemm_args(const PackedGemm& g, const f16* X, int ldx, int Cvalid, int B, int T_in, int T_out,
                              EpiArgs& e) {
  ConvGemmArgs a{};
  a.X = X;
  a.ldx = ldx;
  a.T_in = T_in;
  a.Cp = g.Cp;
  a.Cvalid = Cvalid;
  a.W = g.W;
  a.K = g.K;
  a.Kpad = g.Kpad;
  a.tap_mul = g.tap_mul;
  a.tap_add = g.tap_add;
  a.istride = g.istride;
  a.B = B;
  a.T_out = T_out;
  a.N = g.N;
  a.bf16 = g.bf16 ? 1 : 0;
  a.Wfrag = g.Wfrag;
  if (e.T_ostore == 0) {
    e.T_ostore = T_out;
    e.ostride = 1;
    e.ophase = 0;
  }
  if (!e.bias) e.bias = g.bias;
  return a;
}


// tv / tv_mul: ragged batches, utterance b's valid input rows are tv[b] * tv_mul (ConvGemmArgs::tv; NULL = all)
int run_gemm(const PackedGemm& g, const f16* X, int ldx, int Cvalid, int B, int T_in, int T_out, EpiArgs e,
             hipStream_t s, const char* site = "", const int* tv = nullptr, int tv_mul = 1) {
  prof_site(site);
  const Tuning& tu = tuning();
  // conv_gemm3's register epilogues (gemm3_direct mask, gemm3.hip) stay off inside the DiffSVC sampler unless
  // bit 8 is set: there its sub-batch GEMMs run beside the gate GEMMs of the other streams, which then ran slower
  if (!(tu.gemm3_direct & 8) && site && strncmp(site, "diffsvc.", 8) == 0) e.no_reg_epi = 1;
  ConvGemmArgs a = gemm_args(g, X, ldx, Cvalid, B, T_in, T_out, e);
  a.tv = tv;
  a.tv_mul = tv_mul;
  const bool pair = e.kind == EPI_GATE;
  // gemm_variant: 15 (default) = conv_gemm3 with the fitted tile choice, except the DiffSVC gate GEMM (paired
  // epilogue, K = 1152) which runs conv_gemm4 with its register gate epilogue (24; 3-9 % faster than conv_gemm3);
  // 10..14 = a fixed conv_gemm3 tile; 20 / 24 = conv_gemm4 with the LDS-staged / register gate epilogue.
  int variant = tu.gemm_variant;
  // site_variant = "site=variant,...": per-call-site override (tile / kernel A/B runs, e.g. diffsvc.outproj=20)
  if (!tu.site_variant.empty()) {
    const char* senv = tu.site_variant.c_str();
    const size_t sl = site ? strlen(site) : 0;
    for (const char* p = senv; sl && (p = strstr(p, site)) != nullptr; p += sl)
      if ((p == senv || p[-1] == ',') && p[sl] == '=') {
        variant = atoi(p + sl + 1);
        break;
      }
  }
  // the DiffSVC dilated conv + gate: the weight-stationary row stream (gate_ws.hip) where it fits, else conv_gemm4
  if (variant == 15 && pair && tu.gate_ws && gate_ws_fits(a, e)) return gate_ws(a, e, s);
  if (variant == 15 && pair) variant = 24;
  // The skip-sum GEMM of a sampler sub-batch (K = 20 x 384, M <= 20 k rows) takes conv_gemm3's 256 x 128 tile although
  // pick3's fit prefers narrower-M tiles alone: beside the other sampler stream it measured +1.5 % end to end (826-828
  // vs 813-818 audio-s/s in three alternating rounds, profiles/r03w_skipsum_tile_ab.txt)
  if (variant == 15 && site && strcmp(site, "diffsvc.skipsum") == 0 && (int64_t)B * T_out <= 20000) variant = 12;
  SVC_REQUIRE((variant >= 10 && variant <= 16) || variant == 20 || variant == 24, "gemm_variant %d: 10..16, 20 or 24",
              variant);
  // N <= 64 (the last BigVGAN up-sampling phases, 48 / 24 channels) takes conv_gemm3's 128 x 128 tile: 1.9 vs
  // 3.0 ms per step on the round-1 256 x 64 / 256 x 32 tiles (tools/ab_ups.sh), although 63-81 % of its N is padding
  if (variant == 20 || variant == 24) {
    if (pair || g.N > 64) return conv_gemm4(a, e, zero_page(), s, variant == 24);
    variant = 15;  // conv_gemm4's tiles are 128 wide in N: small-N GEMMs keep conv_gemm3
  }
  return conv_gemm3(a, e, zero_page(), variant - 10, s);
}

EpiArgs epi() {
  EpiArgs e{};
  e.kind = EPI_GENERIC;
  e.acc_div = 1.0f;
  return e;
}

// ---------------------------------------------------------------------------- finalize: whisper
int build_whisper(svc_ctx* c) {
  GETP(c1w, "whisper.encoder.conv1.weight", -1, -1, 3);
  const int D = (int)c1w->shape[0];
  const int nm = (int)c1w->shape[1];
  GETP(pos, "whisper.encoder.positional_embedding", -1, D);
  c->wD = D;
  c->wH = D / 64;
  c->wmels = nm;
  c->wctx = (int)pos->shape[0];
  int L = 0;
  while (c->params.count("whisper.encoder.blocks." + std::to_string(L) + ".attn.query.weight")) ++L;
  c->wL = L;
  GETP(c1b, "whisper.encoder.conv1.bias", D);
  GETP(c2w, "whisper.encoder.conv2.weight", D, D, 3);
  GETP(c2b, "whisper.encoder.conv2.bias", D);
  // precision: the conv stem is split-fp16 in both split modes; the blocks' linears follow content_mode
  const int mode = c->content_mode;
  const bool sp = mode != 0;
  SVC_REQUIRE(!sp || nm % 8 == 0, "whisper split precision: n_mels %d", nm);
  // the split stem's operand rows [hi | lo | hi] (3 n_mels = 240 wide) are stored 256 wide with a zero pad, and each
  // tap's K segment padded to match, so a K-tile of 64 lies in one tap (the K-loop's buffer-descriptor form):
  // 768 instead of 720-deep K, but no per-lane tap arithmetic
  int st;
  if (sp) {
    c->wstem_ld = (int)round_up(3 * nm, 64);
    st = pack_gemm_split3(
        c, c->wconv1, D, nm, [&](int n, int ci, int t) { return c1w->host[((int64_t)n * nm + ci) * 3 + t]; },
        [&](int n) { return c1b->host[n]; }, 3, c->wstem_ld);
    c->wconv1.tap_mul = 1;
    c->wconv1.tap_add = -1;
    c->wconv1.istride = 1;
  } else {
    c->wstem_ld = (int)round_up(nm, 8);
    st = pack_conv1d(c, c->wconv1, c1w->host, c1b->host, D, nm, 3, c->wstem_ld, 1, 1, 1);
  }
  if (st) return st;
  st = pack_conv1d_opt(c, c->wconv2, c2w->host, c2b->host, D, D, 3, D, 1, 1, 2, sp);
  if (st) return st;
  if ((st = upload_param(c, pos, &c->wpos))) return st;
  c->wblocks.resize(L);
  // default: the attention linears of every block and the MLP linears of blocks 0-3 (tools/precision_sweep.py, three
  // clips: de-normalised mel-L1 0.76-0.78e-3 against 0.72-0.74e-3 with every linear split and 0.84-0.86e-3 with the
  // attention linears only; the error enters early and through the attention; DESIGN.md "precision")
  const uint64_t wsplit_attn = (uint64_t)cfgv(c, "content.wsplit_attn", 9007199254740991.0);  // 2^53 - 1: all blocks
  const uint64_t wsplit_mlp = (uint64_t)cfgv(c, "content.wsplit_mlp", 15.0);
  // finer masks for the attention linears (default: wsplit_attn for each): q / k, v, out
  const uint64_t wsplit_qk = (uint64_t)cfgv(c, "content.wsplit_qk", (double)wsplit_attn);
  const uint64_t wsplit_v = (uint64_t)cfgv(c, "content.wsplit_v", (double)wsplit_attn);
  const uint64_t wsplit_out = (uint64_t)cfgv(c, "content.wsplit_out", (double)wsplit_attn);
  for (int i = 0; i < L; ++i) {
    std::string p = "whisper.encoder.blocks." + std::to_string(i) + ".";
    WBlock& b = c->wblocks[i];
    GETP(qw, p + "attn.query.weight", D, D);
    GETP(qb, p + "attn.query.bias", D);
    GETP(kw, p + "attn.key.weight", D, D);
    GETP(vw, p + "attn.value.weight", D, D);
    GETP(vb, p + "attn.value.bias", D);
    GETP(ow, p + "attn.out.weight", D, D);
    GETP(ob, p + "attn.out.bias", D);
    GETP(l1g, p + "attn_ln.weight", D);
    GETP(l1b, p + "attn_ln.bias", D);
    GETP(l2g, p + "mlp_ln.weight", D);
    GETP(l2b, p + "mlp_ln.bias", D);
    GETP(f1w, p + "mlp.0.weight", 4 * D, D);
    GETP(f1b, p + "mlp.0.bias", 4 * D);
    GETP(f2w, p + "mlp.2.weight", D, 4 * D);
    GETP(f2b, p + "mlp.2.bias", D);
    auto qkv_w = [&](int n, int ci, int) {
      const Param* w = n < D ? qw : (n < 2 * D ? kw : vw);
      return w->host[(int64_t)(n % D) * D + ci];
    };
    auto qkv_b = [&](int n) { return n < D ? qb->host[n] : (n < 2 * D ? 0.0f : vb->host[n - 2 * D]); };
    auto lin = [&](const Param* w) { return [w](int n, int ci, int) { return w->host[(int64_t)n * (w->shape[1]) + ci]; }; };
    auto bias = [&](const Param* b0) { return [b0](int n) { return b0->host[n]; }; };
    // weight-split mode: "content.wsplit_attn" / "content.wsplit_mlp" (bit i: block i) choose the blocks whose
    // attention linears (qkv, out) / MLP linears (fc1, fc2) get [W_hi; W_lo]; the others run on plain fp16 weights.
    // "content.wsplit_qk" / "content.wsplit_v" / "content.wsplit_out" refine the attention mask per linear (bits 1 /
    // 16 / 2 of lmode); fc1 / fc2 are bits 4 / 8
    auto lmode = [&](int bit) {
      if (mode != 2) return mode;
      const uint64_t m = bit == 1 ? wsplit_qk : bit == 2 ? wsplit_out : bit == 16 ? wsplit_v : wsplit_mlp;
      return ((m >> (i < 53 ? i : 52)) & 1) ? 2 : 0;
    };
    b.split_v = lmode(1) != lmode(16);
    if (!b.split_v) {
      if ((st = pack_linear_mode(c, b.qkv, 3 * D, D, lmode(1), qkv_w, qkv_b))) return st;
    } else {  // q | k on one GEMM, v on another, each with its own operand precision
      if ((st = pack_linear_mode(c, b.qkv, 2 * D, D, lmode(1), qkv_w, qkv_b))) return st;
      if ((st = pack_linear_mode(c, b.v, D, D, lmode(16), lin(vw), bias(vb)))) return st;
    }
    // the attention output (A of `out`) is fp16 (the attention kernel's P.V path is fp16 either way): split3 would
    // only split the weights, which the weight-split mode does at 2x
    if ((st = pack_linear_mode(c, b.out, D, D, mode == 2 ? lmode(2) : 0, lin(ow), bias(ob)))) return st;
    if ((st = pack_linear_mode(c, b.fc1, 4 * D, D, lmode(4), lin(f1w), bias(f1b)))) return st;
    if ((st = pack_linear_mode(c, b.fc2, D, 4 * D, lmode(8), lin(f2w), bias(f2b)))) return st;
    if ((st = upload_param(c, l1g, &b.ln1_g)) || (st = upload_param(c, l1b, &b.ln1_b)) ||
        (st = upload_param(c, l2g, &b.ln2_g)) || (st = upload_param(c, l2b, &b.ln2_b)))
      return st;
  }
  GETP(lpg, "whisper.encoder.ln_post.weight", D);
  GETP(lpb, "whisper.encoder.ln_post.bias", D);
  if ((st = upload_param(c, lpg, &c->wlnp_g)) || (st = upload_param(c, lpb, &c->wlnp_b))) return st;
  c->has_whisper = true;
  return SVC_OK;
}

// ---------------------------------------------------------------------------- finalize: hubert (A8)
// fairseq HubertModel (ContentVec) as utils/hubert.py:14-47 drives it; parameter names are fairseq's.
int build_hubert(svc_ctx* c) {
  GETP(c0, "hubert.feature_extractor.conv_layers.0.0.weight", -1, 1, 10);
  const int Cc = (int)c0->shape[0];
  GETP(pw, "hubert.post_extract_proj.weight", -1, Cc);
  const int D = (int)pw->shape[0];
  SVC_REQUIRE(D % 64 == 0 && D <= 1024 && Cc % 64 == 0 && Cc <= 1024, "hubert: embed %d / conv dim %d", D, Cc);
  c->hC = Cc;
  c->hD = D;
  c->hH = D / 64;
  int L = 0;
  while (c->params.count("hubert.encoder.layers." + std::to_string(L) + ".fc1.weight")) ++L;
  const int want = (int)cfgv(c, "hubert.output_layer", 9);
  SVC_REQUIRE(want >= 1 && L >= 1, "hubert: output_layer %d, %d layers", want, L);
  c->hLayers = std::min(want, L);  // fairseq's TransformerEncoder runs every layer when output_layer exceeds them
  int st;
  // conv_layers[0]: W0[n][0][tap*5 + j] -> packed K index tap*8 + j over rows of 5 samples
  c->hconv.assign(7, PackedGemm());
  c->hconv_k = {10, 3, 3, 3, 3, 2, 2};
  c->hconv_s = {5, 2, 2, 2, 2, 2, 2};
  const bool sp = c->content_mode != 0;  // HuBERT: split-fp16 in both split modes
  if (sp)  // split-fp16 frames rows [hi(5) | lo(5) | hi(5) | 0] against [W_hi | W_hi | W_lo | 0] per tap
    st = pack_gemm(
        c, c->hconv[0], Cc, 16, 16, 2,
        [&](int n, int ci, int t) {
          if (ci >= 15) return 0.0f;
          const int seg = ci / 5;
          const float w = c0->host[(int64_t)n * 10 + t * 5 + (ci - seg * 5)];
          const float hi = round16_host(w, c->pack_bf16);
          return seg < 2 ? hi : w - hi;
        },
        [&](int) { return 0.0f; });
  else
    st = pack_gemm(
        c, c->hconv[0], Cc, 5, 8, 2, [&](int n, int ci, int t) { return c0->host[(int64_t)n * 10 + t * 5 + ci]; },
        [&](int) { return 0.0f; });
  if (st) return st;
  c->hconv[0].tap_mul = 1;
  c->hconv[0].tap_add = 0;
  c->hconv[0].istride = 1;
  for (int i = 1; i < 7; ++i) {
    GETP(w, "hubert.feature_extractor.conv_layers." + std::to_string(i) + ".0.weight", Cc, Cc, c->hconv_k[i]);
    if ((st = pack_conv1d_opt(c, c->hconv[i], w->host, nullptr, Cc, Cc, c->hconv_k[i], Cc, 1, 0, 2, sp))) return st;
  }
  GETP(gng, "hubert.feature_extractor.conv_layers.0.2.weight", Cc);
  GETP(gnb, "hubert.feature_extractor.conv_layers.0.2.bias", Cc);
  GETP(lng, "hubert.layer_norm.weight", Cc);
  GETP(lnb, "hubert.layer_norm.bias", Cc);
  GETP(pb, "hubert.post_extract_proj.bias", D);
  if ((st = upload_param(c, gng, &c->hgn_g)) || (st = upload_param(c, gnb, &c->hgn_b)) ||
      (st = upload_param(c, lng, &c->hln_g)) || (st = upload_param(c, lnb, &c->hln_b)))
    return st;
  if ((st = pack_conv1d_opt(c, c->hproj, pw->host, pb->host, D, Cc, 1, Cc, 1, 0, 1, sp))) return st;
  // pos_conv: weight_norm(dim=2) -> w[o][i][k] = g[k] * v[o][i][k] / ||v[:, :, k]||; one GEMM per group
  GETP(pv, "hubert.encoder.pos_conv.0.weight_v", D, -1, -1);
  const int Cg = (int)pv->shape[1], kp = (int)pv->shape[2];
  GETP(pg, "hubert.encoder.pos_conv.0.weight_g", 1, 1, kp);
  GETP(pcb, "hubert.encoder.pos_conv.0.bias", D);
  SVC_REQUIRE(D % Cg == 0 && Cg % 8 == 0 && kp % 2 == 0, "hubert: pos_conv groups of %d, k=%d", Cg, kp);
  c->hPosK = kp;
  c->hPosG = D / Cg;
  std::vector<double> kscale(kp);
  for (int k = 0; k < kp; ++k) {
    double acc = 0;
    for (int64_t oi = 0; oi < (int64_t)D * Cg; ++oi) {
      const double v = pv->host[oi * kp + k];
      acc += v * v;
    }
    kscale[k] = (double)pg->host[k] / sqrt(acc);
  }
  c->hpos.assign(c->hPosG, PackedGemm());
  for (int gi = 0; gi < c->hPosG; ++gi) {
    auto pw_ = [&](int n, int ci, int t) {
      return (float)((double)pv->host[((int64_t)(gi * Cg + n) * Cg + ci) * kp + t] * kscale[t]);
    };
    auto pb_ = [&](int n) { return pcb->host[gi * Cg + n]; };
    st = sp ? pack_gemm_split3(c, c->hpos[gi], Cg, Cg, pw_, pb_, kp) : pack_gemm(c, c->hpos[gi], Cg, Cg, Cg, kp, pw_, pb_);
    if (st) return st;
    c->hpos[gi].tap_mul = 1;
    c->hpos[gi].tap_add = -kp / 2;  // padding k/2, SamePad drops the extra last frame
    c->hpos[gi].istride = 1;
  }
  GETP(elg, "hubert.encoder.layer_norm.weight", D);
  GETP(elb, "hubert.encoder.layer_norm.bias", D);
  if ((st = upload_param(c, elg, &c->henc_ln_g)) || (st = upload_param(c, elb, &c->henc_ln_b))) return st;
  c->hblocks.resize(c->hLayers);
  for (int i = 0; i < c->hLayers; ++i) {
    const std::string p = "hubert.encoder.layers." + std::to_string(i) + ".";
    HBlock& b = c->hblocks[i];
    GETP(qw, p + "self_attn.q_proj.weight", D, D);
    GETP(qb, p + "self_attn.q_proj.bias", D);
    GETP(kw, p + "self_attn.k_proj.weight", D, D);
    GETP(kb, p + "self_attn.k_proj.bias", D);
    GETP(vw, p + "self_attn.v_proj.weight", D, D);
    GETP(vb, p + "self_attn.v_proj.bias", D);
    GETP(ow, p + "self_attn.out_proj.weight", D, D);
    GETP(ob, p + "self_attn.out_proj.bias", D);
    GETP(l1g, p + "self_attn_layer_norm.weight", D);
    GETP(l1b, p + "self_attn_layer_norm.bias", D);
    GETP(l2g, p + "final_layer_norm.weight", D);
    GETP(l2b, p + "final_layer_norm.bias", D);
    GETP(f1w, p + "fc1.weight", -1, D);
    const int Fd = (int)f1w->shape[0];
    GETP(f1b, p + "fc1.bias", Fd);
    GETP(f2w, p + "fc2.weight", D, Fd);
    GETP(f2b, p + "fc2.bias", D);
    auto qkv_w = [&](int n, int ci, int) {
      const Param* w = n < D ? qw : (n < 2 * D ? kw : vw);
      return w->host[(int64_t)(n % D) * D + ci];
    };
    auto qkv_b = [&](int n) { return n < D ? qb->host[n] : (n < 2 * D ? kb->host[n - D] : vb->host[n - 2 * D]); };
    st = sp ? pack_gemm_split3(c, b.qkv, 3 * D, D, qkv_w, qkv_b) : pack_gemm(c, b.qkv, 3 * D, D, D, 1, qkv_w, qkv_b);
    if (st) return st;
    if ((st = pack_conv1d(c, b.out, ow->host, ob->host, D, D, 1, D, 1, 0, 1))) return st;  // A = attention output (fp16)
    SVC_REQUIRE(Fd % 8 == 0, "hubert: ffn width %d", Fd);
    if ((st = pack_conv1d_opt(c, b.fc1, f1w->host, f1b->host, Fd, D, 1, D, 1, 0, 1, sp))) return st;
    if ((st = pack_conv1d_opt(c, b.fc2, f2w->host, f2b->host, D, Fd, 1, Fd, 1, 0, 1, sp))) return st;
    if ((st = upload_param(c, l1g, &b.ln1_g)) || (st = upload_param(c, l1b, &b.ln1_b)) ||
        (st = upload_param(c, l2g, &b.ln2_g)) || (st = upload_param(c, l2b, &b.ln2_b)))
      return st;
  }
  GETP(fw, "hubert.final_proj.weight", -1, D);
  c->hFinal = (int)fw->shape[0];
  GETP(fb, "hubert.final_proj.bias", c->hFinal);
  if ((st = pack_conv1d_opt(c, c->hfinal, fw->host, fb->host, c->hFinal, D, 1, D, 1, 0, 1, sp))) return st;
  c->has_hubert = true;
  return SVC_OK;
}

// ---------------------------------------------------------------------------- finalize: mapper
int build_mapper(svc_ctx* c) {
  const int C = (int)cfgv(c, "mapper.residual_channels", 384);
  const int NL = (int)cfgv(c, "mapper.residual_layer_num", 20);
  const int nmel = (int)cfgv(c, "mapper.n_mel", 100);
  const int fc = (int)cfgv(c, "mapper.diffusion_fc_size", 128);
  c->C = C;
  c->n_layers = NL;
  c->n_mel = nmel;
  c->dil_cycle = (int)cfgv(c, "mapper.dilation_cycle_length", 4);
  const int ks = (int)cfgv(c, "mapper.residual_kernel_size", 3);
  if (ks != 3) {
    set_error("mapper: residual_kernel_size %d unsupported", ks);
    return SVC_ERR_INVALID;
  }
  const std::string p = "mapper.0.registered_modules_dict.";
  // One ContentEncoder Linear per content type (modules/encoder.py:144-148), summed with the other encoders:
  // packed as ONE GEMM over the content types' features concatenated along K in ascending name order
  // (the order of this map), with the biases summed.
  std::vector<const Param*> cws, cbs;
  {
    const std::string pre = p + "content_", suf = ".nn.weight";
    for (auto& kv : c->params) {
      const std::string& k = kv.first;
      if (k.rfind(pre, 0) == 0 && k.size() > pre.size() + suf.size() && k.compare(k.size() - suf.size(), suf.size(), suf) == 0) {
        const std::string ct = k.substr(pre.size(), k.size() - pre.size() - suf.size());
        GETP(w_, k, C, -1);
        GETP(b_, p + "content_" + ct + ".nn.bias", C);
        SVC_REQUIRE(w_->shape[1] % 8 == 0, "mapper: content_%s width %lld not a multiple of 8", ct.c_str(),
                    (long long)w_->shape[1]);
        cws.push_back(w_);
        cbs.push_back(b_);
      }
    }
  }
  SVC_REQUIRE(!cws.empty(), "missing parameter 'mapper.0.registered_modules_dict.content_<type>.nn.weight'");
  c->content_dim = 0;
  for (auto* w_ : cws) c->content_dim += (int)w_->shape[1];
  GETP(mb, p + "melody.melody_bins", -1);
  GETP(me, p + "melody.nn.weight", -1, C);
  GETP(eb, p + "loudness.energy_bins", mb->shape[0]);
  GETP(le, p + "loudness.nn.weight", me->shape[0], C);
  GETP(se, p + "singer.nn.weight", -1, C);
  c->n_bins = (int)me->shape[0];
  if (mb->shape[0] != c->n_bins - 1) {
    set_error("mapper: melody bins %lld vs embedding %d", (long long)mb->shape[0], c->n_bins);
    return SVC_ERR_INVALID;
  }
  int st;
  st = pack_gemm(
      c, c->content_lin, C, c->content_dim, c->content_dim, 1,
      [&](int n, int ci, int) {
        for (auto* w_ : cws) {
          const int d = (int)w_->shape[1];
          if (ci < d) return w_->host[(int64_t)n * d + ci];
          ci -= d;
        }
        return 0.0f;
      },
      [&](int n) {
        float b = 0.0f;
        for (auto* b_ : cbs) b += b_->host[n];
        return b;
      });
  if (st) return st;
  if ((st = upload_param(c, mb, &c->mbins)) || (st = upload_param(c, eb, &c->ebins)) ||
      (st = upload_param(c, me, &c->emb_m)) || (st = upload_param(c, le, &c->emb_l)) ||
      (st = upload_param(c, se, &c->emb_s)))
    return st;

  const std::string q = "mapper.1.";
  GETP(mpw, q + "mel_preprocess.projection.weight", C, nmel, 1);
  GETP(mpb, q + "mel_preprocess.projection.bias", C);
  if ((st = pack_conv1d(c, c->melpre, mpw->host, mpb->host, C, nmel, 1, (int)round_up(nmel, 8), 1, 0, 1))) return st;
  if (C == 384 && c->melpre.Kpad == 128 && c->melpre.K <= 128) {  // mel_proj's shape: W_mel in its fragment order
    void* wf = nullptr;
    SVC_HIP_CHECK(hipMalloc(&wf, mel_proj_pack_elems() * sizeof(f16)));
    c->allocs.push_back(wf);
    c->weight_bytes += (int64_t)(mel_proj_pack_elems() * sizeof(f16));
    c->melpre.Wfrag = reinterpret_cast<f16*>(wf);
    if ((st = mel_proj_pack(c->melpre.W, c->melpre.Kpad, c->melpre.Wfrag, 0))) return st;
    SVC_HIP_CHECK(hipStreamSynchronize(0));
  }
  GETP(p1w, q + "diffusion_embedding.projection1.weight", fc, 128);
  GETP(p1b, q + "diffusion_embedding.projection1.bias", fc);
  GETP(p2w, q + "diffusion_embedding.projection2.weight", fc, fc);
  GETP(p2b, q + "diffusion_embedding.projection2.bias", fc);
  GETP(table, "mapper.step_table", -1, 128);
  const int steps = (int)table->shape[0];
  c->steps = steps;
  std::vector<int> perm = pair_perm(C);
  c->dil.resize(NL);
  c->outres.resize(NL);
  std::vector<const Param*> opw_l(NL), opb_l(NL);
  std::vector<const Param*> cpw(NL), cpb(NL), dpw(NL), dpb(NL);
  for (int i = 0; i < NL; ++i) {
    std::string r = q + "residual_layers." + std::to_string(i) + ".";
    GETP(dw, r + "dilated_conv.weight", 2 * C, C, 3);
    GETP(db, r + "dilated_conv.bias", 2 * C);
    GETP(ow, r + "output_projection.weight", 2 * C, C, 1);
    GETP(ob, r + "output_projection.bias", 2 * C);
    GETP(cw2, r + "conditioner_projection.weight", 2 * C, -1, 1);
    GETP(cb2, r + "conditioner_projection.bias", 2 * C);
    GETP(pw, r + "diffusion_projection.weight", C, fc);
    GETP(pb, r + "diffusion_projection.bias", C);
    cpw[i] = cw2;
    cpb[i] = cb2;
    dpw[i] = pw;
    dpb[i] = pb;
    const int d = 1 << (i % c->dil_cycle);
    if ((st = pack_conv1d(c, c->dil[i], dw->host, db->host, 2 * C, C, 3, C, d, d, 1, &perm))) return st;
    if (C == 384 && c->dil[i].Kpad == 3 * C) {  // gate_ws's shape: its weights once more, in its fragment order
      void* wf = nullptr;
      SVC_HIP_CHECK(hipMalloc(&wf, gate_ws_pack_elems() * sizeof(f16)));
      c->allocs.push_back(wf);
      c->weight_bytes += (int64_t)(gate_ws_pack_elems() * sizeof(f16));
      c->dil[i].Wfrag = reinterpret_cast<f16*>(wf);
      if ((st = gate_ws_pack(c->dil[i].W, c->dil[i].Kpad, c->dil[i].Wfrag, 0))) return st;
      SVC_HIP_CHECK(hipStreamSynchronize(0));
    }
    // rows 0..C-1 of output_projection are the residual, C..2C-1 the skip (modules/diffsvc.py:229-231)
    if ((st = pack_conv1d(c, c->outres[i], ow->host, ob->host, C, C, 1, C, 1, 0, 1))) return st;
    if (C == 384) {  // res_proj's shape: its weights once more, in MFMA fragment order
      void* wf = nullptr;
      SVC_HIP_CHECK(hipMalloc(&wf, res_proj_pack_elems() * sizeof(f16)));
      c->allocs.push_back(wf);
      c->weight_bytes += (int64_t)(res_proj_pack_elems() * sizeof(f16));
      c->outres[i].Wfrag = reinterpret_cast<f16*>(wf);
      if ((st = res_proj_pack(c->outres[i].W, c->outres[i].Kpad, c->outres[i].Wfrag, 0))) return st;
      SVC_HIP_CHECK(hipStreamSynchronize(0));
    }
    opw_l[i] = ow;
    opb_l[i] = ob;
  }
  // sum over layers of skip_i = g_i @ Wskip_i + bskip_i is ONE GEMM over the concatenated gate outputs
  // [g_0 .. g_{L-1}] (K = L*C): no per-layer f32 skip read-modify-write
  st = pack_gemm(
      c, c->skip_all, C, NL * C, NL * C, 1,
      [&](int n, int ci, int) {
        const int l = ci / C, k = ci % C;
        return opw_l[l]->host[(int64_t)(C + n) * C + k];
      },
      [&](int n) {
        double b = 0;
        for (int l = 0; l < NL; ++l) b += opb_l[l]->host[C + n];
        return (float)b;
      });
  if (st) return st;
  const int cond_sz = (int)cpw[0]->shape[1];
  // all 20 conditioner projections as one GEMM (loop-invariant over diffusion steps: hoisted), in split-fp16
  // precision: it runs once per batch, and its rounding is the largest single denoiser-side term of the
  // mel-L1 error (precision sweep)
  st = pack_gemm_split3(
      c, c->cp_all, NL * 2 * C, cond_sz,
      [&](int n, int ci, int) {
        int layer = n / (2 * C), o = perm[n % (2 * C)];
        return cpw[layer]->host[(int64_t)o * cond_sz + ci];
      },
      [&](int n) {
        int layer = n / (2 * C), o = perm[n % (2 * C)];
        return cpb[layer]->host[o];
      });
  if (st) return st;
  GETP(spw, q + "skip_projection.weight", C, C, 1);
  GETP(spb, q + "skip_projection.bias", C);
  GETP(opw, q + "output_projection.weight", nmel, C, 1);
  GETP(opb, q + "output_projection.bias", nmel);
  // The head (skip_projection + output_projection, modules/diffsvc.py:315-319) on split-fp16 operands by default
  // ("mapper.head_split"): its rounding feeds eps directly and is, after the conditioner projection, the largest
  // denoiser-side term of the mel-L1 error (precision); 3x the MFMA work of two small K = 384 GEMMs.
  c->head_split = cfgv(c, "mapper.head_split", 1) != 0;
  if ((st = pack_conv1d_opt(c, c->skipproj, spw->host, spb->host, C, C, 1, C, 1, 0, 1, c->head_split))) return st;
  if ((st = pack_conv1d_opt(c, c->outproj, opw->host, opb->host, nmel, C, 1, C, 1, 0, 1, c->head_split))) return st;

  // step MLP + per-layer diffusion projections for every step (input-independent: precomputed)
  std::vector<float> dp((size_t)steps * NL * C);
  std::vector<double> h1(fc), h2(fc);
  auto silu = [](double x) { return x / (1.0 + exp(-x)); };
  for (int t = 0; t < steps; ++t) {
    const float* e = table->host + (size_t)t * 128;
    for (int o = 0; o < fc; ++o) {
      double a = p1b->host[o];
      for (int i = 0; i < 128; ++i) a += (double)p1w->host[o * 128 + i] * e[i];
      h1[o] = (float)silu((float)a);
    }
    for (int o = 0; o < fc; ++o) {
      double a = p2b->host[o];
      for (int i = 0; i < fc; ++i) a += (double)p2w->host[o * fc + i] * h1[i];
      h2[o] = (float)silu((float)a);
    }
    for (int l = 0; l < NL; ++l)
      for (int o = 0; o < C; ++o) {
        double a = dpb[l]->host[o];
        for (int i = 0; i < fc; ++i) a += (double)dpw[l]->host[o * fc + i] * h2[i];
        dp[((size_t)t * NL + l) * C + o] = (float)a;
      }
  }
  if ((st = upload_vec(c, dp, &c->dproj))) return st;

  // noise schedule constants (modules/diffsvcrepo_inference.py:163-197: numpy f64 -> f32)
  const double b0 = cfgv(c, "mapper.noise_schedule_factors.0", 1e-4);
  const double b1 = cfgv(c, "mapper.noise_schedule_factors.1", 0.02);
  std::vector<double> betas(steps);
  const double stp = (b1 - b0) / (steps - 1);
  for (int i = 0; i < steps; ++i) betas[i] = (i == steps - 1) ? b1 : i * stp + b0;
  c->alphas_cumprod_f32.resize(steps);
  c->sra.resize(steps);
  c->srm1.resize(steps);
  c->pc1.resize(steps);
  c->pc2.resize(steps);
  c->plogvar.resize(steps);
  double ac = 1.0;
  for (int i = 0; i < steps; ++i) {
    const double alpha = 1.0 - betas[i];
    const double prev = ac;
    ac = ac * alpha;
    c->alphas_cumprod_f32[i] = (float)ac;
    c->sra[i] = (float)sqrt(1.0 / ac);
    c->srm1[i] = (float)sqrt(1.0 / ac - 1);
    c->pc1[i] = (float)(betas[i] * sqrt(prev) / (1.0 - ac));
    c->pc2[i] = (float)((1.0 - prev) * sqrt(alpha) / (1.0 - ac));
    const double pv = betas[i] * (1.0 - prev) / (1.0 - ac);
    c->plogvar[i] = (float)log(pv > 1e-20 ? pv : 1e-20);
  }
  GETP(mn, "stats.mel_min", nmel);
  GETP(mx, "stats.mel_max", nmel);
  if ((st = upload_param(c, mn, &c->mel_min)) || (st = upload_param(c, mx, &c->mel_max))) return st;
  c->has_mapper = true;
  return SVC_OK;
}

// ---------------------------------------------------------------------------- finalize: vocoder
// Activation1d parameters (modules/bigvgan.py:234-307). The kernels take log-scale SnakeBeta parameters: the
// magnitude term is 1 / (exp(beta) + 1e-9) and the frequency exp(alpha). Snake (:42-92) is SnakeBeta with beta = alpha;
// linear-scale parameters (snake_logscale = false) are passed as their logarithms, which needs them positive.
int get_act(svc_ctx* c, const std::string& name, int ch, ActP& a) {
  const bool snake = cfgv(c, "vocoder.snake", 0) != 0;
  const bool logscale = cfgv(c, "vocoder.snake_logscale", 1) != 0;
  GETP(al, name + ".act.alpha", ch);
  const Param* be = al;
  if (!snake) {
    GETP(b, name + ".act.beta", ch);
    be = b;
  }
  GETP(fu, name + ".upsample.filter", 1, 1, 12);
  GETP(fd, name + ".downsample.lowpass.filter", 1, 1, 12);
  for (int i = 0; i < 12; ++i)
    if (fu->host[i] != fd->host[i]) {
      set_error("%s: up/down filters differ (unsupported)", name.c_str());
      return SVC_ERR_INVALID;
    }
  std::vector<float> av(al->host, al->host + ch), bv(be->host, be->host + ch);
  if (!logscale) {
    for (int i = 0; i < ch; ++i) {
      if (!(av[i] > 0.f) || !(bv[i] > 0.f)) {
        set_error("%s: snake_logscale=false needs positive alpha/beta (channel %d: %g, %g)", name.c_str(), i, av[i],
                  bv[i]);
        return SVC_ERR_INVALID;
      }
      av[i] = logf(av[i]);
      bv[i] = logf(bv[i]);
    }
  }
  int st;
  if ((st = upload_vec(c, av, &a.alpha)) || (st = upload_vec(c, bv, &a.beta)) || (st = upload_param(c, fu, &a.filt)))
    return st;
  return SVC_OK;
}

int build_vocoder(svc_ctx* c) {
  const int ns = (int)cfgv(c, "vocoder.n_stages", 6);
  const int nk = (int)cfgv(c, "vocoder.n_kernels", 3);
  const int C0 = (int)cfgv(c, "vocoder.upsample_initial_channel", 1536);
  const int vin = (int)cfgv(c, "vocoder.input_dim", 100);
  c->v_c0 = C0;
  c->v_in = vin;
  c->v_rb2 = cfgv(c, "vocoder.resblock", 1) == 2;
  int st;
  GETP(pv, "vocoder.conv_pre.weight_v", C0, vin, 7);
  GETP(pg, "vocoder.conv_pre.weight_g", C0, 1, 1);
  GETP(pb, "vocoder.conv_pre.bias", C0);
  if ((st = pack_conv1d(c, c->vpre, pv->host, pb->host, C0, vin, 7, (int)round_up(vin, 8), 1, 3, 1, nullptr, pg->host)))
    return st;
  c->vstages.resize(ns);
  int hop = 1;
  for (int i = 0; i < ns; ++i) {
    VStage& S = c->vstages[i];
    S.cin = C0 >> i;
    S.cout = C0 >> (i + 1);
    S.rate = (int)cfgv(c, ("vocoder.upsample_rates." + std::to_string(i)).c_str(), 2);
    S.k = (int)cfgv(c, ("vocoder.upsample_kernel_sizes." + std::to_string(i)).c_str(), 4);
    hop *= S.rate;
    std::string u = "vocoder.ups." + std::to_string(i) + ".0.";
    GETP(uv, u + "weight_v", S.cin, S.cout, S.k);
    GETP(ug, u + "weight_g", S.cin, 1, 1);
    GETP(ub, u + "bias", S.cout);
    if ((st = pack_conv_transpose(c, S.phases, uv->host, ug->host, ub->host, S.cin, S.cout, S.k, S.rate,
                                  (S.k - S.rate) / 2)))
      return st;
    if ((st = pack_conv_transpose_comb(c, S, uv->host, ug->host, ub->host))) return st;
    S.c1.resize(nk);
    S.c2.resize(nk);
    S.acts.resize(nk);
    S.rk.resize(nk);
    S.rd.resize(nk);
    const int ch = S.cout;
    for (int j = 0; j < nk; ++j) {
      const int kk = (int)cfgv(c, ("vocoder.resblock_kernel_sizes." + std::to_string(j)).c_str(), 3);
      S.rk[j] = kk;
      std::string rb = "vocoder.resblocks." + std::to_string(i * nk + j) + ".";
      const int nd = (int)cfgv(c, ("vocoder.resblock_dilation_sizes." + std::to_string(j) + ".n").c_str(), 3);
      S.c1[j].resize(nd);
      S.c2[j].resize(nd);
      S.acts[j].resize(2 * nd);
      S.rd[j].resize(nd);
      for (int l = 0; l < nd; ++l) {
        const int d =
            (int)cfgv(c, ("vocoder.resblock_dilation_sizes." + std::to_string(j) + "." + std::to_string(l)).c_str(), 1);
        S.rd[j][l] = d;
        if (c->v_rb2) {  // AMPBlock2 (modules/bigvgan.py:442-512): x = x + convs[l](activations[l](x)), dilation d
          std::string n = rb + "convs." + std::to_string(l) + ".";
          GETP(v, n + "weight_v", ch, ch, kk);
          GETP(g, n + "weight_g", ch, 1, 1);
          GETP(bb, n + "bias", ch);
          if ((st = pack_conv1d(c, S.c2[j][l], v->host, bb->host, ch, ch, kk, ch, d, (kk * d - d) / 2, 1, nullptr,
                                g->host)))
            return st;
          if ((st = get_act(c, rb + "activations." + std::to_string(l), ch, S.acts[j][2 * l + 1]))) return st;
          continue;
        }
        std::string n1 = rb + "convs1." + std::to_string(l) + ".", n2 = rb + "convs2." + std::to_string(l) + ".";
        GETP(v1, n1 + "weight_v", ch, ch, kk);
        GETP(g1, n1 + "weight_g", ch, 1, 1);
        GETP(b1, n1 + "bias", ch);
        GETP(v2, n2 + "weight_v", ch, ch, kk);
        GETP(g2, n2 + "weight_g", ch, 1, 1);
        GETP(b2, n2 + "bias", ch);
        if ((st = pack_conv1d(c, S.c1[j][l], v1->host, b1->host, ch, ch, kk, ch, d, (kk * d - d) / 2, 1, nullptr,
                              g1->host)))
          return st;
        if ((st = pack_conv1d(c, S.c2[j][l], v2->host, b2->host, ch, ch, kk, ch, 1, (kk - 1) / 2, 1, nullptr,
                              g2->host)))
          return st;
        if ((st = get_act(c, rb + "activations." + std::to_string(2 * l), ch, S.acts[j][2 * l]))) return st;
        if ((st = get_act(c, rb + "activations." + std::to_string(2 * l + 1), ch, S.acts[j][2 * l + 1]))) return st;
      }
    }
  }
  c->hop_out = hop;
  const int chl = C0 >> ns;
  if ((st = get_act(c, "vocoder.activation_post", chl, c->vact_post))) return st;
  GETP(qv, "vocoder.conv_post.weight_v", 1, chl, 7);
  GETP(qg, "vocoder.conv_post.weight_g", 1, 1, 1);
  GETP(qb, "vocoder.conv_post.bias", 1);
  {
    double s = 0;
    for (int i = 0; i < chl * 7; ++i) s += (double)qv->host[i] * qv->host[i];
    const double sc = qg->host[0] / sqrt(s);
    std::vector<float> w(chl * 7);
    for (int i = 0; i < chl * 7; ++i) w[i] = (float)(qv->host[i] * sc);
    if ((st = upload_vec(c, w, &c->vpost_w))) return st;
    c->vpost_b = qb->host[0];
  }
  GETP(fade, "vocoder.fade_out", -1);
  c->nfade = (int)fade->shape[0];
  if ((st = upload_param(c, fade, &c->fade))) return st;
  c->has_vocoder = true;
  return SVC_OK;
}

int build_features(svc_ctx* c) {
  c->fs = (int)cfgv(c, "fs", 24000);
  c->n_fft = (int)cfgv(c, "n_fft", 1024);
  c->hop = (int)cfgv(c, "hop_length", 256);
  c->n_mels = (int)cfgv(c, "n_mels", 100);
  c->fmin = cfgv(c, "fmin", 0);
  c->fmax = cfgv(c, "fmax", 12000);
  c->f0_min = cfgv(c, "f0_min", 65);
  c->f0_max = cfgv(c, "f0_max", 800);
  if ((int)cfgv(c, "win_length", 1024) != c->n_fft || !dft_mel_supported(c->n_fft)) {
    set_error("n_fft %d / win_length unsupported (n_fft 512, 1024 or 2048 and win_length == n_fft)", c->n_fft);
    return SVC_ERR_INVALID;
  }
  int st;
  const std::vector<float> fb24 = slaney_mel(c->fs, c->n_fft, c->n_mels, c->fmin, c->fmax);
  const std::vector<float> fb16 = slaney_mel(16000, 400, 80, 0.0, 8000.0);
  const FilterBands b24 = filter_bands(fb24, c->n_mels), b16 = filter_bands(fb16, 80);
  c->fb24_len = (int)b24.w.size();
  c->fb16_len = (int)b16.w.size();
  if ((st = upload_vec(c, b24.w, &c->fb24)) || (st = upload_vec(c, b16.w, &c->fb16))) return st;
  if ((st = upload_vec(c, b24.band, &c->band24)) || (st = upload_vec(c, b16.band, &c->band16))) return st;
  if ((st = upload_vec(c, fft_twiddles(c->n_fft), &c->tw24)) || (st = upload_vec(c, fft_twiddles(400), &c->tw16)))
    return st;
  if ((st = upload_vec(c, hann_periodic(c->n_fft), &c->win_mel))) return st;
  if ((st = upload_vec(c, hann_periodic(400), &c->win16))) return st;
  return SVC_OK;
}

}  // namespace

// ============================================================================ C-ABI
extern "C" {

const char* svc_last_error(void) { return get_error(); }
// 2: ragged-batch length tables (utt_samples / frames) in the stage entry points
int svc_abi_version(void) { return 3; }

svc_status svc_ctx_create(int device, svc_ctx** out) {
  SVC_REQUIRE(out, "svc_ctx_create: null out");
  int n = 0;
  SVC_HIP_CHECK(hipGetDeviceCount(&n));
  SVC_REQUIRE(device >= 0 && device < n, "svc_ctx_create: device %d of %d", device, n);
  SVC_HIP_CHECK(hipSetDevice(device));
  svc_ctx* c = new svc_ctx();
  c->device = device;
  c->tune.from_env();
  c->tune0 = c->tune;
  *out = c;
  return SVC_OK;
}

svc_status svc_ctx_destroy(svc_ctx* c) {
  if (!c) return SVC_OK;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  for (void* p : c->allocs) (void)hipFree(p);
  if (c->ws.base) (void)hipFree(c->ws.base);
  if (c->auxws.base) (void)hipFree(c->auxws.base);
  for (int i = 0; i < c->n_sub_streams; ++i) {
    (void)hipStreamDestroy(c->sub_streams[i]);
    (void)hipEventDestroy(c->ev_join[i]);
  }
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  c->lens_feat.release();
  c->lens_main.release();
  delete c;
  return SVC_OK;
}

static int op_ws(svc_ctx** tmp);

// the configuration keys the context reads (config.json's, flattened as SVCEngine._set_config writes them, and the
// precision keys): a misspelt or obsolete key fails instead of silently leaving its default in place
static bool known_config_key(const char* key) {
  static const char* exact[] = {
      "fs", "n_fft", "hop_length", "win_length", "n_mels", "fmin", "fmax", "f0_min", "f0_max",
      "mapper.residual_channels", "mapper.residual_layer_num", "mapper.n_mel", "mapper.diffusion_fc_size",
      "mapper.dilation_cycle_length", "mapper.residual_kernel_size", "mapper.noise_schedule_factors.0",
      "mapper.noise_schedule_factors.1", "mapper.head_split", "content.split", "content.wsplit_attn",
      "content.wsplit_mlp", "content.wsplit_qk", "content.wsplit_v", "content.wsplit_out", "hubert.output_layer",
      "vocoder.n_stages", "vocoder.n_kernels", "vocoder.upsample_initial_channel", "vocoder.input_dim",
      "vocoder.resblock", "vocoder.snake", "vocoder.snake_logscale", "operands.bf16"};
  for (const char* k : exact)
    if (strcmp(key, k) == 0) return true;
  // indexed lists: <prefix><i> or, for the dilations, <prefix><j>.n / <prefix><j>.<l>
  static const char* indexed[] = {"vocoder.upsample_rates.", "vocoder.upsample_kernel_sizes.",
                                  "vocoder.resblock_kernel_sizes.", "vocoder.resblock_dilation_sizes."};
  for (int i = 0; i < 4; ++i) {
    const size_t n = strlen(indexed[i]);
    if (strncmp(key, indexed[i], n) != 0) continue;
    const char* p = key + n;
    if (!isdigit((unsigned char)*p)) return false;
    while (isdigit((unsigned char)*p)) ++p;
    if (i < 3) return *p == 0;
    if (*p++ != '.') return false;
    if (strcmp(p, "n") == 0) return true;
    if (!isdigit((unsigned char)*p)) return false;
    while (isdigit((unsigned char)*p)) ++p;
    return *p == 0;
  }
  return false;
}

svc_status svc_ctx_set_config(svc_ctx* c, const char* key, double value) {
  SVC_REQUIRE(key, "set_config: null key");
  if (strncmp(key, "tune.", 5) == 0) {  // kernel switches (Tuning); NULL context: the op-level entry points'
    if (!c) op_ws(&c);
    if (strcmp(key + 5, "reset") == 0) {
      c->tune = c->tune0;
      return SVC_OK;
    }
    SVC_REQUIRE(c->tune.set(key + 5, value), "set_config: unknown kernel switch %s", key);
    return SVC_OK;
  }
  SVC_REQUIRE(c, "set_config: null context");
  SVC_REQUIRE(known_config_key(key), "set_config: unknown configuration key %s", key);
  c->cfg[key] = value;
  return SVC_OK;
}

int svc_config_key_known(const char* key) { return key && known_config_key(key) ? 1 : 0; }

svc_status svc_ctx_get_config(svc_ctx* c, const char* key, double* value) {
  SVC_REQUIRE(key && value, "get_config: null argument");
  if (strncmp(key, "tune.", 5) == 0) {
    if (!c) op_ws(&c);
    SVC_REQUIRE(c->tune.get(key + 5, value), "get_config: unknown kernel switch %s", key);
    return SVC_OK;
  }
  SVC_REQUIRE(c, "get_config: null context");
  auto it = c->cfg.find(key);
  SVC_REQUIRE(it != c->cfg.end(), "get_config: %s is not set", key);
  *value = it->second;
  return SVC_OK;
}

svc_status svc_ctx_add_param(svc_ctx* c, const char* name, const float* host, int ndim, const int64_t* shape) {
  SVC_REQUIRE(c && name && host && ndim >= 0 && ndim <= 8, "add_param: bad args");
  if (c->finalized) {
    set_error("add_param after finalize");
    return SVC_ERR_STATE;
  }
  Param p;
  p.host = host;
  p.numel = 1;
  for (int i = 0; i < ndim; ++i) {
    p.shape.push_back(shape[i]);
    p.numel *= shape[i];
  }
  c->params[name] = p;
  return SVC_OK;
}

svc_status svc_ctx_finalize(svc_ctx* c) {
  SVC_REQUIRE(c, "finalize: null");
  if (c->finalized) {
    set_error("finalize called twice");
    return SVC_ERR_STATE;
  }
  SVC_HIP_CHECK(hipSetDevice(c->device));
  int st;
  if ((st = build_features(c))) return st;
  bool any_w = false, any_m = false, any_v = false, any_h = false;
  for (auto& kv : c->params) {
    any_w |= kv.first.rfind("whisper.", 0) == 0;
    any_h |= kv.first.rfind("hubert.", 0) == 0;
    any_m |= kv.first.rfind("mapper.", 0) == 0;
    any_v |= kv.first.rfind("vocoder.", 0) == 0;
  }
  c->content_mode = (int)cfgv(c, "content.split", 0);
  SVC_REQUIRE(c->content_mode >= 0 && c->content_mode <= 2, "content.split %d: 0 fp16, 1 split-fp16, 2 weight-split",
              c->content_mode);
  c->content_split = c->content_mode == 1;
  c->bf16 = cfgv(c, "operands.bf16", 0) != 0;
  c->pack_bf16 = c->bf16;  // the content encoders, the conditioner and DiffSVC
  if (any_w && (st = build_whisper(c))) return st;
  if (any_h && (st = build_hubert(c))) return st;
  if (any_m && (st = build_mapper(c))) return st;
  c->pack_bf16 = false;  // BigVGAN stays binary16
  if (any_v && (st = build_vocoder(c))) return st;
  c->params.clear();  // host arrays are no longer referenced
  c->finalized = true;
  return SVC_OK;
}

// One of the context's own sub-streams (created on first use, the same ones the sampler / vocoder / Whisper
// sub-batches run on), so a host pipeline can overlap stage calls without adding a stream (measured: 737 -> 644
// audio-s/s when the F0 stage got a stream of its own, presumably from sharing the 4 hardware queues).
svc_status svc_ctx_stream(svc_ctx* c, int index, void** stream) {
  SVC_REQUIRE(c && stream && index >= 0 && index < kMaxSubStreams, "ctx_stream: bad args");
  SVC_HIP_CHECK(hipSetDevice(c->device));
  int st;
  if ((st = c->ensure_sub_streams(index + 1))) return st;
  *stream = (void*)c->sub_streams[index];
  return SVC_OK;
}

svc_status svc_ctx_memory(svc_ctx* c, int64_t* wb, int64_t* wsb) {
  SVC_REQUIRE(c, "memory: null");
  if (wb) *wb = c->weight_bytes;
  if (wsb) *wsb = (int64_t)c->ws.cap;
  return SVC_OK;
}

svc_status svc_profile_enable(int enable) {
  if (!enable || !g_prof) {
    for (auto& r : g_prof_recs) {
      g_ev_pool.push_back(r.a);
      g_ev_pool.push_back(r.b);
    }
    g_prof_recs.clear();
  }
  g_prof = enable != 0;
  return SVC_OK;
}

svc_status svc_profile_filter(const char* kernel_prefix) {
  g_prof_filter = kernel_prefix ? kernel_prefix : "";
  return SVC_OK;
}

svc_status svc_profile_read(int idx, char* name, int name_len, double* total_ms, int64_t* launches, double* flops,
                            double* bytes, int* n_kernels) {
  // aggregate by kernel name (synchronises on the recorded events)
  std::vector<std::string> names;
  std::map<std::string, std::tuple<double, int64_t, double, double>> agg;
  for (auto& r : g_prof_recs) {
    SVC_HIP_CHECK(hipEventSynchronize(r.b));
    float ms = 0;
    SVC_HIP_CHECK(hipEventElapsedTime(&ms, r.a, r.b));
    if (!agg.count(r.name)) names.push_back(r.name);
    auto& t = agg[r.name];
    std::get<0>(t) += ms;
    std::get<1>(t) += 1;
    std::get<2>(t) += r.flops;
    std::get<3>(t) += r.bytes;
  }
  if (n_kernels) *n_kernels = (int)names.size();
  if (idx < 0 || idx >= (int)names.size()) return SVC_OK;
  auto& t = agg[names[idx]];
  if (name && name_len > 0) snprintf(name, name_len, "%s", names[idx].c_str());
  if (total_ms) *total_ms = std::get<0>(t);
  if (launches) *launches = std::get<1>(t);
  if (flops) *flops = std::get<2>(t);
  if (bytes) *bytes = std::get<3>(t);
  return SVC_OK;
}

svc_status svc_mel_filterbank(int sr, int n_fft, int n_mels, double fmin, double fmax, float* out) {
  SVC_REQUIRE(out && n_fft > 0 && n_mels > 0, "mel_filterbank: bad args");
  auto w = slaney_mel(sr, n_fft, n_mels, fmin, fmax);
  memcpy(out, w.data(), w.size() * sizeof(float));
  return SVC_OK;
}

#define CTX_READY(c)                                                        \
  TuningScope tuning_scope_((c) ? &(c)->tune : nullptr);                    \
  do {                                                                      \
    SVC_REQUIRE((c), "null context");                                       \
    if (!(c)->finalized) {                                                  \
      set_error("context not finalized");                                   \
      return SVC_ERR_STATE;                                                 \
    }                                                                       \
    SVC_HIP_CHECK(hipSetDevice((c)->device));                               \
  } while (0)

#define WS_GET(T, var, n)                                                               \
  T* var = c->ws.get<T>((size_t)(n));                                                   \
  if (!var) {                                                                           \
    set_error("workspace exhausted at %s (need %zu bytes more)", #var, (size_t)(n) * sizeof(T)); \
    return SVC_ERR_STATE;                                                               \
  }

// ---------------------------------------------------------------------------- mel + energy
// mel frames of an n-sample clip (utils/mel.py:148-167: reflect pad (n_fft - hop) / 2 each side, center=False)
static int64_t mel_frames_of(const svc_ctx* c, int64_t n) {
  const int pad = (c->n_fft - c->hop) / 2;
  return (n + 2 * pad - c->n_fft) / c->hop + 1;
}

// ragged batches: validate the per-utterance sample counts (host) and stage them with their mel frame counts
// (int64 n[B] then int T[B]) to the device through `ring`
static int stage_samples(svc_ctx* c, StageRing& ring, const int64_t* n_samples, int B, int64_t n, hipStream_t s,
                         const int64_t** nb_dev, const int** Tb_dev, std::vector<int>* Tb_host) {
  *nb_dev = nullptr;
  *Tb_dev = nullptr;
  if (!n_samples) return SVC_OK;
  const int pad = (c->n_fft - c->hop) / 2;
  std::vector<char> buf((size_t)B * (8 + 4));
  int64_t* nv = reinterpret_cast<int64_t*>(buf.data());
  int* tv = reinterpret_cast<int*>(buf.data() + (size_t)B * 8);
  Tb_host->resize(B);
  for (int b = 0; b < B; ++b) {
    SVC_REQUIRE(n_samples[b] > pad && n_samples[b] <= n, "utterance %d: %lld samples (batch length %lld)", b,
                (long long)n_samples[b], (long long)n);
    nv[b] = n_samples[b];
    tv[b] = (int)mel_frames_of(c, n_samples[b]);
    (*Tb_host)[b] = tv[b];
  }
  void* dev = nullptr;
  int st = ring.put(buf.data(), buf.size(), s, &dev);
  if (st) return st;
  *nb_dev = reinterpret_cast<const int64_t*>(dev);
  *Tb_dev = reinterpret_cast<const int*>(reinterpret_cast<char*>(dev) + (size_t)B * 8);
  return SVC_OK;
}

svc_status svc_mel_energy(svc_ctx* c, const float* wav, int B, int64_t n, const int64_t* n_samples, float* mel,
                          float* energy, void* stream) {
  CTX_READY(c);
  hipStream_t s = (hipStream_t)stream;
  const int pad = (c->n_fft - c->hop) / 2;
  const int64_t T64 = mel_frames_of(c, n);
  SVC_REQUIRE(B > 0 && n > pad && T64 > 0 && T64 < (1 << 30), "mel_energy: n=%lld", (long long)n);
  const int T = (int)T64, nb = c->n_fft / 2 + 1;
  const int64_t* nb_dev;
  const int* Tb_dev;
  std::vector<int> Tb_host;
  RingRetire retire_(c->lens_feat, s);
  int st0 = stage_samples(c, c->lens_feat, n_samples, B, n, s, &nb_dev, &Tb_dev, &Tb_host);
  if (st0) return st0;
  int st;
  DftArgs a{};
  a.wav = wav;
  a.wav_stride = n;
  a.n_valid = n;
  a.n_logical = n;
  a.n_fft = c->n_fft;
  a.hop = c->hop;
  a.pad = pad;
  a.n_frames = T;
  a.nbins = nb;
  a.window = c->win_mel;
  a.twiddle = reinterpret_cast<const double2*>(c->tw24);
  a.mode = 0;
  a.fb = c->fb24;
  a.band = c->band24;
  a.fb_len = c->fb24_len;
  a.n_mels = c->n_mels;
  a.out = mel;
  a.energy = energy;
  a.nb = nb_dev;
  a.Tb = Tb_dev;
  if ((st = dft_mel(a, B, s))) return st;
  if (Tb_dev && ((st = zero_tail_rows(mel, B, T, c->n_mels, Tb_dev, s)) || (st = zero_tail_rows(energy, B, T, 1, Tb_dev, s))))
    return st;
  return SVC_OK;
}

// ---------------------------------------------------------------------------- F0
svc_status svc_f0_ac(svc_ctx* c, const float* wav, int B, int64_t n, const int64_t* n_samples, int T, double* f0,
                     void* stream) {
  CTX_READY(c);
  const double ts = (double)c->hop / c->fs;
  size_t need = f0_workspace_bytes(B, n, c->fs, ts, c->f0_min);
  int st;
  if ((st = c->auxws.reserve(std::max(need + 4096, c->auxws.cap)))) return st;
  std::vector<int> Tb;
  if (n_samples) {
    Tb.resize(B);
    for (int b = 0; b < B; ++b) Tb[b] = (int)mel_frames_of(c, n_samples[b]);
  }
  const double key[2] = {(double)c->fs, c->f0_min};
  double* f0_tab = c->f0_tabs.find(key, 2);
  if (!f0_tab) {
    std::vector<double> tab(f0_table_doubles(c->fs, c->f0_min));
    if ((st = f0_tables(c->fs, c->f0_min, tab.data()))) return st;
    void* p = nullptr;
    SVC_HIP_CHECK(hipMalloc(&p, tab.size() * 8));
    const hipError_t me = hipMemcpy(p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice);
    if (me != hipSuccess) (void)hipFree(p);
    SVC_HIP_CHECK(me);
    f0_tab = reinterpret_cast<double*>(p);
    if ((st = c->f0_tabs.insert(key, 2, f0_tab))) return st;
  }
  RingRetire retire_(c->lens_feat, (hipStream_t)stream);
  return f0_praat_ac(wav, B, n, c->fs, ts, c->f0_min, c->f0_max, 0.6, T, f0, c->auxws.base, c->auxws.cap, f0_tab,
                     (hipStream_t)stream, n_samples, n_samples ? Tb.data() : nullptr, &c->lens_feat);
}

svc_status svc_f0_pyin(svc_ctx* c, const float* wav, int B, int64_t n, const int64_t* n_samples, double fs,
                       int win_length, int hop_length, double f0_min, double f0_max, int T, double* f0, void* stream) {
  SVC_REQUIRE(c, "null context");
  TuningScope tuning_scope_(&c->tune);
  SVC_HIP_CHECK(hipSetDevice(c->device));
  const int FL = 2048;  // librosa.pyin frame_length default (utils/f0.py:107 leaves it unset)
  const size_t nt = pyin_table_doubles(fs, f0_min, f0_max, FL, win_length, hop_length);
  if (!nt) return SVC_ERR_INVALID;  // (pyin_plan set the error)
  SVC_REQUIRE(B > 0 && n > 0 && T > 0, "pyin: B=%d n=%lld T=%d", B, (long long)n, T);
  const size_t need = pyin_workspace_bytes(B, T, fs, f0_min, f0_max, FL, win_length, hop_length);
  int st;
  if ((st = c->auxws.reserve(std::max(need + 4096, c->auxws.cap)))) return st;
  // the tables depend only on (fs, f0_min, f0_max, win, hop): built and uploaded once per parameter set
  const double key[5] = {fs, f0_min, f0_max, (double)win_length, (double)hop_length};
  double* pyin_tab = c->pyin_tabs.find(key, 5);
  if (!pyin_tab) {
    std::vector<double> tab(nt);
    if ((st = pyin_tables(fs, f0_min, f0_max, FL, win_length, hop_length, tab.data()))) return st;
    void* p = nullptr;
    SVC_HIP_CHECK(hipMalloc(&p, nt * 8));
    const hipError_t me = hipMemcpy(p, tab.data(), nt * 8, hipMemcpyHostToDevice);
    if (me != hipSuccess) (void)hipFree(p);
    SVC_HIP_CHECK(me);
    pyin_tab = reinterpret_cast<double*>(p);
    if ((st = c->pyin_tabs.insert(key, 5, pyin_tab))) return st;
  }
  // only the per-call lengths are staged (the ring retires its last slot)
  hipStream_t s = (hipStream_t)stream;
  RingRetire retire_(c->lens_feat, s);
  const int64_t* nb_dev = nullptr;
  if (n_samples) {
    void* dev = nullptr;
    if ((st = c->lens_feat.put(n_samples, (size_t)B * 8, s, &dev))) return st;
    nb_dev = reinterpret_cast<const int64_t*>(dev);
  }
  return f0_pyin(wav, B, n, nb_dev, n_samples, fs, f0_min, f0_max, FL, win_length, hop_length, T, f0, c->auxws.base,
                 c->auxws.cap, pyin_tab, s);
}

svc_status svc_pitch_shift(svc_ctx* c, double* f0, int B, int T, double target_median, void* stream) {
  SVC_REQUIRE(c && f0 && B > 0 && T > 0, "pitch_shift: bad args");
  SVC_HIP_CHECK(hipSetDevice(c->device));
  return pitch_shift(f0, B, T, target_median, (hipStream_t)stream);
}

// ---------------------------------------------------------------------------- whisper
svc_status svc_whisper_encode(svc_ctx* c, const float* wav16, int B, int64_t n, float* feats, void* stream) {
  CTX_READY(c);
  SVC_REQUIRE(c->has_whisper, "whisper weights not loaded");
  hipStream_t s = (hipStream_t)stream;
  const int64_t NS = 480000;  // utils/whisper_extractor/audio.py:18 (30 s @ 16 kHz)
  const int F = 3000, D = c->wD, L = c->wctx;
  SVC_REQUIRE(B > 0 && n > 0, "whisper: B=%d n=%lld", B, (long long)n);
  SVC_REQUIRE(L * 2 == F, "whisper: n_ctx %d != 1500", L);
  const int nb = 201;
  const size_t rows1 = (size_t)B * F, rows2 = (size_t)B * L;
  const int X3 = c->content_split ? 3 : 1;  // split-fp16 block operands are [hi | lo | hi] rows
  const int XS = c->content_mode != 0 ? 3 : 1;  // the conv stem is split-fp16 in both split modes
  const int LDM = XS == 3 ? c->wstem_ld : c->wmels;  // the stem operand's row stride
  size_t need = rows1 * c->wmels * 4 + rows1 * LDM * 2 + rows1 * D * 2 * XS /*h1*/ +
                rows2 * D * 4 + rows2 * D * 2 * X3 + rows2 * 3 * D * 2 + rows2 * D * 2 + rows2 * 4 * D * 2 * X3 + 64 * 4096;
  int st;
  if ((st = c->ws.reserve(std::max(need, c->ws.cap)))) return st;
  c->ws.reset();
  WS_GET(float, ls, rows1 * c->wmels);
  WS_GET(f16, lm16, rows1 * LDM);
  WS_GET(float, mx, B);
  DftArgs a{};
  a.wav = wav16;
  a.wav_stride = n;
  a.n_valid = std::min<int64_t>(n, NS);
  a.n_logical = NS;
  a.n_fft = 400;
  a.hop = 160;
  a.pad = 200;
  a.n_frames = F;
  a.nbins = nb;
  a.window = c->win16;
  a.twiddle = reinterpret_cast<const double2*>(c->tw16);
  a.mode = 1;
  a.fb = c->fb16;
  a.band = c->band16;
  a.fb_len = c->fb16_len;
  a.n_mels = c->wmels;
  a.out = ls;
  if ((st = dft_mel(a, B, s))) return st;
  if ((st = whisper_normalize(ls, mx, lm16, B, (int64_t)F * c->wmels, s, XS == 3 ? c->wmels : 0, c->bf16, LDM)))
    return st;
  // conv stem
  WS_GET(f16, h1, rows1 * D * XS);
  EpiArgs e = epi();
  e.act = ACT_GELU;
  e.out16 = h1;
  e.ld16 = D * XS;
  e.split16 = XS == 3 ? D : 0;
  if ((st = run_gemm(c->wconv1, lm16, LDM, LDM, B, F, F, e, s, "whisper.conv1"))) return st;
  WS_GET(float, x, rows2 * D);
  e = epi();
  e.act = ACT_GELU;
  e.add_t = c->wpos;
  e.ld_add_t = D;
  e.out32 = x;
  e.ld32 = D;
  if ((st = run_gemm(c->wconv2, h1, D * XS, D * XS, B, F, L, e, s, "whisper.conv2"))) return st;
  WS_GET(f16, n16, rows2 * D * X3);
  WS_GET(f16, qkv, rows2 * 3 * D);
  WS_GET(f16, o16, rows2 * D);
  WS_GET(f16, h16, rows2 * 4 * D * X3);
  const float qk_scale = powf((float)(D / c->wH), -0.25f);
  // whisper_streams = n > 1 runs the 24 blocks as utterance-aligned sub-batches on n streams (as the sampler
  // does): rows are time-major per utterance, so a sub-batch is a row range of every buffer, and one sub-batch's
  // HBM-bound GEMM epilogues / layer norms run beside the other's MFMA phases. Default 1: with the F0 stage on its
  // side stream the single full-batch stream measured 0.3-0.4 % faster end to end (three A/B pairs, r01i kernels).
  const int NSW = std::max(1, std::min(std::min(tuning().whisper_streams, B), (int)kMaxSubStreams));
  if ((st = c->ensure_sub_streams(NSW))) return st;
  if (NSW > 1) {
    SVC_HIP_CHECK(hipEventRecord(c->ev_fork, s));
    for (int h = 0; h < NSW; ++h) SVC_HIP_CHECK(hipStreamWaitEvent(c->sub_streams[h], c->ev_fork, 0));
  }
  for (int i = 0; i < c->wL; ++i) {
    WBlock& b = c->wblocks[i];
    for (int h = 0; h < NSW; ++h) {
      const int b0 = h * B / NSW, Bh = (h + 1) * B / NSW - b0;
      const size_t r = (size_t)b0 * L, rows_h = (size_t)Bh * L;
      hipStream_t hs = NSW == 1 ? s : c->sub_streams[h];
      float* xh = x + r * D;
      f16* n16h = n16 + r * D * X3;
      f16* qkvh = qkv + r * 3 * D;
      f16* o16h = o16 + r * D;
      f16* h16h = h16 + r * 4 * D * X3;
      auto ln16 = [&](const float* g, const float* bb) {
        return X3 == 3 ? layernorm_f16x3(xh, g, bb, n16h, (int)rows_h, D, hs, c->bf16)
                       : layernorm_f16(xh, g, bb, n16h, (int)rows_h, D, D, hs, c->bf16);
      };
      if ((st = ln16(b.ln1_g, b.ln1_b))) return st;
      e = epi();
      e.out16 = qkvh;
      e.ld16 = 3 * D;
      e.scale_cols = 2 * D;
      e.col_scale = qk_scale;
      e.scale_cols2 = D;  // q also carries log2(e): the attention kernel's scores are in exp2 units
      e.col_scale2 = qk_scale * ATT_LOG2E;
      if ((st = run_gemm(b.qkv, n16h, D * X3, D * X3, Bh, L, L, e, hs, "whisper.qkv"))) return st;
      if (b.split_v) {
        e = epi();
        e.out16 = qkvh + 2 * D;
        e.ld16 = 3 * D;
        if ((st = run_gemm(b.v, n16h, D * X3, D * X3, Bh, L, L, e, hs, "whisper.v"))) return st;
      }
      if ((st = attention(qkvh, o16h, Bh, L, D, hs, c->bf16))) return st;
      e = epi();
      e.add_row = xh;
      e.ld_add_row = D;
      e.out32 = xh;
      e.ld32 = D;
      if ((st = run_gemm(b.out, o16h, D, D, Bh, L, L, e, hs, "whisper.out"))) return st;
      if ((st = ln16(b.ln2_g, b.ln2_b))) return st;
      e = epi();
      e.act = ACT_GELU;
      e.out16 = h16h;
      e.ld16 = 4 * D * X3;
      e.split16 = X3 == 3 ? 4 * D : 0;
      if ((st = run_gemm(b.fc1, n16h, D * X3, D * X3, Bh, L, L, e, hs, "whisper.fc1"))) return st;
      e = epi();
      e.add_row = xh;
      e.ld_add_row = D;
      e.out32 = xh;
      e.ld32 = D;
      if ((st = run_gemm(b.fc2, h16h, 4 * D * X3, 4 * D * X3, Bh, L, L, e, hs, "whisper.fc2"))) return st;
    }
  }
  if (NSW > 1) {
    for (int h = 0; h < NSW; ++h) {
      SVC_HIP_CHECK(hipEventRecord(c->ev_join[h], c->sub_streams[h]));
      SVC_HIP_CHECK(hipStreamWaitEvent(s, c->ev_join[h], 0));
    }
  }
  return layernorm_f32(x, c->wlnp_g, c->wlnp_b, feats, (int)rows2, D, D, s);
}

svc_status svc_map_content(svc_ctx* c, const float* feats, int B, int src_rows, int T, int D, void* out, void* stream) {
  SVC_REQUIRE(c && feats && out, "map_content: null");
  SVC_HIP_CHECK(hipSetDevice(c->device));
  return content_map(feats, B, src_rows, D, T, D, (f16*)out, D, (hipStream_t)stream, c->bf16);
}

svc_status svc_map_content_ex(svc_ctx* c, const float* feats, int B, int src_rows, int T, int D, int mode, void* out,
                              int ld_out, void* stream) {
  SVC_REQUIRE(c && feats && out && B > 0 && D > 0 && ld_out >= D, "map_content_ex: bad args");
  SVC_REQUIRE(mode == 0 || mode == 1, "map_content_ex: mode %d", mode);
  SVC_HIP_CHECK(hipSetDevice(c->device));
  if (mode == 0) return content_map(feats, B, src_rows, D, T, D, (f16*)out, ld_out, (hipStream_t)stream, c->bf16);
  return content_map_hubert(feats, B, src_rows, D, T, D, (f16*)out, ld_out, (hipStream_t)stream, c->bf16);
}

// ---------------------------------------------------------------------------- hubert / contentvec (A8)
static int64_t hubert_len(int64_t n, int upto) {
  static const int k[7] = {10, 3, 3, 3, 3, 2, 2}, st[7] = {5, 2, 2, 2, 2, 2, 2};
  for (int i = 0; i < upto; ++i) n = n < k[i] ? 0 : (n - k[i]) / st[i] + 1;
  return n;
}

svc_status svc_hubert_encode(svc_ctx* c, const float* wav16, int B, int64_t n, float* feats, void* stream) {
  CTX_READY(c);
  SVC_REQUIRE(c->has_hubert, "hubert weights not loaded");
  hipStream_t s = (hipStream_t)stream;
  const int64_t F64 = hubert_len(n, 7);
  SVC_REQUIRE(B > 0 && F64 >= 1 && (int64_t)B * hubert_len(n, 1) < (1LL << 31), "hubert: B=%d n=%lld", B,
              (long long)n);
  int64_t t[8];
  for (int i = 0; i <= 7; ++i) t[i] = hubert_len(n, i);  // t[0] = n samples, t[7] = frames
  const int Cc = c->hC, D = c->hD, F = (int)F64;
  const int Fd = c->hblocks[0].fc1.N;
  const bool sp = c->content_mode != 0;  // HuBERT: split-fp16 in both split modes
  const int X3 = sp ? 3 : 1;  // split-fp16 operands are [hi | lo | hi] rows
  const int w5 = sp ? 16 : 8;
  const int64_t R5 = cdiv64(n, 5);
  const size_t rows0 = (size_t)B * t[1], rowsF = (size_t)B * F;
  const int kChunks = 64;
  size_t need = (size_t)B * R5 * w5 * 2 + rows0 * Cc * 4 + rows0 * Cc * 2 * X3 + (size_t)B * kChunks * Cc * 16 +
                (size_t)B * Cc * 8 + (size_t)B * (t[2] + t[3]) * Cc * 2 * X3 + rowsF * Cc * (4 + 2 * X3) +
                rowsF * D * (4 + 2 * X3) + rowsF * 3 * D * 2 + rowsF * D * 2 + rowsF * Fd * 2 * X3 + 32 * 4096;
  int st;
  if ((st = c->ws.reserve(std::max(need, c->ws.cap)))) return st;
  c->ws.reset();
  // ---- feature extractor (wav2vec2 ConvFeatureExtractionModel, mode "default")
  WS_GET(f16, f5, (size_t)B * R5 * w5);
  WS_GET(float, c0, rows0 * Cc);
  WS_GET(f16, g16, rows0 * Cc * X3);
  WS_GET(double, part, (size_t)B * kChunks * Cc * 2);
  WS_GET(float2, gss, (size_t)B * Cc);
  WS_GET(f16, pa, (size_t)B * t[2] * Cc * X3);
  WS_GET(f16, pb, (size_t)B * t[3] * Cc * X3);
  WS_GET(float, c6, rowsF * Cc);
  WS_GET(f16, ln16, rowsF * Cc * X3);
  if ((st = hubert_frames5(wav16, B, n, f5, sp, s, c->bf16))) return st;
  EpiArgs e = epi();
  e.out32 = c0;
  e.ld32 = Cc;
  if ((st = run_gemm(c->hconv[0], f5, w5, w5, B, (int)R5, (int)t[1], e, s, "hubert.conv0"))) return st;
  if ((st = groupnorm_gelu(c0, B, (int)t[1], Cc, c->hgn_g, c->hgn_b, part, kChunks, gss, g16, sp, s, c->bf16)))
    return st;
  const f16* in = g16;
  for (int i = 1; i < 7; ++i) {
    e = epi();
    e.act = ACT_GELU;
    if (i == 6) {
      e.out32 = c6;
      e.ld32 = Cc;
    } else {
      e.out16 = (i & 1) ? pa : pb;
      e.ld16 = Cc * X3;
      e.split16 = sp ? Cc : 0;
    }
    if ((st = run_gemm(c->hconv[i], in, Cc * X3, Cc * X3, B, (int)t[i], (int)t[i + 1], e, s, "hubert.convs"))) return st;
    in = e.out16;
  }
  // ---- HubertModel.forward_features tail: LayerNorm(C) -> post_extract_proj
  if ((st = sp ? layernorm_f16x3(c6, c->hln_g, c->hln_b, ln16, (int)rowsF, Cc, s, c->bf16)
               : layernorm_f16(c6, c->hln_g, c->hln_b, ln16, (int)rowsF, Cc, Cc, s, c->bf16)))
    return st;
  WS_GET(float, x, rowsF * D);
  WS_GET(f16, x16, rowsF * D * X3);
  e = epi();
  e.out32 = x;
  e.ld32 = D;
  if (!sp) {
    e.out16 = x16;
    e.ld16 = D;
  }
  if ((st = run_gemm(c->hproj, ln16, Cc * X3, Cc * X3, B, F, F, e, s, "hubert.proj"))) return st;
  // ---- TransformerEncoder: x += GELU(pos_conv(x)) per group, then LayerNorm (layer_norm_first = False)
  const int Cg = D / c->hPosG;
  if (sp && (st = f32_to_f16x3_grouped(x, x16, (int)rowsF, D, Cg, s, c->bf16))) return st;  // group g: [hi | lo | hi] x Cg
  for (int gi = 0; gi < c->hPosG; ++gi) {
    e = epi();
    e.act = ACT_GELU;
    e.add_row = x + gi * Cg;
    e.ld_add_row = D;
    e.out32 = x + gi * Cg;
    e.ld32 = D;
    if ((st = run_gemm(c->hpos[gi], x16 + (size_t)gi * Cg * X3, D * X3, Cg * X3, B, F, F, e, s, "hubert.pos_conv")))
      return st;
  }
  if ((st = layernorm_dual(x, c->henc_ln_g, c->henc_ln_b, x, x16, (int)rowsF, D, sp, s, c->bf16))) return st;
  WS_GET(f16, qkv, rowsF * 3 * D);
  WS_GET(f16, o16, rowsF * D);
  WS_GET(f16, h16, rowsF * Fd * X3);
  const float qk_scale = powf(64.0f, -0.25f);  // q * dh^-1/2 split over q and k
  for (int i = 0; i < c->hLayers; ++i) {
    HBlock& b = c->hblocks[i];
    e = epi();
    e.out16 = qkv;
    e.ld16 = 3 * D;
    e.scale_cols = 2 * D;
    e.col_scale = qk_scale;
    e.scale_cols2 = D;
    e.col_scale2 = qk_scale * ATT_LOG2E;
    if ((st = run_gemm(b.qkv, x16, D * X3, D * X3, B, F, F, e, s, "hubert.qkv"))) return st;
    if ((st = attention(qkv, o16, B, F, D, s, c->bf16))) return st;
    e = epi();
    e.add_row = x;
    e.ld_add_row = D;
    e.out32 = x;
    e.ld32 = D;
    if ((st = run_gemm(b.out, o16, D, D, B, F, F, e, s, "hubert.out"))) return st;
    if ((st = layernorm_dual(x, b.ln1_g, b.ln1_b, x, x16, (int)rowsF, D, sp, s, c->bf16))) return st;
    e = epi();
    e.act = ACT_GELU;
    e.out16 = h16;
    e.ld16 = Fd * X3;
    e.split16 = sp ? Fd : 0;
    if ((st = run_gemm(b.fc1, x16, D * X3, D * X3, B, F, F, e, s, "hubert.fc1"))) return st;
    e = epi();
    e.add_row = x;
    e.ld_add_row = D;
    e.out32 = x;
    e.ld32 = D;
    if ((st = run_gemm(b.fc2, h16, Fd * X3, Fd * X3, B, F, F, e, s, "hubert.fc2"))) return st;
    if ((st = layernorm_dual(x, b.ln2_g, b.ln2_b, x, x16, (int)rowsF, D, sp, s, c->bf16))) return st;
  }
  e = epi();
  e.out32 = feats;
  e.ld32 = c->hFinal;
  return run_gemm(c->hfinal, x16, D * X3, D * X3, B, F, F, e, s, "hubert.final_proj");
}

int64_t svc_hubert_frames(int64_t n_samples) { return hubert_len(n_samples, 7); }

int svc_hubert_dims(svc_ctx* c, int* final_dim, int* embed_dim) {
  SVC_REQUIRE(c && c->has_hubert, "hubert weights not loaded");
  if (final_dim) *final_dim = c->hFinal;
  if (embed_dim) *embed_dim = c->hD;
  return SVC_OK;
}

// ---------------------------------------------------------------------------- conditioner
static int condition_impl(svc_ctx* c, const void* content16, const double* f0, const float* energy,
                          const int32_t* singer, int B, int T, float* cond, f16* cond16, hipStream_t s) {
  const int rows = B * T;
  WS_GET(int, im, rows);
  WS_GET(int, ie, rows);
  int st;
  if ((st = bucketize(f0, energy, c->mbins, c->ebins, c->n_bins - 1, im, ie, rows, s))) return st;
  EpiArgs e = epi();
  e.kind = EPI_COND;
  e.idx_m = im;
  e.idx_l = ie;
  e.singer = singer;
  e.emb_m = c->emb_m;
  e.emb_l = c->emb_l;
  e.emb_s = c->emb_s;
  e.ld_emb = c->C;
  e.out32 = cond;
  e.ld32 = c->C;
  e.out16 = cond16;
  e.ld16 = c->C;
  return run_gemm(c->content_lin, (const f16*)content16, c->content_dim, c->content_dim, B, T, T, e, s, "cond.content");
}

svc_status svc_condition_indices(svc_ctx* c, const double* f0, const float* energy, int n, int32_t* melody_idx,
                                 int32_t* loudness_idx, void* stream) {
  CTX_READY(c);
  SVC_REQUIRE(c->has_mapper, "mapper weights not loaded");
  SVC_REQUIRE(n >= 0 && (n == 0 || (f0 && energy && melody_idx && loudness_idx)), "condition_indices: n %d", n);
  if (n == 0) return SVC_OK;
  return bucketize(f0, energy, c->mbins, c->ebins, c->n_bins - 1, melody_idx, loudness_idx, n, (hipStream_t)stream);
}

svc_status svc_condition(svc_ctx* c, const void* content16, const double* f0, const float* energy,
                         const int32_t* singer, int B, int T, float* cond, void* stream) {
  CTX_READY(c);
  SVC_REQUIRE(c->has_mapper, "mapper weights not loaded");
  int st;
  if ((st = c->ws.reserve(std::max((size_t)B * T * 8 + 4096, c->ws.cap)))) return st;
  c->ws.reset();
  return condition_impl(c, content16, f0, energy, singer, B, T, cond, nullptr, (hipStream_t)stream);
}

// ---------------------------------------------------------------------------- DiffSVC denoiser
struct DenoiseBufs {
  f16* cp16;     // [rows][NL*2C] conditioner projections of every layer (hoisted out of the sampler loop)
  f16* y16;      // [rows][C] next layer input x + diffusion_projection (the high half of the split residual stream)
  f16* g16;      // [rows][NL*C] gate outputs of every layer (A operand of the skip GEMM)
  f16* s16;      // [rows][3C] sum(skip) / sqrt(NL) ([hi | lo | hi] split-fp16 with head_split, else [rows][C])
  f16* u16;      // [rows][3C] relu(skip_projection), same layout
  f16* lo16;     // [rows][C] low half of the split residual stream: x + dproj = y16 + lo16
  size_t cp_ls;  // elements between layers of cp16, which is LAYER-major [NL][rows_total][2C]: each layer's gate
                 // epilogue reads one contiguous block (row-major over all layers put 30 KB between its rows)
  size_t g_ls;   // elements between layers of g16, also layer-major [NL][rows_total][C]: the gate GEMM writes and the
                 // residual GEMM reads one contiguous block; the skip GEMM reads the NL blocks as NL "taps" whose row
                 // shift is the layer stride (tap_mul = rows_total)
};


// tv (device, optional): ragged batches, utterance b has tv[b] valid frames; only the dilated convs look across frames
// plms (optional): the PLMS update that consumes this eps, launched right after the head
static int denoise(svc_ctx* c, const DenoiseBufs& bb, const f16* x16, int B, int T, int t, float* eps, hipStream_t s,
                   const int* tv, const PlmsArgs* plms = nullptr) {
  const int C = c->C, NL = c->n_layers, rows = B * T;
  const int ldx16 = (int)round_up(c->n_mel, 8);
  const float* dp = c->dproj + (size_t)t * NL * C;
  int st;
  // Residual stream x in split-fp16 storage (x + dproj_l = y16 + lo16, ~22 significand bits in 4 bytes): the layer's
  // GEMM operand y16 is its high half, so each residual update moves 10 instead of 12 bytes per element (an f32
  // residual stream measured 1.1 % slower end to end at the same mel-L1, round 1; removed in round 3).
  EpiArgs e = epi();
  e.act = ACT_RELU;
  e.lo16 = bb.lo16;
  e.out16 = bb.y16;
  e.ld16 = C;
  e.add16 = dp;  // layer 0 diffusion projection
  if (tuning().res_proj && c->melpre.Wfrag && ldx16 <= 128) {
    // weight-stationary store stream (res_proj.hip mel_proj), bit-identical to the tiled GEMM
    prof_site("diffsvc.melpre");
    if ((st = mel_proj(x16, ldx16, c->melpre.Wfrag, c->melpre.bias, dp, bb.y16, bb.lo16, rows, c->melpre.bf16, s)))
      return st;
  } else if ((st = run_gemm(c->melpre, x16, ldx16, c->n_mel, B, T, T, e, s, "diffsvc.melpre"))) {
    return st;
  }
  // the split residual stream's high half, updated in place (y16) by gate + res_proj
  f16* hi = bb.y16;
  for (int i = 0; i < NL; ++i) {
    EpiArgs g = epi();
    g.kind = EPI_GATE;
    g.cp = bb.cp16 + (size_t)i * bb.cp_ls;
    g.ld_cp = 2 * C;
    g.y16 = bb.g16 + (size_t)i * bb.g_ls;
    g.ldy16 = C;
    if ((st = run_gemm(c->dil[i], hi, C, C, B, T, T, g, s, "diffsvc.dilated", tv, 1))) return st;
    if (i + 1 == NL) break;  // the last layer's residual output is unused (only skips feed the head)
    // x = (x + residual) / sqrt(2); next input x + diffusion_projection_{i+1}(step):
    // x_i = (y16 + lo16) - dproj_i, and x_{i+1} + dproj_{i+1} goes back split into y16 / lo16
    if (tuning().res_proj && C == 384 && c->outres[i].Wfrag && c->outres[i].N == C && c->outres[i].K == C) {
      // weight-stationary row stream (res_proj.hip), bit-identical to the tiled GEMM below
      prof_site("diffsvc.outproj");
      if ((st = res_proj(bb.g16 + (size_t)i * bb.g_ls, c->outres[i].Wfrag, c->outres[i].bias,
                         dp + (size_t)i * C, dp + (size_t)(i + 1) * C, 1.41421356237309515f, hi, bb.lo16, rows,
                         c->outres[i].bf16,
                         tuning().res_proj > 1 ? tuning().res_proj : (tuning().sampler_streams == 1 ? -2 : 0), s)))
        return st;
      continue;
    }
    EpiArgs r = epi();
    r.ld_acc = C;
    r.acc_div = 1.41421356237309515f;
    r.acc16_hi = hi;
    r.acc16_lo = bb.lo16;
    r.acc_sub = dp + (size_t)i * C;
    r.lo16 = bb.lo16;
    r.out16 = hi;
    r.ld16 = C;
    r.add16 = dp + (size_t)(i + 1) * C;
    if ((st = run_gemm(c->outres[i], bb.g16 + (size_t)i * bb.g_ls, C, C, B, T, T, r, s, "diffsvc.outproj"))) return st;
  }
  // skip = sum_i skip_i (modules/diffsvc.py:311); x = skip / sqrt(len(layers)) (:315)
  const int H3 = c->head_split ? 3 : 1;  // split-fp16 head operands are [hi | lo | hi] rows
  e = epi();
  e.scale_cols = C;
  e.col_scale = 1.0f / sqrtf((float)NL);
  e.out16 = bb.s16;
  e.ld16 = C * H3;
  e.split16 = H3 == 3 ? C : 0;
  {
    PackedGemm sk = c->skip_all;  // K index l * C + k = "tap" l * Cp + k with Cp = C: same packed weights
    sk.Cp = C;
    sk.taps = NL;
    sk.tap_mul = (int)(bb.g_ls / C);
    sk.tap_add = 0;
    sk.istride = 1;
    const int rows_sub = B * T;
    if ((st = run_gemm(sk, bb.g16, C, C, 1, NL * sk.tap_mul, rows_sub, e, s, "diffsvc.skipsum"))) return st;
  }
  // relu(skip_projection) and output_projection in one launch: u never reaches HBM (diff_head.hip)
  if (tuning().diff_head && H3 == 3 && C == 384 && c->skipproj.N == C && c->skipproj.Npad >= C &&
      c->skipproj.K == 3 * C && c->skipproj.Kpad == 3 * C && c->outproj.K == 3 * C && c->outproj.Kpad == 3 * C &&
      c->outproj.Npad >= 128 && c->outproj.N <= 128 && c->n_mel % 4 == 0) {
    if ((st = diff_head(bb.s16, c->skipproj.W, c->skipproj.bias, C, 3 * C, c->outproj.W, c->outproj.bias,
                        c->outproj.N, 3 * C, c->outproj.Npad, eps, c->n_mel, (int)rows, zero_page(), s,
                        c->skipproj.bf16)))
      return st;
    return plms ? plms_update(*plms, rows, c->n_mel, s) : SVC_OK;
  }
  e = epi();
  e.act = ACT_RELU;
  e.out16 = bb.u16;
  e.ld16 = C * H3;
  e.split16 = H3 == 3 ? C : 0;
  if ((st = run_gemm(c->skipproj, bb.s16, C * H3, C * H3, B, T, T, e, s, "diffsvc.skipproj"))) return st;
  e = epi();
  e.out32 = eps;
  e.ld32 = c->n_mel;
  if ((st = run_gemm(c->outproj, bb.u16, C * H3, C * H3, B, T, T, e, s, "diffsvc.eps_out"))) return st;
  return plms ? plms_update(*plms, rows, c->n_mel, s) : SVC_OK;
}

static int alloc_denoise(svc_ctx* c, int B, int T, DenoiseBufs& bb) {
  const size_t rows = (size_t)B * T, C = c->C;
  WS_GET(f16, cp16, rows * c->n_layers * 2 * C);
  WS_GET(f16, y16, rows * C);
  WS_GET(f16, g16, rows * c->n_layers * C);
  WS_GET(f16, s16, rows * C * 3);  // [hi | lo | hi] when head_split
  WS_GET(f16, u16, rows * C * 3);
  WS_GET(f16, lo16, rows * C);
  bb = DenoiseBufs{cp16, y16, g16, s16, u16, lo16, rows * 2 * C, rows * C};
  return SVC_OK;
}

static size_t denoise_bytes(svc_ctx* c, int B, int T) {
  const size_t rows = (size_t)B * T, C = c->C;
  return rows * c->n_layers * 2 * C * 2 + rows * c->n_layers * C * 2 + rows * C * 2 * 9 + 26 * 4096;
}

static int project_cond(svc_ctx* c, const float* cond, int B, int T, const DenoiseBufs& bb, hipStream_t s) {
  const int rows = B * T, C = c->C;
  WS_GET(f16, cond16, (size_t)rows * 3 * C);
  int st;
  if ((st = f32_to_f16x3(cond, C, cond16, rows, C, s, c->bf16))) return st;  // [hi | lo | hi] split-fp16 operand
  // the projections of all layers as ONE GEMM over the packed weights (N = NL x 2C), each layer's 2C columns written
  // to its layer-major cp block (EpiArgs col_block): 20 launches of 470 tiles (1.8 rounds of workgroups each) became
  // one launch of 9 400 (round 5)
  EpiArgs e = epi();
  e.out16 = bb.cp16;
  e.ld16 = 2 * C;
  e.col_block = 2 * C;
  e.col_block_stride = (int64_t)bb.cp_ls;
  if ((st = run_gemm(c->cp_all, cond16, 3 * C, 3 * C, B, T, T, e, s, "diffsvc.condproj"))) return st;
  return SVC_OK;
}

// ragged batches: validate the per-utterance frame counts (host) and stage them to the device through `ring`
static int stage_frames(StageRing& ring, const int32_t* frames, int B, int T, hipStream_t s, const int** dev_out) {
  *dev_out = nullptr;
  if (!frames) return SVC_OK;
  for (int b = 0; b < B; ++b)
    SVC_REQUIRE(frames[b] >= 1 && frames[b] <= T, "utterance %d: %d frames (batch length %d)", b, frames[b], T);
  void* dev = nullptr;
  int st = ring.put(frames, (size_t)B * sizeof(int32_t), s, &dev);
  *dev_out = reinterpret_cast<const int*>(dev);
  return st;
}

svc_status svc_diffsvc_eps(svc_ctx* c, const float* cond, const float* x, int B, int T, const int32_t* frames, int t,
                           float* eps, void* stream) {
  CTX_READY(c);
  SVC_REQUIRE(c->has_mapper, "mapper weights not loaded");
  SVC_REQUIRE(t >= 0 && t < c->steps, "eps: t=%d", t);
  hipStream_t s = (hipStream_t)stream;
  const int* tv;
  RingRetire retire_(c->lens_main, s);
  if (int st0 = stage_frames(c->lens_main, frames, B, T, s, &tv)) return st0;
  const int rows = B * T, ld16 = (int)round_up(c->n_mel, 8);
  int st;
  if ((st = c->ws.reserve(std::max(denoise_bytes(c, B, T) + (size_t)rows * (ld16 * 2 + c->C * 6) + 8192, c->ws.cap))))
    return st;
  c->ws.reset();
  DenoiseBufs bb;
  if ((st = alloc_denoise(c, B, T, bb))) return st;
  if ((st = project_cond(c, cond, B, T, bb, s))) return st;
  WS_GET(f16, x16, (size_t)rows * ld16);
  if ((st = f32_to_f16(x, c->n_mel, x16, ld16, rows, c->n_mel, ld16, s, c->bf16))) return st;
  if ((st = denoise(c, bb, x16, B, T, t, eps, s, tv))) return st;
  return tv ? zero_tail_rows(eps, B, T, c->n_mel, tv, s) : SVC_OK;
}

static int sample_impl(svc_ctx* c, const float* cond, int B, int T, const int* tv, int mode, int interval,
                       const float* x_T, const float* noise, uint64_t seed, const int32_t* utt_ids, float* x0,
                       hipStream_t stream);

svc_status svc_diffsvc_sample(svc_ctx* c, const float* cond, int B, int T, const int32_t* frames, int mode,
                              int interval, const float* x_T, const float* noise, uint64_t seed,
                              const int32_t* utt_ids, float* x0, void* stream) {
  CTX_READY(c);
  hipStream_t s = (hipStream_t)stream;
  const int* tv;
  RingRetire retire_(c->lens_main, s);
  int st = stage_frames(c->lens_main, frames, B, T, s, &tv);
  if (st || (st = sample_impl(c, cond, B, T, tv, mode, interval, x_T, noise, seed, utt_ids, x0, s))) return st;
  // frames past an utterance's end hold no sample: zero them
  return tv ? zero_tail_rows(x0, B, T, c->n_mel, tv, s) : SVC_OK;
}

static int sample_impl(svc_ctx* c, const float* cond, int B, int T, const int* tv, int mode, int interval,
                       const float* x_T, const float* noise, uint64_t seed, const int32_t* utt_ids, float* x0,
                       hipStream_t stream) {
  SVC_REQUIRE(c->has_mapper, "mapper weights not loaded");
  SVC_REQUIRE(mode == SVC_MODE_DDPM || (mode == SVC_MODE_PLMS && interval >= 1), "sample: mode %d interval %d", mode,
              interval);
  SVC_REQUIRE(x_T || utt_ids, "sample: need x_T or utt_ids for device noise");
  // DDPM draws step noise on the device unless `noise` is given; that noise is keyed by utterance id
  SVC_REQUIRE(mode != SVC_MODE_DDPM || noise || utt_ids, "sample: DDPM without `noise` needs utt_ids");
  hipStream_t s = (hipStream_t)stream;
  const int rows = B * T, nm = c->n_mel, ld16 = (int)round_up(nm, 8);
  int st;
  const size_t extra = (size_t)rows * (ld16 * 2 * 2 + nm * 4 * 8 + c->C * 6) + 32 * 4096;
  if ((st = c->ws.reserve(std::max(denoise_bytes(c, B, T) + extra, c->ws.cap)))) return st;
  c->ws.reset();
  DenoiseBufs bb;
  if ((st = alloc_denoise(c, B, T, bb))) return st;
  if ((st = project_cond(c, cond, B, T, bb, s))) return st;
  float* x = x0;  // the sampler state lives in the output buffer
  WS_GET(f16, x16, (size_t)rows * ld16);
  SVC_HIP_CHECK(hipMemsetAsync(x16, 0, (size_t)rows * ld16 * sizeof(f16), s));  // zero pad channels
  if (x_T) {
    SVC_HIP_CHECK(hipMemcpyAsync(x, x_T, (size_t)rows * nm * 4, hipMemcpyDeviceToDevice, s));
    if ((st = f32_to_f16(x, nm, x16, ld16, rows, nm, ld16, s, c->bf16))) return st;
  } else {
    if ((st = init_noise(x, x16, ld16, B, T, nm, seed, utt_ids, 1.0f / 1.2f, s, c->bf16))) return st;
  }
  WS_GET(float, eps, (size_t)rows * nm);
  float* hist[5];
  for (int k = 0; k < 5; ++k) {
    WS_GET(float, hb, (size_t)rows * nm);
    hist[k] = hb;
  }
  WS_GET(float, xp, (size_t)rows * nm);
  WS_GET(f16, xp16, (size_t)rows * ld16);
  SVC_HIP_CHECK(hipMemsetAsync(xp16, 0, (size_t)rows * ld16 * sizeof(f16), s));

  // Utterance-aligned sub-batches on their own streams, issued kernel by kernel in alternation: their
  // launches overlap on the GPU, so one sub-batch's epilogue / prologue phases (HBM-bound, ~40 % of a
  // denoiser GEMM launch at this size) run beside the other's MFMA phases. Utterances are independent,
  // so results are identical to a single stream. Default 2 (round-2 final code, alternating A/B on two boxes:
  // +0.9 % over 3, 4: -15 %; profiles/r02zf_streams_ab.txt); sampler_streams = 1 disables the split.
  const int S = std::max(1, std::min(std::min(tuning().sampler_streams, B), (int)kMaxSubStreams));
  struct Sub {
    int B, b0;
    size_t r0;
    hipStream_t s;
  } sub[kMaxSubStreams];
  if ((st = c->ensure_sub_streams(S))) return st;
  for (int h = 0; h < S; ++h) {
    sub[h].b0 = h * B / S;
    sub[h].B = (h + 1) * B / S - sub[h].b0;
    sub[h].r0 = (size_t)sub[h].b0 * T;
    sub[h].s = S == 1 ? s : c->sub_streams[h];
  }
  auto sub_bufs = [&](const Sub& u) {
    const size_t r = u.r0;
    const int C = c->C;
    return DenoiseBufs{bb.cp16 + r * 2 * C, bb.y16 + r * C, bb.g16 + r * C, bb.s16 + r * 3 * C, bb.u16 + r * 3 * C,
                       bb.lo16 + r * C, bb.cp_ls, bb.g_ls};
  };
  SVC_HIP_CHECK(hipEventRecord(c->ev_fork, s));
  for (int h = 0; h < S && S > 1; ++h) SVC_HIP_CHECK(hipStreamWaitEvent(sub[h].s, c->ev_fork, 0));
  auto join = [&]() -> int {
    if (S == 1) return SVC_OK;
    for (int h = 0; h < S; ++h) {
      SVC_HIP_CHECK(hipEventRecord(c->ev_join[h], sub[h].s));
      SVC_HIP_CHECK(hipStreamWaitEvent(s, c->ev_join[h], 0));
    }
    return SVC_OK;
  };

  if (mode == SVC_MODE_DDPM) {
    for (int i = c->steps - 1; i >= 0; --i) {
      for (int h = 0; h < S; ++h) {
        const Sub& u = sub[h];
        const size_t r = u.r0;
        if ((st = denoise(c, sub_bufs(u), x16 + r * ld16, u.B, T, i, eps + r * nm, u.s, tv ? tv + u.b0 : nullptr)))
          return st;
        DdpmArgs a{};
        a.sra = c->sra[i];
        a.srm1 = c->srm1[i];
        a.c1 = c->pc1[i];
        a.c2 = c->pc2[i];
        a.sigma = i > 0 ? expf(0.5f * c->plogvar[i]) : 0.0f;
        a.z = noise ? noise + (size_t)(c->steps - 1 - i) * rows * nm + r * nm : nullptr;
        a.seed = seed;
        a.utt_ids = utt_ids ? utt_ids + u.b0 : nullptr;
        a.step = i;
        a.bf16 = c->bf16;
        if ((st = ddpm_update(x + r * nm, eps + r * nm, x16 + r * ld16, ld16, u.B, T, nm, a, u.s))) return st;
      }
    }
    return join();
  }
  // PLMS: history ring of 4 epsilons + the first step's predictor buffers (the ring position is shared)
  int nh = 0, head = 0;  // hist slots: newest at hist[(head - 1) mod 5]
  const std::vector<float>& ac = c->alphas_cumprod_f32;
  for (int i = ((c->steps - 1) / interval) * interval; i >= 0; i -= interval) {
    const int tp = i - interval > 0 ? i - interval : 0;
    // get_x_pred coefficients in f32 exactly as the reference's tensor ops (:96-113)
    const float a_t = ac[i], a_prev = ac[tp];
    const float a_t_sq = sqrtf(a_t), a_prev_sq = sqrtf(a_prev);
    const float A = 1.0f / (a_t_sq * (a_t_sq + a_prev_sq));
    const float Bc = 1.0f / (a_t_sq * (sqrtf((1.0f - a_prev) * a_t) + sqrtf((1.0f - a_t) * a_prev)));
    const float d = a_prev - a_t;
    for (int h = 0; h < S; ++h) {
      const Sub& u = sub[h];
      const size_t r = u.r0;
      const int urows = u.B * T;
      const DenoiseBufs ub = sub_bufs(u);
      float* ecur = hist[head] + r * nm;
      PlmsArgs p{};
      p.bf16 = c->bf16;
      p.d = d;
      p.A = A;
      p.Bc = Bc;
      p.xin = x + r * nm;
      p.xout = x + r * nm;
      p.x16 = x16 + r * ld16;
      p.ld16 = ld16;
      auto H = [&](int back) { return hist[((head - back) % 5 + 5) % 5] + r * nm; };
      // each update runs in (or right after) the denoise whose eps it consumes (denoise's plms argument)
      if (nh == 0) {
        PlmsArgs q = p;
        q.e[0] = ecur;
        q.c[0] = 1.0f;
        q.ne = 1;
        q.div = 1.0f;
        q.xout = xp + r * nm;
        q.x16 = xp16 + r * ld16;
        if ((st = denoise(c, ub, x16 + r * ld16, u.B, T, i, ecur, u.s, tv ? tv + u.b0 : nullptr, &q)))
          return st;
        float* eprev = hist[(head + 1) % 5] + r * nm;
        p.e[0] = ecur;
        p.e[1] = eprev;
        p.c[0] = 1.0f;
        p.c[1] = 1.0f;
        p.ne = 2;
        p.div = 2.0f;
        if ((st = denoise(c, ub, xp16 + r * ld16, u.B, T, tp, eprev, u.s, tv ? tv + u.b0 : nullptr, &p)))
          return st;
        continue;
      } else if (nh == 1) {
        p.e[0] = ecur;
        p.e[1] = H(1);
        p.c[0] = 3.0f;
        p.c[1] = -1.0f;
        p.ne = 2;
        p.div = 2.0f;
      } else if (nh == 2) {
        p.e[0] = ecur;
        p.e[1] = H(1);
        p.e[2] = H(2);
        p.c[0] = 23.0f;
        p.c[1] = -16.0f;
        p.c[2] = 5.0f;
        p.ne = 3;
        p.div = 12.0f;
      } else {
        p.e[0] = ecur;
        p.e[1] = H(1);
        p.e[2] = H(2);
        p.e[3] = H(3);
        p.c[0] = 55.0f;
        p.c[1] = -59.0f;
        p.c[2] = 37.0f;
        p.c[3] = -9.0f;
        p.ne = 4;
        p.div = 24.0f;
      }
      if ((st = denoise(c, ub, x16 + r * ld16, u.B, T, i, ecur, u.s, tv ? tv + u.b0 : nullptr, &p)))
        return st;
    }
    head = (head + 1) % 5;
    nh = nh < 4 ? nh + 1 : 4;
  }
  return join();
}

// ---------------------------------------------------------------------------- BigVGAN
svc_status svc_bigvgan(svc_ctx* c, const float* x0, int B, int T, const int32_t* frames, float* wav, float* mel_out,
                       void* stream) {
  CTX_READY(c);
  SVC_REQUIRE(c->has_vocoder && c->has_mapper, "vocoder (and mapper stats) not loaded");
  hipStream_t s = (hipStream_t)stream;
  // ragged batches: utterance b has frames[b] mel frames; at a point where the signal is `mul` times the mel rate
  // its valid length is tv[b] * mul, and every conv / activation / the fade-out ends there
  const int* tv;
  RingRetire retire_(c->lens_main, s);
  if (int st0 = stage_frames(c->lens_main, frames, B, T, s, &tv)) return st0;
  for (int b = 0; frames && b < B; ++b)
    SVC_REQUIRE(frames[b] * c->hop_out >= c->nfade, "bigvgan: utterance %d (%d frames) shorter than the fade-out", b,
                frames[b]);
  const int nm = c->v_in, ldm = (int)round_up(nm, 8);
  int maxLC = 0, Lr = T;  // max over stages of L_i*C_i / T  (6144 for the reference config)
  for (auto& S : c->vstages) {
    Lr *= S.rate;
    maxLC = std::max(maxLC, (Lr / T) * S.cout);
  }
  // the activation kernels address one utterance's f32 stage buffer through 32-bit buffer offsets: T * maxLC * 4 bytes
  // must stay below 2 GiB (87 381 frames = 15.5 min of 24 kHz audio for the reference config); longer utterances are
  // rejected here rather than silently wrapped
  SVC_REQUIRE((int64_t)T * maxLC * 4 < ((int64_t)1 << 31),
              "bigvgan: T=%d frames per utterance exceeds the vocoder's limit of %lld frames (2 GiB stage span)", T,
              (long long)((((int64_t)1 << 31) - 1) / ((int64_t)maxLC * 4)));
  const size_t big = (size_t)B * T * maxLC;
  const size_t need = (size_t)B * T * ldm * 2 + (size_t)B * T * c->v_c0 * 2 + big * (4 * 4 + 2 * 2) + 32 * 4096;
  int st;
  if ((st = c->ws.reserve(std::max(need, c->ws.cap)))) return st;
  c->ws.reset();
  SVC_REQUIRE(T * c->hop_out >= c->nfade, "bigvgan: T=%d shorter than the fade-out", T);
  WS_GET(f16, mel16, (size_t)B * T * ldm);
  WS_GET(f16, pre16, (size_t)B * T * c->v_c0);
  WS_GET(float, X, big);
  WS_GET(float, Xj, big);
  WS_GET(float, tmp, big);
  WS_GET(float, XS, big);
  WS_GET(f16, a16, big);
  WS_GET(f16, next16, big);
  // amp_maxc: widest channel count that takes the fused kernel (0: activation1d + GEMM everywhere). C = 48 unfused is
  // 9 % slower (its N = 48 GEMMs are too narrow for the MFMA tiles); C = 96 fused is 1.0 ms per step faster than
  // activation1d + amp_conv's plain conv since both run on 256-row tiles of 2 x 2 waves (round 6; on the round-5 128-row
  // tiles, where every wave read all of W per k-loop, fused C = 96 had been 1 % slower end to end)
  const int amp_maxc = tuning().amp_maxc;
  const int ns = (int)c->vstages.size();

  // Utterance-aligned sub-batches on their own streams (as in svc_diffsvc_sample): every buffer is
  // time-major per utterance, so a sub-batch is a row offset into each; launches alternate between streams.
  // Default 1: its launches are long (0.3-2 ms) and measured no faster split (vocoder_streams = 2 / 3).
  const int NS = std::max(1, std::min(std::min(tuning().vocoder_streams, B), (int)kMaxSubStreams));
  if ((st = c->ensure_sub_streams(NS))) return st;
  SVC_HIP_CHECK(hipEventRecord(c->ev_fork, s));
  int b0[kMaxSubStreams + 1];
  hipStream_t ss[kMaxSubStreams];
  for (int h = 0; h <= NS; ++h) b0[h] = h * B / NS;
  for (int h = 0; h < NS; ++h) {
    ss[h] = NS == 1 ? s : c->sub_streams[h];
    if (NS > 1) SVC_HIP_CHECK(hipStreamWaitEvent(ss[h], c->ev_fork, 0));
  }
  for (int h = 0; h < NS; ++h) {  // de-normalise + conv_pre
    const int Bh = b0[h + 1] - b0[h];
    const size_t r = (size_t)b0[h] * T;
    if ((st = denorm_mel(x0 + r * nm, mel16 + r * ldm, mel_out ? mel_out + r * nm : nullptr, ldm, Bh * T, nm,
                         c->mel_min, c->mel_max, ss[h])))
      return st;
    EpiArgs e = epi();
    e.out16 = pre16 + r * c->v_c0;
    e.ld16 = c->v_c0;
    if ((st = run_gemm(c->vpre, mel16 + r * ldm, ldm, nm, Bh, T, T, e, ss[h], "bigvgan.conv_pre",
                       tv ? tv + b0[h] : nullptr, 1)))
      return st;
  }
  int L = T;
  int mul = 1;  // samples of the current stage per mel frame
  for (int i = 0; i < ns; ++i) {
    VStage& S = c->vstages[i];
    const int Lin = L;
    const int mul_in = mul;
    L = Lin * S.rate;
    mul = mul_in * S.rate;
    const int ch = S.cout;
    for (int h = 0; h < NS; ++h) {
      const int Bh = b0[h + 1] - b0[h];
      const hipStream_t sh = ss[h];
      const int* tvh = tv ? tv + b0[h] : nullptr;
      // each sub-batch owns the fixed region [b0 * T * maxLC, b1 * T * maxLC) of every stage buffer for all
      // stages (offsets that moved with L * C would let a lagging stream's reads overlap another's writes)
      const size_t ro = (size_t)b0[h] * T * maxLC;
      float *Xh = X + ro, *Xjh = Xj + ro, *tmph = tmp + ro, *XSh = XS + ro;
      f16* a16h = a16 + ro;
      const f16* in16 = i == 0 ? pre16 + (size_t)b0[h] * T * c->v_c0 : next16 + ro;
      f16* next16h = next16 + ro;
      // ConvTranspose1d as `rate` phase GEMMs writing rows t*rate + r, or (rate 2, tune.amp_ups) as one conv
      if (S.up_comb && tuning().amp_ups) {
        AmpConvArgs q{nullptr, Bh, Lin, 3, -1, nullptr, nullptr, nullptr, S.upc.W, S.upc.Kpad, S.upc.bias};
        q.x16 = in16;
        q.noact = true;
        q.tv = tvh;
        q.tv_mul = mul_in;
        EpiArgs u = epi();
        u.out32 = Xh;
        u.ld32 = S.cin;
        prof_site("bigvgan.ups");
        if ((st = amp_conv(q, S.cin, u, sh))) return st;
      } else
      for (int r = 0; r < S.rate; ++r) {
        EpiArgs u = epi();
        u.T_ostore = L;
        u.ostride = S.rate;
        u.ophase = r;
        u.out32 = Xh;
        u.ld32 = ch;
        if ((st = run_gemm(S.phases[r], in16, S.cin, S.cin, Bh, Lin, Lin, u, sh, "bigvgan.ups", tvh, mul_in))) return st;
      }
      const int nk = (int)S.c1.size();
      for (int j = 0; j < nk; ++j) {
        const int nd = (int)S.c1[j].size();
        for (int l = 0; l < nd; ++l) {
          // AMPBlock2 reads its activation halo from the x it updates, so its x ping-pongs between Xj and tmp
          // (AMPBlock1 updates x in place: its second activation reads tmp)
          const float* src = (l == 0) ? Xh : ((c->v_rb2 && l % 2 == 0) ? tmph : Xjh);
          float* xnext = (c->v_rb2 && l % 2 == 1) ? tmph : Xjh;
          const ActP& a1 = S.acts[j][2 * l];
          const ActP& a2 = S.acts[j][2 * l + 1];
          // AMPBlock1: tmp = c1(a1(x)), x' = x + c2(a2(tmp)); AMPBlock2: x' = x + c(a(x)) with c = c2[l] (dilation d)
          const bool rb2 = c->v_rb2;
          const int d2 = rb2 ? S.rd[j][l] : 1;
          // AMPBlock1's intermediate c1(a1(x)) is stored f16 (tmp16, in tmp's memory): it is read once, by a2, whose
          // output is rounded to the f16 MFMA operand anyway; 4 B less per element read and written (round 3)
          f16* tmp16 = reinterpret_cast<f16*>(tmph);
          const float* act_in = rb2 ? src : nullptr;  // input of the activation before the second (or only) conv
          const f16* act_in16 = rb2 ? nullptr : tmp16;
          // small channel counts: SnakeBeta fused into the conv (amp_conv.hip); otherwise activation1d + GEMM
          const bool fuse = ch <= amp_maxc && amp_conv_supported(ch, S.rk[j], S.rd[j][l]);
          if (!rb2) {
            EpiArgs e1 = epi();
            e1.out16 = tmp16;
            e1.ld16 = ch;
            if (fuse) {
              const PackedGemm& g1 = S.c1[j][l];
              AmpConvArgs p1{src, Bh, L, S.rk[j], S.rd[j][l], a1.alpha, a1.beta, a1.filt, g1.W, g1.Kpad, g1.bias};
              p1.tv = tvh;
              p1.tv_mul = mul;
              prof_site("bigvgan.amp_c1");
              if ((st = amp_conv(p1, ch, e1, sh))) return st;
            } else {
              if ((st = activation1d(src, a16h, Bh, L, ch, ch, a1.alpha, a1.beta, a1.filt, sh, tvh, mul))) return st;
              if ((st = run_gemm(S.c1[j][l], a16h, ch, ch, Bh, L, L, e1, sh, "bigvgan.amp_c1", tvh, mul))) return st;
            }
          }
          if (!fuse &&
              (st = activation1d(act_in, a16h, Bh, L, ch, ch, a2.alpha, a2.beta, a2.filt, sh, tvh, mul, act_in16)))
            return st;
          EpiArgs e2 = epi();
          e2.add_row = src;
          e2.ld_add_row = ch;
          if (l + 1 < nd) {
            e2.out32 = xnext;
            e2.ld32 = ch;
          } else if (j == 0) {
            e2.out32 = XSh;
            e2.ld32 = ch;
          } else {
            e2.acc32 = XSh;
            e2.ld_acc = ch;
            if (j + 1 == nk) {
              e2.acc_div = (float)nk;
              if (i + 1 < ns) {
                e2.out16 = next16h;
                e2.ld16 = ch;
              } else {
                e2.out32 = XSh;
                e2.ld32 = ch;
              }
            } else {
              e2.out32 = XSh;
              e2.ld32 = ch;
            }
          }
          if (fuse) {
            const PackedGemm& g2 = S.c2[j][l];
            AmpConvArgs p2{act_in, Bh, L, S.rk[j], d2, a2.alpha, a2.beta, a2.filt, g2.W, g2.Kpad, g2.bias};
            p2.tv = tvh;
            p2.tv_mul = mul;
            p2.x16 = act_in16;
            prof_site("bigvgan.amp_c2");
            if ((st = amp_conv(p2, ch, e2, sh))) return st;
          } else if ((st = run_gemm(S.c2[j][l], a16h, ch, ch, Bh, L, L, e2, sh, "bigvgan.amp_c2", tvh, mul))) {
            return st;
          }
        }
      }
      // the stage output next16 feeds the next ConvTranspose; it is rewritten only after that ran (same stream)
    }
  }
  const int chl = c->vstages.back().cout;
  for (int h = 0; h < NS; ++h) {
    const int Bh = b0[h + 1] - b0[h];
    const size_t ro = (size_t)b0[h] * T * maxLC;
    const int* tvh = tv ? tv + b0[h] : nullptr;
    if ((st = activation1d(XS + ro, a16 + ro, Bh, L, chl, chl, c->vact_post.alpha, c->vact_post.beta,
                           c->vact_post.filt, ss[h], tvh, mul)))
      return st;
    if ((st = conv_post(a16 + ro, chl, Bh, L, chl, c->vpost_w, c->vpost_b, c->fade, c->nfade,
                        wav + (size_t)b0[h] * L, ss[h], tvh, mul)))
      return st;
    if (NS > 1) {
      SVC_HIP_CHECK(hipEventRecord(c->ev_join[h], ss[h]));
      SVC_HIP_CHECK(hipStreamWaitEvent(s, c->ev_join[h], 0));
    }
  }
  return (tv && mel_out) ? zero_tail_rows(mel_out, B, T, nm, tv, s) : SVC_OK;
}

// ---------------------------------------------------------------------------- op-level (tests)
static int op_ws(svc_ctx** tmp) {
  static svc_ctx* g = nullptr;
  if (!g) {
    g = new svc_ctx();
    g->tune.from_env();
    g->tune0 = g->tune;
    int dev = 0;
    (void)hipGetDevice(&dev);
    g->device = dev;
    g->finalized = true;
  }
  *tmp = g;
  return SVC_OK;
}

static int pack_from_device(svc_ctx* c, PackedGemm& g, const float* w_dev, size_t wn, const float* b_dev, int bn,
                            std::vector<float>& wh, std::vector<float>& bh) {
  wh.resize(wn);
  bh.assign(bn, 0.0f);
  SVC_HIP_CHECK(hipDeviceSynchronize());
  SVC_HIP_CHECK(hipMemcpy(wh.data(), w_dev, wn * 4, hipMemcpyDeviceToHost));
  if (b_dev) SVC_HIP_CHECK(hipMemcpy(bh.data(), b_dev, bn * 4, hipMemcpyDeviceToHost));
  (void)c;
  (void)g;
  return SVC_OK;
}

static void free_packed(svc_ctx* c, PackedGemm& g) {
  // op-level packs are temporary: release the two allocations made by pack_gemm
  for (void* p : {(void*)g.W, (void*)g.bias}) {
    for (auto it = c->allocs.begin(); it != c->allocs.end(); ++it)
      if (*it == p) {
        c->allocs.erase(it);
        break;
      }
    (void)hipFree(p);
  }
}

svc_status svc_op_conv1d(const float* x, int B, int T_in, int Cin, const float* w, const float* bias, int Cout, int k,
                         int stride, int dilation, int pad, int act, float* y, void* stream) {
  svc_ctx* c;
  op_ws(&c);
  TuningScope tuning_scope_(&c->tune);
  hipStream_t s = (hipStream_t)stream;
  const int T_out = (T_in + 2 * pad - dilation * (k - 1) - 1) / stride + 1;
  SVC_REQUIRE(T_out > 0, "op_conv1d: T_out=%d", T_out);
  std::vector<float> wh, bh;
  PackedGemm g;
  int st;
  if ((st = pack_from_device(c, g, w, (size_t)Cout * Cin * k, bias, Cout, wh, bh))) return st;
  const int Cp = (int)round_up(Cin, 8);
  if ((st = pack_conv1d(c, g, wh.data(), bh.data(), Cout, Cin, k, Cp, dilation, pad, stride))) return st;
  if ((st = c->ws.reserve(std::max((size_t)B * T_in * Cp * 2 + 4096, c->ws.cap)))) return st;
  c->ws.reset();
  WS_GET(f16, x16, (size_t)B * T_in * Cp);
  if ((st = f32_to_f16(x, Cin, x16, Cp, B * T_in, Cin, Cp, s, false))) return st;
  EpiArgs e = epi();
  e.act = act;
  e.out32 = y;
  e.ld32 = Cout;
  st = run_gemm(g, x16, Cp, Cin, B, T_in, T_out, e, s);
  (void)hipStreamSynchronize(s);
  free_packed(c, g);
  return st;
}

svc_status svc_op_amp_conv(const float* x, int B, int L, int C, const float* alpha_log, const float* beta_log,
                           const float* filt, const float* w, const float* bias, int k, int d, const float* add_row,
                           float* y, void* stream) {
  svc_ctx* c;
  op_ws(&c);
  TuningScope tuning_scope_(&c->tune);
  hipStream_t s = (hipStream_t)stream;
  SVC_REQUIRE(amp_conv_supported(C, k, d), "op_amp_conv: C=%d k=%d d=%d unsupported", C, k, d);
  std::vector<float> wh, bh;
  PackedGemm g;
  int st;
  if ((st = pack_from_device(c, g, w, (size_t)C * C * k, bias, C, wh, bh))) return st;
  if ((st = pack_conv1d(c, g, wh.data(), bh.data(), C, C, k, C, d, (k - 1) / 2 * d, 1))) return st;
  EpiArgs e = epi();
  e.out32 = y;
  e.ld32 = C;
  e.add_row = add_row;
  e.ld_add_row = C;
  const AmpConvArgs p{x, B, L, k, d, alpha_log, beta_log, filt, g.W, g.Kpad, g.bias};
  st = amp_conv(p, C, e, s);
  (void)hipStreamSynchronize(s);
  free_packed(c, g);
  return st;
}

svc_status svc_op_conv_transpose1d(const float* x, int B, int T_in, int Cin, const float* w, const float* bias,
                                   int Cout, int k, int stride, int pad, float* y, void* stream) {
  svc_ctx* c;
  op_ws(&c);
  TuningScope tuning_scope_(&c->tune);
  hipStream_t s = (hipStream_t)stream;
  const int T_out = (T_in - 1) * stride - 2 * pad + k;
  SVC_REQUIRE(T_out == T_in * stride, "op_conv_transpose1d: only T_out = T_in*stride supported (got %d)", T_out);
  SVC_REQUIRE(Cin % 8 == 0, "op_conv_transpose1d: Cin %% 8");
  std::vector<float> wh, bh;
  PackedGemm g;
  int st;
  if ((st = pack_from_device(c, g, w, (size_t)Cout * Cin * k, bias, Cout, wh, bh))) return st;
  std::vector<PackedGemm> ph;
  if ((st = pack_conv_transpose(c, ph, wh.data(), nullptr, bh.data(), Cin, Cout, k, stride, pad))) return st;
  if ((st = c->ws.reserve(std::max((size_t)B * T_in * Cin * 2 + 4096, c->ws.cap)))) return st;
  c->ws.reset();
  WS_GET(f16, x16, (size_t)B * T_in * Cin);
  if ((st = f32_to_f16(x, Cin, x16, Cin, B * T_in, Cin, Cin, s, false))) return st;
  for (int r = 0; r < stride && !st; ++r) {
    EpiArgs e = epi();
    e.T_ostore = T_out;
    e.ostride = stride;
    e.ophase = r;
    e.out32 = y;
    e.ld32 = Cout;
    st = run_gemm(ph[r], x16, Cin, Cin, B, T_in, T_in, e, s);
  }
  (void)hipStreamSynchronize(s);
  for (auto& p : ph) free_packed(c, p);
  return st;
}

svc_status svc_op_activation1d(const float* x, int B, int L, int C, const float* al, const float* be, const float* f,
                               float* y, void* stream) {
  svc_ctx* c;
  op_ws(&c);
  TuningScope tuning_scope_(&c->tune);
  hipStream_t s = (hipStream_t)stream;
  int st;
  if ((st = c->ws.reserve(std::max((size_t)B * L * C * 2 + 4096, c->ws.cap)))) return st;
  c->ws.reset();
  WS_GET(f16, y16, (size_t)B * L * C);
  if ((st = activation1d(x, y16, B, L, C, C, al, be, f, s))) return st;
  // widen for the caller (the product path feeds the f16 tensor straight into the next conv)
  return f16_to_f32(y16, y, (int64_t)B * L * C, s);
}

svc_status svc_op_activation1d_x16(const void* x16, int B, int L, int C, const float* al, const float* be,
                                   const float* f, float* y, void* stream) {
  svc_ctx* c;
  op_ws(&c);
  TuningScope tuning_scope_(&c->tune);
  hipStream_t s = (hipStream_t)stream;
  int st;
  if ((st = c->ws.reserve(std::max((size_t)B * L * C * 2 + 4096, c->ws.cap)))) return st;
  c->ws.reset();
  WS_GET(f16, y16, (size_t)B * L * C);
  if ((st = activation1d(nullptr, y16, B, L, C, C, al, be, f, s, nullptr, 1, (const f16*)x16))) return st;
  return f16_to_f32(y16, y, (int64_t)B * L * C, s);
}

svc_status svc_op_attention(const float* q, const float* k, const float* v, int B, int L, int D, float* out,
                            void* stream) {
  svc_ctx* c;
  op_ws(&c);
  TuningScope tuning_scope_(&c->tune);
  hipStream_t s = (hipStream_t)stream;
  int st;
  const size_t rows = (size_t)B * L;
  if ((st = c->ws.reserve(std::max(rows * D * 2 * 4 + 4096, c->ws.cap)))) return st;
  c->ws.reset();
  WS_GET(f16, qkv, rows * 3 * D);
  WS_GET(f16, o16, rows * D);
  if ((st = pack_qkv(q, k, v, qkv, (int64_t)rows, D, powf(64.0f, -0.25f), s))) return st;
  if ((st = attention(qkv, o16, B, L, D, s, false))) return st;
  return f16_to_f32(o16, out, (int64_t)rows * D, s);
}

svc_status svc_op_layernorm(const float* x, const float* g, const float* b, int rows, int D, float* y, void* stream) {
  return layernorm_f32(x, g, b, y, rows, D, D, (hipStream_t)stream);
}

}  // extern "C"

// ---------------------------------------------------------------------------- GEMM microbenchmark
// Times `iters` launches of one implicit-GEMM configuration on synthetic operands (tools/gemm_bench.py):
// M rows, N packed columns, K = taps*Cp, 1-tap or 3-tap conv, epilogue 0 = f16 store, 1 = paired gate.
__global__ void fill_f16_kernel(f16* p, int64_t n, uint32_t seed) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t h = (uint32_t)i * 2654435761u ^ seed;
  h ^= h >> 13;
  h *= 0x5bd1e995u;
  h ^= h >> 15;
  p[i] = (f16)(((h & 0xFFFF) / 65536.0f - 0.5f) * 0.5f);
}

extern "C" svc_status svc_gemm_bench(int M, int N, int Cin, int taps, int epi_kind, int variant, int iters, double* ms_out) {
  svc_ctx* oc;
  op_ws(&oc);
  TuningScope tuning_scope_(&oc->tune);
  SVC_REQUIRE(M > 0 && N > 0 && Cin % 8 == 0 && taps >= 1 && iters != 0, "gemm_bench: bad args");
  SVC_REQUIRE(epi_kind < 3 || epi_kind == 6 || variant == 24,
              "gemm_bench: the diagnostic gate epilogues (3-5) exist in variant 24 only");
  SVC_REQUIRE((variant >= 10 && variant <= 16) || variant == 20 || variant == 24 ||
                  (variant == 30 && epi_kind == 6 && N == 384 && Cin == 384 && taps == 1) ||
                  (variant == 40 && epi_kind == 1 && N == 768 && Cin == 384 && taps == 3),
              "gemm_bench: variant %d (30: res_proj, split residual epilogue, N = Cin = 384, 1 tap; 40: gate_ws, "
              "gate epilogue, N = 768, Cin = 384, 3 taps)", variant);
  const int K = taps * Cin, Kpad = (int)round_up(K, 64), Npad = (int)std::max(round_up(N, 256), round_up(N, 384));
  f16 *X, *W, *Y, *cp;
  float *bias, *R = nullptr;
  if (epi_kind == 2 || epi_kind == 6) {  // DiffSVC residual epilogue: x32 (6: split-fp16 lo half) read-modify-write
    SVC_HIP_CHECK(hipMalloc(&R, (size_t)M * N * 4));
    SVC_HIP_CHECK(hipMemset(R, 0, (size_t)M * N * 4));
  }
  SVC_HIP_CHECK(hipMalloc(&X, (size_t)M * Cin * 2));
  SVC_HIP_CHECK(hipMalloc(&W, (size_t)Npad * Kpad * 2));
  SVC_HIP_CHECK(hipMalloc(&Y, (size_t)M * N * 2));
  SVC_HIP_CHECK(hipMalloc(&cp, (size_t)M * N * 2));
  SVC_HIP_CHECK(hipMalloc(&bias, (size_t)Npad * 4));
  SVC_HIP_CHECK(hipMemset(bias, 0, (size_t)Npad * 4));
  hipLaunchKernelGGL(fill_f16_kernel, dim3(cdiv((int64_t)M * Cin, 256)), dim3(256), 0, 0, X, (int64_t)M * Cin, 1u);
  hipLaunchKernelGGL(fill_f16_kernel, dim3(cdiv((int64_t)Npad * Kpad, 256)), dim3(256), 0, 0, W, (int64_t)Npad * Kpad, 2u);
  hipLaunchKernelGGL(fill_f16_kernel, dim3(cdiv((int64_t)M * N, 256)), dim3(256), 0, 0, cp, (int64_t)M * N, 3u);
  // Y is also the residual hi half of the split epilogue (epi 6 / res_proj): defined values, no NaN / Inf patterns
  hipLaunchKernelGGL(fill_f16_kernel, dim3(cdiv((int64_t)M * N, 256)), dim3(256), 0, 0, Y, (int64_t)M * N, 4u);
  ConvGemmArgs a{};
  a.X = X; a.ldx = Cin; a.T_in = M; a.Cp = Cin; a.Cvalid = Cin; a.W = W; a.K = K; a.Kpad = Kpad;
  a.tap_mul = 1; a.tap_add = -(taps / 2); a.istride = 1; a.B = 1; a.T_out = M; a.N = N;
  if (const char* dv = getenv("SVC_BENCH_DIL")) {  // (bench tool only) the dilated conv's tap shift
    a.tap_mul = atoi(dv);
    a.tap_add = -(taps / 2) * a.tap_mul;
  }
  EpiArgs e = epi();
  e.bias = bias; e.T_ostore = M; e.ostride = 1;
  if (epi_kind == 1 || (epi_kind >= 3 && epi_kind <= 5)) {  // diagnostics: 3 = no cp read, no y store; 4 = no cp read; 5 = no y store
    e.kind = EPI_GATE; e.cp = (epi_kind == 3 || epi_kind == 4) ? nullptr : cp; e.ld_cp = N;
    e.y16 = (epi_kind == 3 || epi_kind == 5) ? nullptr : Y;
    e.ldy16 = N / 2;
  } else {
    e.out16 = Y; e.ld16 = N;
    if (epi_kind == 2) {
      e.acc32 = R; e.ld_acc = N; e.acc_div = 1.41421356237309515f; e.out32 = R; e.ld32 = N; e.add16 = bias;
    } else if (epi_kind == 6) {  // split residual in place, as diffsvc.outproj: (Y + lo) - sub -> Y / lo
      e.acc16_hi = Y; e.acc16_lo = reinterpret_cast<f16*>(R); e.acc_sub = bias; e.lo16 = reinterpret_cast<f16*>(R);
      e.ld_acc = N; e.acc_div = 1.41421356237309515f; e.add16 = bias;
    }
  }
  f16* Wf = nullptr;  // variant 30 / 40: res_proj's / gate_ws's fragment-order weights
  int st = SVC_OK;
  if (variant == 30) {
    SVC_HIP_CHECK(hipMalloc(&Wf, res_proj_pack_elems() * sizeof(f16)));
    st = res_proj_pack(W, Kpad, Wf, 0);  // (on failure: no launches below, the buffers are freed at the end)
  } else if (variant == 40) {
    SVC_HIP_CHECK(hipMalloc(&Wf, gate_ws_pack_elems() * sizeof(f16)));
    st = gate_ws_pack(W, Kpad, Wf, 0);
    a.Wfrag = Wf;
  }
  hipEvent_t e0, e1;
  SVC_HIP_CHECK(hipEventCreate(&e0));
  SVC_HIP_CHECK(hipEventCreate(&e1));
  // iters < 0: |iters| launches each after a 1 GiB (SVC_BENCH_FLUSH_MB) memset (operands evicted from L2 and the 256 MiB Infinity Cache,
  // as inside the sampler, where other layers' buffers stream between two launches of one GEMM), timed one by one
  const bool cold = iters < 0;
  if (cold) iters = -iters;
  void* flush = nullptr;
  size_t flush_bytes = (size_t)1 << 30;
  if (const char* fm = getenv("SVC_BENCH_FLUSH_MB")) flush_bytes = (size_t)atoi(fm) << 20;  // (bench tool only)
  if (cold) SVC_HIP_CHECK(hipMalloc(&flush, flush_bytes));
  auto run = [&]() {
    if (variant == 30) return res_proj(X, Wf, bias, bias, bias, e.acc_div, Y, reinterpret_cast<f16*>(R), M, false, 0, 0);
    if (variant == 20 || variant == 24) return conv_gemm4(a, e, zero_page(), 0, variant == 24);
    if (variant == 40) return gate_ws(a, e, 0);
    return conv_gemm3(a, e, zero_page(), variant - 10, 0);
  };
  for (int w = 0; w < 2 && !st; ++w) st = run();
  if (const char* sp = variant == 40 ? getenv("SVC_GWS_STAMPS") : nullptr) {  // (bench tool only) step timeline
    unsigned long long* ds = nullptr;
    const size_t n = (size_t)256 * gate_ws_nstamp();
    SVC_HIP_CHECK(hipMalloc(&ds, n * 8));
    SVC_HIP_CHECK(hipMemset(ds, 0, n * 8));
    SVC_HIP_CHECK(hipDeviceSynchronize());
    gate_ws_stamps = ds;
    for (int w = 0; w < 3 && !st; ++w) st = run();  // the last launch's stamps remain
    gate_ws_stamps = nullptr;
    SVC_HIP_CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> hs(n);
    SVC_HIP_CHECK(hipMemcpy(hs.data(), ds, n * 8, hipMemcpyDeviceToHost));
    (void)hipFree(ds);
    if (FILE* f = fopen(sp, "wb")) {
      fwrite(hs.data(), 8, n, f);
      fclose(f);
    }
  }
  if (const char* dump = getenv("SVC_BENCH_DUMP")) {  // (bench tool only) the gate output of the warm-up launches
    SVC_HIP_CHECK(hipDeviceSynchronize());
    std::vector<f16> hy((size_t)M * N / 2);
    SVC_HIP_CHECK(hipMemcpy(hy.data(), Y, hy.size() * sizeof(f16), hipMemcpyDeviceToHost));
    if (FILE* f = fopen(dump, "wb")) {
      fwrite(hy.data(), sizeof(f16), hy.size(), f);
      fclose(f);
    }
  }
  float ms = 0;
  if (cold) {
    for (int i = 0; i < iters && !st; ++i) {
      SVC_HIP_CHECK(hipMemsetAsync(flush, i & 0xff, flush_bytes, 0));
      SVC_HIP_CHECK(hipEventRecord(e0, 0));
      st = run();
      SVC_HIP_CHECK(hipEventRecord(e1, 0));
      SVC_HIP_CHECK(hipEventSynchronize(e1));
      float one = 0;
      SVC_HIP_CHECK(hipEventElapsedTime(&one, e0, e1));
      ms += one;
    }
    (void)hipFree(flush);
  } else if (getenv("SVC_BENCH_PERLAUNCH")) {  // (bench tool only) each launch between its own event pair, as
    // bench.py's live profile brackets them: the event markers' own cost per launch
    std::vector<hipEvent_t> ev(2 * (size_t)iters);
    for (auto& x : ev) SVC_HIP_CHECK(hipEventCreate(&x));
    for (int i = 0; i < iters && !st; ++i) {  // back to back, no host synchronisation in between
      SVC_HIP_CHECK(hipEventRecord(ev[2 * i], 0));
      st = run();
      SVC_HIP_CHECK(hipEventRecord(ev[2 * i + 1], 0));
    }
    SVC_HIP_CHECK(hipEventSynchronize(ev.back()));
    for (int i = 0; i < iters; ++i) {
      float one = 0;
      SVC_HIP_CHECK(hipEventElapsedTime(&one, ev[2 * i], ev[2 * i + 1]));
      ms += one;
    }
    for (auto& x : ev) (void)hipEventDestroy(x);
  } else {
    SVC_HIP_CHECK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters && !st; ++i)
      st = run();
    SVC_HIP_CHECK(hipEventRecord(e1, 0));
    SVC_HIP_CHECK(hipEventSynchronize(e1));
    SVC_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  }
  *ms_out = ms / iters;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  for (void* p : {(void*)X, (void*)W, (void*)Y, (void*)cp, (void*)bias, (void*)R, (void*)Wf}) if (p) (void)hipFree(p);
  return st;
}
