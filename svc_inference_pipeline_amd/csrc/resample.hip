// Rational-ratio resampling: the reference resamples the source wav to 24 kHz with
// librosa (soxr, utils/audio.py:49-53) and decodes a 16 kHz int16 copy with ffmpeg for Whisper
// (utils/whisper_extractor/audio.py:22-49). Neither library is in this image, so the algorithm implemented
// (and pinned by tests/test_audio.py against scipy) is scipy.signal.resample_poly's, with its default
// Kaiser(beta = 5) window:
//   g = gcd(sr_in, sr_out), up = sr_out/g, down = sr_in/g, R = max(up, down), half = 10 R
//   h = firwin(2 half + 1, cutoff 1/R, kaiser(5)) * up, pre-padded with (down - half % down) zeros
//   y[n] = sum_k h[k] * xu[(n + pre_remove) * down - k],  xu = x up-sampled by zero insertion
// Every output sample needs only the ~(2 half + 1)/up taps congruent to its phase: one thread per output,
// f64 taps and accumulation (the filter is designed in f64 on the host), coalesced input reads.
#include <cmath>
#include <map>
#include <mutex>
#include <numeric>
#include <vector>

#include "common.h"
#include "svc_hip.h"

namespace svc {

struct ResamplePlan {
  int up = 1, down = 1, half = 0, pre_pad = 0, pre_remove = 0, taps = 0;  // taps = len(h) incl. padding
  double* h = nullptr;                                                  // device, f64
};

namespace {

double bessel_i0(double x) {
  double sum = 1.0, term = 1.0, q = x * x / 4.0;
  for (int k = 1; k < 200; ++k) {
    term *= q / ((double)k * k);
    sum += term;
    if (term < 1e-17 * sum) break;
  }
  return sum;
}

// scipy.signal.firwin(numtaps, cutoff, window=('kaiser', beta)) for a low-pass, scale=True
std::vector<double> firwin_kaiser(int numtaps, double cutoff, double beta) {
  std::vector<double> h(numtaps);
  const double alpha = 0.5 * (numtaps - 1), i0b = bessel_i0(beta);
  double s = 0.0;
  for (int n = 0; n < numtaps; ++n) {
    const double m = n - alpha;
    const double xm = cutoff * m;
    const double sinc = xm == 0.0 ? 1.0 : std::sin(M_PI * xm) / (M_PI * xm);
    const double r = 2.0 * n / (numtaps - 1) - 1.0;
    const double w = bessel_i0(beta * std::sqrt(std::max(0.0, 1.0 - r * r))) / i0b;
    h[n] = cutoff * sinc * w;
    s += h[n];
  }
  for (double& v : h) v /= s;
  return h;
}

int64_t out_len(int64_t n_in, int up, int down) {
  const int64_t n = n_in * up;
  return n / down + (n % down ? 1 : 0);
}

}  // namespace

__global__ void resample_kernel(const float* __restrict__ x, int64_t n_in, int64_t n_out, ResamplePlan p,
                                int quantize16, float* __restrict__ y) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (n >= n_out) return;
  const float* xb = x + (int64_t)b * n_in;
  const int64_t j = (n + p.pre_remove) * p.down;  // index into the filtered up-sampled signal
  const int k0 = (int)(j % p.up);
  const int64_t i0 = j / p.up;                    // x index paired with tap k0
  // taps k = k0 + up*r (r >= 0) pair with x[i0 - r]; keep 0 <= k < taps and 0 <= i0 - r < n_in
  int64_t r_lo = i0 - (n_in - 1);
  if (r_lo < 0) r_lo = 0;
  int64_t r_hi = (p.taps - 1 - k0) / p.up;
  if (r_hi > i0) r_hi = i0;
  double acc = 0.0;
  for (int64_t r = r_lo; r <= r_hi; ++r) acc += p.h[k0 + p.up * r] * (double)xb[i0 - r];
  float v = (float)acc;
  if (quantize16) {  // ffmpeg s16le decode: lrint(x * 32768) clipped, back to float / 32768
    double q = rint((double)v * 32768.0);
    q = q < -32768.0 ? -32768.0 : (q > 32767.0 ? 32767.0 : q);
    v = (float)(q / 32768.0);
  }
  y[(int64_t)b * n_out + n] = v;
}

// host-side filter design (no device memory): the padded taps and the plan's integers
static ResamplePlan design_plan(int sr_in, int sr_out, std::vector<double>& hp) {
  ResamplePlan p;
  const int g = std::gcd(sr_in, sr_out);
  p.up = sr_out / g;
  p.down = sr_in / g;
  const int R = std::max(p.up, p.down);
  p.half = 10 * R;
  std::vector<double> h = firwin_kaiser(2 * p.half + 1, 1.0 / R, 5.0);
  for (double& v : h) v *= p.up;
  p.pre_pad = p.down - p.half % p.down;
  p.pre_remove = (p.half + p.pre_pad) / p.down;
  hp.assign(p.pre_pad, 0.0);
  hp.insert(hp.end(), h.begin(), h.end());
  p.taps = (int)hp.size();  // trailing zero padding adds nothing to the sum: omitted
  return p;
}

static const ResamplePlan* get_plan(int sr_in, int sr_out) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, ResamplePlan> plans;
  std::lock_guard<std::mutex> lock(mu);
  auto it = plans.find({sr_in, sr_out});
  if (it != plans.end()) return &it->second;
  std::vector<double> hp;
  ResamplePlan p = design_plan(sr_in, sr_out, hp);
  if (hipMalloc(&p.h, hp.size() * sizeof(double)) != hipSuccess) return nullptr;
  if (hipMemcpy(p.h, hp.data(), hp.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
  return &(plans[{sr_in, sr_out}] = p);
}

}  // namespace svc

using namespace svc;

extern "C" int64_t svc_resample_len(int64_t n_in, int sr_in, int sr_out) {
  if (n_in < 0 || sr_in <= 0 || sr_out <= 0) return -1;
  const int g = std::gcd(sr_in, sr_out);
  return out_len(n_in, sr_out / g, sr_in / g);
}

// the designed filter (host only, for tests): taps h_pad[0..n) and the integers of the plan
extern "C" svc_status svc_resample_filter(int sr_in, int sr_out, double* h, int cap, int* n, int* up, int* down,
                                          int* pre_remove) {
  SVC_REQUIRE(sr_in > 0 && sr_out > 0 && n && up && down && pre_remove, "resample_filter: bad arguments");
  std::vector<double> hp;
  const ResamplePlan p = design_plan(sr_in, sr_out, hp);
  *n = p.taps;
  *up = p.up;
  *down = p.down;
  *pre_remove = p.pre_remove;
  if (h) {
    SVC_REQUIRE(cap >= p.taps, "resample_filter: capacity %d < %d taps", cap, p.taps);
    std::copy(hp.begin(), hp.end(), h);
  }
  return SVC_OK;
}

extern "C" svc_status svc_resample(const float* x, int B, int64_t n_in, int sr_in, int sr_out, int quantize16, float* y,
                                   void* stream) {
  SVC_REQUIRE(x && y && B >= 1 && n_in >= 1 && sr_in > 0 && sr_out > 0, "resample: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  const int64_t n_out = svc_resample_len(n_in, sr_in, sr_out);
  if (sr_in == sr_out && !quantize16) {
    SVC_HIP_CHECK(hipMemcpyAsync(y, x, (size_t)B * n_in * sizeof(float), hipMemcpyDeviceToDevice, s));
    return SVC_OK;
  }
  const ResamplePlan* p = get_plan(sr_in, sr_out);
  SVC_REQUIRE(p != nullptr, "resample: filter upload failed");
  const int tok = prof_begin("resample", 0.0, (double)B * (n_in + n_out) * 4.0, s);
  hipLaunchKernelGGL(resample_kernel, dim3((unsigned)cdiv64(n_out, 256), (unsigned)B), dim3(256), 0, s, x, n_in, n_out,
                     *p, quantize16, y);
  prof_end(tok, s);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}
