// Spectral front-ends on gfx950:
//   * 24 kHz log-mel + energy: utils/mel.py:130-174,199 (reflect pad 384, n_fft 1024, hop 256,
//     periodic Hann, sqrt(re^2+im^2+1e-9), slaney mel [100x513], ln(clamp 1e-5))
//   * Whisper log-mel: utils/whisper_extractor/audio.py:92-124 (pad/trim 480000, center reflect pad
//     200, n_fft 400, hop 160, |X|^2, mel_80, log10(clamp 1e-10), max(x, max-8), (x+4)/4)
// One kernel per spectrogram: each workgroup takes FR consecutive frames from the waveform to the log-mel rows (the
// spectrum never leaves LDS):
//   1. frame j of n real windowed samples -> LDS as n/2 complex f64 z[m] = x[2m] + i x[2m+1];
//   2. Z = FFT_{n/2}(z): Stockham autosort stages (radix 4 / 2 for n/2 = 256 / 512 / 1024, 8 / 5 / 5 for Whisper's
//      n/2 = 200), one thread per butterfly, read -> barrier -> write in place, twiddles from an exact f64 table;
//   3. X[k] = (Z[k] + Z*[n/2-k]) / 2 + W_n^k (Z[k] - Z*[n/2-k]) / 2i, k = 0..n/2 (the real-input split), |X| (f32, as
//      torch) -> LDS, then the slaney filterbank over each filter's nonzero band only (the same f32 fma sequence as a
//      dense dot product: the skipped products are exact zeros), the log, and optionally the frame energy.
// f64 throughout the transform (the oracle's torch.stft is an f32 FFT; f64 keeps this side's error far below it); the
// window multiply is f32 as in torch.stft.
#include "common.h"
#include "spectral.h"
#include "fft.h"

namespace svc {

__device__ __forceinline__ float spec_value(double re, double im, int mode) {
  const float r = (float)re, i = (float)im;
  if (mode == 0) return sqrtf(r * r + i * i + 1e-9f);
  const float m = sqrtf(r * r + i * i);
  return m * m;
}

// radix plans: N = n/2 complex points, TPF threads per frame (one per butterfly of the widest stage), FR frames per
// workgroup
template <int N>
struct FftPlan;
template <>
struct FftPlan<200> {  // Whisper n_fft 400
  static constexpr int TPF = 40, FR = 8;
  __device__ static void run(double2* z, const double2* twp, int t) {
    const auto tw = [twp](int m) { return twp[m]; };
    fft_stage<200, 8, 1, TPF>(z, tw, t);
    fft_stage<200, 5, 8, TPF>(z, tw, t);
    fft_stage<200, 5, 40, TPF>(z, tw, t);
  }
};
template <>
struct FftPlan<256> {
  static constexpr int TPF = 64, FR = 4;
  __device__ static void run(double2* z, const double2* twp, int t) {
    const auto tw = [twp](int m) { return twp[m]; };
    fft_stage<256, 4, 1, TPF>(z, tw, t);
    fft_stage<256, 4, 4, TPF>(z, tw, t);
    fft_stage<256, 4, 16, TPF>(z, tw, t);
    fft_stage<256, 4, 64, TPF>(z, tw, t);
  }
};
template <>
struct FftPlan<512> {  // n_fft 1024
  static constexpr int TPF = 128, FR = 2;
  __device__ static void run(double2* z, const double2* twp, int t) {
    const auto tw = [twp](int m) { return twp[m]; };
    fft_stage<512, 4, 1, TPF>(z, tw, t);
    fft_stage<512, 4, 4, TPF>(z, tw, t);
    fft_stage<512, 4, 16, TPF>(z, tw, t);
    fft_stage<512, 4, 64, TPF>(z, tw, t);
    fft_stage<512, 2, 256, TPF>(z, tw, t);
  }
};
template <>
struct FftPlan<1024> {
  static constexpr int TPF = 256, FR = 1;
  __device__ static void run(double2* z, const double2* twp, int t) {
    const auto tw = [twp](int m) { return twp[m]; };
    fft_stage<1024, 4, 1, TPF>(z, tw, t);
    fft_stage<1024, 4, 4, TPF>(z, tw, t);
    fft_stage<1024, 4, 16, TPF>(z, tw, t);
    fft_stage<1024, 4, 64, TPF>(z, tw, t);
    fft_stage<1024, 4, 256, TPF>(z, tw, t);
  }
};

template <int N>
struct MelLds {  // dynamic LDS layout (bytes)
  using P = FftPlan<N>;
  static constexpr size_t Z = (size_t)P::FR * N * 16, TW = (size_t)2 * N * 16, SP = (size_t)P::FR * (N + 1) * 4;
  static size_t bytes(int fb_len, int n_mels) { return Z + TW + SP + (size_t)(fb_len + P::FR * n_mels) * 4; }
};

template <int N>
__global__ __launch_bounds__(FftPlan<N>::TPF * FftPlan<N>::FR) void dft_mel_kernel(DftArgs a) {
  using P = FftPlan<N>;
  using L = MelLds<N>;
  constexpr int n = 2 * N, NT = P::TPF * P::FR;
  extern __shared__ __align__(16) unsigned char dsm[];
  double2* zs = reinterpret_cast<double2*>(dsm);         // [FR][N] frame / spectrum
  double2* tw = reinterpret_cast<double2*>(dsm + L::Z);  // [n] W_n^m = (cos, -sin)(2 pi m / n)
  float* sp = reinterpret_cast<float*>(dsm + L::Z + L::TW);  // [FR][N + 1] |X|
  float* fbs = sp + P::FR * (N + 1);                     // packed filterbank bands
  float* ml = fbs + a.fb_len;                            // [FR][n_mels] log-mel (energy)
  const int f0 = blockIdx.x * P::FR;
  const int b = blockIdx.y;
  const float* w = a.wav + (int64_t)b * a.wav_stride;
  const int64_t n_valid = a.nb ? a.nb[b] : a.n_valid, n_logical = a.nb ? a.nb[b] : a.n_logical;
  const int n_frames = a.Tb ? min(a.n_frames, a.Tb[b]) : a.n_frames;
  if (f0 >= n_frames) return;  // block-uniform, before any barrier (zero_tail_rows clears those rows' outputs)
  const int nf = min(P::FR, n_frames - f0);
  const int tid = threadIdx.x, fr = tid / P::TPF, t = tid - fr * P::TPF;
  for (int i = tid; i < n; i += NT) tw[i] = a.twiddle[i];
  for (int i = tid; i < a.fb_len; i += NT) fbs[i] = a.fb[i];
  // 1. frame fr: sample j -> the j-th double of z (even samples real, odd imaginary)
  double* zf = reinterpret_cast<double*>(zs + fr * N);
  for (int j = t; j < n; j += P::TPF) {
    float x = 0.f;
    if (fr < nf) {
      int64_t idx = (int64_t)(f0 + fr) * a.hop + j - a.pad;
      if (idx < 0) idx = -idx;
      if (idx >= n_logical) idx = 2 * (n_logical - 1) - idx;
      x = idx < n_valid ? w[idx] : 0.f;
    }
    zf[j] = (double)(x * a.window[j]);
  }
  __syncthreads();
  // 2. FFT
  P::run(zs + fr * N, tw, t);
  // 3. real-input split and magnitudes
  const double2* Z = zs + fr * N;
  for (int k = t; k <= N; k += P::TPF) {
    const double2 zk = Z[k == N ? 0 : k], zm = Z[k == 0 ? 0 : N - k];
    const double2 e = make_double2(0.5 * (zk.x + zm.x), 0.5 * (zk.y - zm.y));   // (Z[k] + Z*[N-k]) / 2
    const double2 o = make_double2(0.5 * (zk.y + zm.y), -0.5 * (zk.x - zm.x));  // (Z[k] - Z*[N-k]) / 2i
    const double2 X = cadd(e, cmul(o, tw[k]));
    sp[fr * (N + 1) + k] = spec_value(X.x, X.y, a.mode);
  }
  __syncthreads();
  const int64_t row0 = (int64_t)b * a.n_frames + f0;
  for (int i = tid; i < nf * a.n_mels; i += NT) {
    const int f = i / a.n_mels, m = i - f * a.n_mels;
    const int lo = a.band[3 * m], hi = a.band[3 * m + 1];
    const float* fbm = fbs + a.band[3 * m + 2] - lo;
    const float* x = sp + f * (N + 1);
    float acc = 0.f;
    for (int kk = lo; kk < hi; ++kk) acc = fmaf(fbm[kk], x[kk], acc);
    const float v = a.mode == 0 ? logf(fmaxf(acc, 1e-5f)) : log10f(fmaxf(acc, 1e-10f));
    a.out[row0 * a.n_mels + i] = v;
    ml[i] = v;
  }
  if (a.energy) {
    __syncthreads();
    if (tid < nf) {
      float acc = 0.f;
      for (int m = 0; m < a.n_mels; ++m) {
        const float e = expf(ml[tid * a.n_mels + m]);
        acc += e * e;
      }
      a.energy[row0 + tid] = sqrtf(acc);
    }
  }
}

bool dft_mel_supported(int n_fft) { return n_fft == 400 || n_fft == 512 || n_fft == 1024 || n_fft == 2048; }

template <int N>
static int launch_dft_mel(const DftArgs& a, int B, hipStream_t s) {
  using P = FftPlan<N>;
  const size_t lds = MelLds<N>::bytes(a.fb_len, a.n_mels);
  SVC_REQUIRE(lds <= 160 * 1024, "dft_mel: %zu B of LDS", lds);
  if (int st = ensure_dyn_lds((const void*)dft_mel_kernel<N>, 160 * 1024)) return st;
  DftArgs p = a;
  dim3 grid(cdiv(a.n_frames, P::FR), B);
  hipLaunchKernelGGL(dft_mel_kernel<N>, grid, dim3(P::TPF * P::FR), lds, s, p);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

int dft_mel(const DftArgs& a, int B, hipStream_t s) {
  SVC_REQUIRE(dft_mel_supported(a.n_fft) && a.nbins == a.n_fft / 2 + 1 && a.n_frames > 0 && a.fb && a.band &&
                  a.n_mels > 0 && a.fb_len > 0 && a.twiddle,
              "dft_mel: n_fft=%d nbins=%d frames=%d mels=%d", a.n_fft, a.nbins, a.n_frames, a.n_mels);
  switch (a.n_fft) {
    case 400: return launch_dft_mel<200>(a, B, s);
    case 512: return launch_dft_mel<256>(a, B, s);
    case 1024: return launch_dft_mel<512>(a, B, s);
    default: return launch_dft_mel<1024>(a, B, s);
  }
}

// ragged batches: rows t >= Tb[b] of a [B][T][C] f32 tensor are set to zero (the frames a clip of that length
// does not have)
__global__ void zero_tail_kernel(float* __restrict__ x, int T, int C, const int* __restrict__ Tb) {
  const int b = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int t0 = Tb[b];
  const int64_t n = (int64_t)(T - t0) * C;
  if (t0 >= T || i >= n) return;
  x[((int64_t)b * T + t0) * C + i] = 0.f;
}

int zero_tail_rows(float* x, int B, int T, int C, const int* Tb, hipStream_t s) {
  hipLaunchKernelGGL(zero_tail_kernel, dim3(cdiv((int64_t)T * C, 256), B), dim3(256), 0, s, x, T, C, Tb);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// mel projection + log: out[row][m] = log(clamp(sum_k fb[m][k] spec[row][k])) ; mode 0 ln/1e-5, 1 log10/1e-10
// Whisper: per-utterance global max of the log10 spectrogram, then clamp/shift -> f16 GEMM operand
__global__ void rowblock_max_kernel(const float* __restrict__ x, int64_t n_per_utt, float* __restrict__ mx) {
  const int b = blockIdx.x;
  const float* xb = x + (int64_t)b * n_per_utt;
  float m = -INFINITY;
  for (int64_t i = threadIdx.x; i < n_per_utt; i += blockDim.x) m = fmaxf(m, xb[i]);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float red[16];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = red[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = fmaxf(r, red[i]);
    mx[b] = r;
  }
}

__global__ void whisper_norm_kernel(const float* __restrict__ x, const float* __restrict__ mx, f16* __restrict__ y,
                                    int64_t n_per_utt, int B, int split_c, bool bf, int ldo) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_per_utt * B) return;
  int b = (int)(i / n_per_utt);
  float v = fmaxf(x[i], mx[b] - 8.0f);
  const float o = (v + 4.0f) / 4.0f;
  if (split_c == 0) {
    y[i] = enc16_lo(o, bf);
    return;
  }
  // split-fp16 operand rows [hi | lo | hi] of split_c (= n_mels) columns each, ldo apart; columns 3 split_c .. ldo - 1
  // are zeros (the conv stem's K padding)
  const int64_t r = i / split_c;
  const int c = (int)(i - r * split_c);
  const f16 hi = enc16_lo(o, bf);
  f16* yr = y + r * ldo;
  yr[c] = hi;
  yr[split_c + c] = enc16_lo(o - dec16(hi, bf), bf);
  yr[2 * split_c + c] = hi;
  if (c < ldo - 3 * split_c) yr[3 * split_c + c] = (f16)0.0f;
}

int whisper_normalize(const float* logspec, float* mx_scratch, f16* out, int B, int64_t n_per_utt, hipStream_t s,
                      int split_c, bool bf, int ldo) {
  SVC_REQUIRE(split_c == 0 || (ldo >= 3 * split_c && ldo - 3 * split_c <= split_c), "whisper_normalize: ldo %d", ldo);
  hipLaunchKernelGGL(rowblock_max_kernel, dim3(B), dim3(1024), 0, s, logspec, n_per_utt, mx_scratch);
  SVC_LAUNCH_CHECK();
  int64_t n = n_per_utt * B;
  hipLaunchKernelGGL(whisper_norm_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, logspec, mx_scratch, out, n_per_utt, B,
                     split_c, bf, ldo);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
