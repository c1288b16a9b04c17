// Spectral front-ends on gfx950:
//   * 24 kHz log-mel + energy: utils/mel.py:130-174,199 (reflect pad 384, n_fft 1024, hop 256,
//     periodic Hann, sqrt(re^2+im^2+1e-9), slaney mel [100x513], ln(clamp 1e-5))
//   * Whisper log-mel: utils/whisper_extractor/audio.py:92-124 (pad/trim 480000, center reflect pad
//     200, n_fft 400, hop 160, |X|^2, mel_80, log10(clamp 1e-10), max(x, max-8), (x+4)/4)
// The DFT is evaluated directly per (frame, bin) with f64 accumulation and an f64 twiddle table in
// LDS (8 frames per workgroup share every twiddle read); the window multiply is f32 as in torch.stft.
#include "common.h"

namespace svc {

constexpr int DFT_FR = 8;  // frames per workgroup

struct DftArgs {
  const float* wav; int64_t wav_stride; int64_t n_valid;  // samples per utterance actually present
  int64_t n_logical;  // length of the (zero-extended) signal the reflection is taken on
  int n_fft, hop, pad, n_frames, nbins;
  const float* window;  // [n_fft]
  int mode;             // 0: sqrt(|X|^2 + 1e-9) ; 1: |X|^2
  float* out;           // [B*n_frames][nbins]
  // ragged batches (optional): utterance b has nb[b] samples (its n_valid and n_logical) and Tb[b] frames
  const int64_t* nb;
  const int* Tb;
};

__global__ __launch_bounds__(256) void dft_kernel(DftArgs a) {
  extern __shared__ __align__(16) unsigned char dsm[];
  double* cs = reinterpret_cast<double*>(dsm);      // [n_fft] cos
  double* sn = cs + a.n_fft;                          // [n_fft] sin
  float* xs = reinterpret_cast<float*>(sn + a.n_fft);  // [DFT_FR][n_fft]
  const int f0 = blockIdx.y * DFT_FR;
  const int b = blockIdx.z;
  const float* w = a.wav + (int64_t)b * a.wav_stride;
  const int64_t n_valid = a.nb ? a.nb[b] : a.n_valid, n_logical = a.nb ? a.nb[b] : a.n_logical;
  const int n_frames = a.Tb ? min(a.n_frames, a.Tb[b]) : a.n_frames;
  if (f0 >= n_frames) return;  // block-uniform, before any barrier (zero_tail_rows clears those rows' outputs)
  for (int i = threadIdx.x; i < a.n_fft; i += blockDim.x) {
    double s, c;
    sincospi(2.0 * (double)i / (double)a.n_fft, &s, &c);
    cs[i] = c;
    sn[i] = s;
  }
  for (int i = threadIdx.x; i < DFT_FR * a.n_fft; i += blockDim.x) {
    int fr = i / a.n_fft, j = i - fr * a.n_fft;
    int f = f0 + fr;
    float v = 0.f;
    if (f < n_frames) {
      int64_t idx = (int64_t)f * a.hop + j - a.pad;
      if (idx < 0) idx = -idx;
      if (idx >= n_logical) idx = 2 * (n_logical - 1) - idx;
      v = idx < n_valid ? w[idx] : 0.f;
      v = v * a.window[j];
    }
    xs[i] = v;
  }
  __syncthreads();
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.nbins) return;
  double re[DFT_FR], im[DFT_FR];
#pragma unroll
  for (int fr = 0; fr < DFT_FR; ++fr) re[fr] = im[fr] = 0.0;
  int idx = 0;
  for (int j = 0; j < a.n_fft; ++j) {
    const double c = cs[idx], s = sn[idx];
#pragma unroll
    for (int fr = 0; fr < DFT_FR; ++fr) {
      const double x = (double)xs[fr * a.n_fft + j];
      re[fr] += x * c;
      im[fr] -= x * s;
    }
    idx += k;
    if (idx >= a.n_fft) idx -= a.n_fft;
  }
#pragma unroll
  for (int fr = 0; fr < DFT_FR; ++fr) {
    const int f = f0 + fr;
    if (f >= n_frames) break;
    const float r = (float)re[fr], i = (float)im[fr];
    float v;
    if (a.mode == 0) {
      v = sqrtf(r * r + i * i + 1e-9f);
    } else {
      float m = sqrtf(r * r + i * i);
      v = m * m;
    }
    a.out[((int64_t)b * a.n_frames + f) * a.nbins + k] = v;
  }
}

int dft_frames(const DftArgs& a, int B, hipStream_t s) {
  SVC_REQUIRE(a.n_fft <= 1024 && a.n_frames > 0, "dft: n_fft=%d frames=%d", a.n_fft, a.n_frames);
  size_t lds = (size_t)a.n_fft * 2 * sizeof(double) + (size_t)DFT_FR * a.n_fft * sizeof(float);
  dim3 grid(cdiv(a.nbins, 256), cdiv(a.n_frames, DFT_FR), B);
  hipLaunchKernelGGL(dft_kernel, grid, dim3(256), lds, s, a);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
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
__global__ void mel_log_kernel(const float* __restrict__ spec, int nbins, const float* __restrict__ fb, int n_mels,
                               float* __restrict__ out, int rows, int mode) {
  const int row = blockIdx.x;
  extern __shared__ float sp[];
  for (int k = threadIdx.x; k < nbins; k += blockDim.x) sp[k] = spec[(int64_t)row * nbins + k];
  __syncthreads();
  for (int m = threadIdx.x; m < n_mels; m += blockDim.x) {
    const float* fr = fb + (int64_t)m * nbins;
    float acc = 0.f;
    for (int k = 0; k < nbins; ++k) acc = fmaf(fr[k], sp[k], acc);
    float v = mode == 0 ? logf(fmaxf(acc, 1e-5f)) : log10f(fmaxf(acc, 1e-10f));
    out[(int64_t)row * n_mels + m] = v;
  }
}

int mel_log(const float* spec, int nbins, const float* fb, int n_mels, float* out, int rows, int mode, hipStream_t s) {
  hipLaunchKernelGGL(mel_log_kernel, dim3(rows), dim3(128), nbins * sizeof(float), s, spec, nbins, fb, n_mels, out,
                     rows, mode);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

// energy = sqrt(sum_m exp(mel)^2) (utils/mel.py:199)
__global__ void energy_kernel(const float* __restrict__ mel, int n_mels, float* __restrict__ en, int rows) {
  int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  float acc = 0.f;
  for (int m = 0; m < n_mels; ++m) {
    float e = expf(mel[(int64_t)r * n_mels + m]);
    acc += e * e;
  }
  en[r] = sqrtf(acc);
}

int energy_from_mel(const float* mel, int n_mels, float* en, int rows, hipStream_t s) {
  hipLaunchKernelGGL(energy_kernel, dim3(cdiv(rows, 256)), dim3(256), 0, s, mel, n_mels, en, rows);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

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
                                    int64_t n_per_utt, int B, int split_c) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_per_utt * B) return;
  int b = (int)(i / n_per_utt);
  float v = fmaxf(x[i], mx[b] - 8.0f);
  const float o = (v + 4.0f) / 4.0f;
  if (split_c == 0) {
    y[i] = (f16)o;
    return;
  }
  // split-fp16 operand rows [hi | lo | hi] of split_c (= n_mels) columns each
  const int64_t r = i / split_c;
  const int c = (int)(i - r * split_c);
  const f16 hi = (f16)o;
  f16* yr = y + r * 3 * split_c;
  yr[c] = hi;
  yr[split_c + c] = (f16)(o - (float)hi);
  yr[2 * split_c + c] = hi;
}

int whisper_normalize(const float* logspec, float* mx_scratch, f16* out, int B, int64_t n_per_utt, hipStream_t s,
                      int split_c) {
  hipLaunchKernelGGL(rowblock_max_kernel, dim3(B), dim3(1024), 0, s, logspec, n_per_utt, mx_scratch);
  SVC_LAUNCH_CHECK();
  int64_t n = n_per_utt * B;
  hipLaunchKernelGGL(whisper_norm_kernel, dim3(cdiv(n, 256)), dim3(256), 0, s, logspec, mx_scratch, out, n_per_utt, B,
                     split_c);
  SVC_LAUNCH_CHECK();
  return SVC_OK;
}

}  // namespace svc
