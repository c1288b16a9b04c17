// Spectral front-end launch arguments (features.hip), shared with engine.hip.
#pragma once
#include "common.h"

namespace svc {

struct DftArgs {
  const float* wav; int64_t wav_stride; int64_t n_valid;  // samples per utterance actually present
  int64_t n_logical;  // length of the (zero-extended) signal the reflection is taken on
  int n_fft, hop, pad, n_frames, nbins;
  const float* window;  // [n_fft]
  const double2* twiddle;  // [n_fft] W^m = (cos, -sin)(2 pi m / n_fft)
  int mode;             // 0: sqrt(|X|^2 + 1e-9) -> ln(max(mel, 1e-5)) ; 1: |X|^2 -> log10(max(mel, 1e-10))
  const float* fb;      // the filterbank's nonzero band of each filter, packed: fb_len floats
  const int* band;      // [n_mels][3]: band [lo, hi) of each filter and its offset in fb
  int fb_len;
  int n_mels;
  float* out;           // [B*n_frames][n_mels] log-mel
  float* energy;        // optional [B*n_frames]: sqrt(sum_m exp(mel)^2) (utils/mel.py:199)
  // ragged batches (optional): utterance b has nb[b] samples (its n_valid and n_logical) and Tb[b] frames
  const int64_t* nb;
  const int* Tb;
};

// windowed frames -> f64 FFT -> |X| or |X|^2 -> filterbank -> ln / log10 (-> energy), one launch
int dft_mel(const DftArgs& a, int B, hipStream_t s);
bool dft_mel_supported(int n_fft);  // 400, 512, 1024, 2048

}  // namespace svc
