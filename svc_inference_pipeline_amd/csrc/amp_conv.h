// Fused BigVGAN AMP activation + conv for C = 24 / 48 / 96 (amp_conv.hip).
#pragma once
#include "common.h"

namespace svc {

struct AmpConvArgs {
  const float* x;  // [B*L][C] activation input (f32)
  int B, L, k, d;  // conv taps and dilation; padding (k-1)/2*d keeps the length
  const float* alpha_log;
  const float* beta_log;
  const float* filt;  // 12-tap kaiser-sinc filter shared by up- and down-sampling
  const f16* W;       // packed weights [Npad][Kpad], K index = tap*C + ci (pack_conv1d with Cp = C)
  int Kpad;
  const float* bias;
  const int* tv = nullptr;  // ragged batches: utterance b has min(L, tv[b] * tv_mul) rows (NULL = all L)
  int tv_mul = 1;
  const f16* x16 = nullptr;  // when set, the activation input is this f16 tensor instead of x (an AMPBlock1 intermediate)
  bool noact = false;  // x16 is the conv's input itself, already activated (C = 96): the plain conv, no SnakeBeta
  int dbg = 0;  // (diagnostics, SVC_AMP_DBG) 1 / 2 / 4: skip the activation / conv MFMAs / epilogue; 8: register epilogue
};

bool amp_conv_supported(int C, int k, int d);
// act + conv + epilogue; e may use out32 / out16 / add_row / acc32 (+ acc_div), all with leading dimension C
int amp_conv(const AmpConvArgs& p, int C, const EpiArgs& e, hipStream_t s);

}  // namespace svc
