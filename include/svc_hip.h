/*
 * svc_hip.h — C-ABI of libsvc_hip.so, the MI355X (gfx950) singing-voice-conversion hot path.
 *
 * The reference (WallaceRao/svc_inference_pipeline) has no FFI: its boundary is the set of Python
 * functions infer.py calls. Each entry point below replaces one of them (file:line in the reference):
 *
 *   svc_mel_energy      <- utils/mel.py:179-201 extract_mel_features (mel_spectrogram :130-174, energy :199)
 *   svc_f0_ac           <- utils/f0.py:120-161 get_f0_features_using_parselmouth (Praat to_pitch_ac + pad)
 *   svc_pitch_shift     <- utils/acoustic_feature_extraction.py:48-52 pitch_shift
 *   svc_whisper_encode  <- utils/whisper.py:13-28 whisper_encoder (log_mel_spectrogram + AudioEncoder)
 *   svc_map_content     <- utils/whisper.py:31-81 get_mapped_whisper_features
 *   svc_condition       <- modules/encoder.py:165-201 EncoderFramework.forward
 *   svc_diffsvc_sample  <- modules/diffsvcrepo_inference.py:154-240 svc_model_inference (DDPM or PLMS)
 *   svc_bigvgan         <- utils/acoustic_feature_extraction.py:83-97 denormalize_mel_channel
 *                          + modules/bigvgan_inference.py:29-44 synthesis_audios (Generator + trim + fade)
 *
 * Conventions
 *   - Tensors are caller-owned DEVICE buffers, time-major: row = b*T + t, channels contiguous.
 *   - Every call is asynchronous and ordered on `stream` (a hipStream_t; NULL = default stream).
 *   - One context per device; a context is not thread-safe. Calls that share the context's workspace must be
 *     ordered on one stream; svc_mel_energy, svc_f0_ac and svc_pitch_shift are the exception (their own workspace /
 *     none) and may run, ordered among themselves, on a second stream beside the content encoders (the host
 *     pipeline overlaps them with Whisper that way, on svc_ctx_stream(ctx, 2)).
 *   - Parameters are given in the reference's own state_dict naming with a model prefix
 *     ("mapper.", "vocoder.", "whisper.") as host float32 arrays; they are folded (weight_norm),
 *     packed into MFMA layouts and uploaded by svc_ctx_finalize. Host arrays must stay valid until
 *     svc_ctx_finalize returns. A missing or mis-shaped parameter makes finalize fail (the reference
 *     silently keeps random init, utils/load_models.py:34-43).
 *   - Status codes instead of exceptions; svc_last_error() describes the last failure of this thread.
 *   - Ragged batches: a batch holds B utterances of different lengths padded to the longest (rows keep the batch
 *     stride). The per-utterance lengths are HOST arrays — n_samples (int64 [B], samples) for the 24 kHz feature
 *     stages, frames (int32 [B], mel frames) for the sampler and the vocoder; NULL means every utterance has the
 *     batch length. Each utterance is then computed exactly as a clip of its own length (its own reflect / zero /
 *     replicate padding, STFT frames, Praat frame grid, fade-out): outputs are bit-identical to converting it alone,
 *     and the rows past its end are written as zeros. Whisper needs no lengths: pad its 16 kHz input with zeros (as
 *     pad_or_trim does). The tables are staged to the device through a ring of 8 slots per stage group; a slot is
 *     reused only after every kernel of the call that read it has finished (its event is re-recorded on the call's
 *     stream after the call's last launch), so calls may use any streams.
 */
#ifndef SVC_HIP_H
#define SVC_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct svc_ctx svc_ctx;
typedef int svc_status; /* 0 = ok, 1 = invalid argument, 2 = HIP error, 3 = bad state */

#define SVC_MODE_DDPM 0
#define SVC_MODE_PLMS 1

const char* svc_last_error(void);
int svc_abi_version(void);

svc_status svc_ctx_create(int device, svc_ctx** out);
svc_status svc_ctx_destroy(svc_ctx* ctx);
/* numeric configuration (config.json keys, flattened: "fs", "mapper.residual_layer_num", "vocoder.upsample_rates.0",
   ...; and the precision keys "content.split", "content.wsplit_attn" / _mlp / _qk / _v / _out, "mapper.head_split",
   "operands.bf16" (1: the content encoders, conditioner and DiffSVC GEMMs take bfloat16 operands on
   v_mfma_f32_16x16x32_bf16, and content features cross svc_map_content* / svc_condition as bfloat16; BigVGAN stays
   fp16), "hubert.output_layer"). An unknown key is SVC_ERR_INVALID (a misspelt key must not leave a default in place).
   "tune.<name>" keys set a kernel switch of this context at any time (gemm_variant, gemm3_direct, whisper_streams,
   sampler_streams, vocoder_streams, diff_head, amp_maxc, amp_ups, res_proj, gate_ws; "tune.reset" restores the creation-time values). Defaults
   are the measured production kernels; at creation an SVC_<NAME> environment variable overrides each. ctx may be
   NULL for "tune.*" keys: the switches of the op-level entry points (svc_op_*, svc_gemm_bench). */
svc_status svc_ctx_set_config(svc_ctx* ctx, const char* key, double value);
/* the value of a configuration key set on this context, or of a kernel switch ("tune.<name>"; ctx NULL: the
   op-level context's); a key that was never set is SVC_ERR_INVALID */
svc_status svc_ctx_get_config(svc_ctx* ctx, const char* key, double* value);
/* host-only: 1 when `key` is a configuration key svc_ctx_set_config accepts (not "tune.*"), else 0 */
int svc_config_key_known(const char* key);
svc_status svc_ctx_add_param(svc_ctx* ctx, const char* name, const float* host, int ndim, const int64_t* shape);
svc_status svc_ctx_finalize(svc_ctx* ctx);
/* bytes of device memory held by packed weights / by the workspace arena */
svc_status svc_ctx_memory(svc_ctx* ctx, int64_t* weight_bytes, int64_t* workspace_bytes);
/* the context's sub-stream `index` (< 8; created on first use, owned by the context): lets a caller overlap
   svc_f0_ac with the content encoder without creating a stream of its own */
svc_status svc_ctx_stream(svc_ctx* ctx, int index, void** stream);

/* A2/A3-energy: wav24k [B][n_samples] f32 -> mel [B*T][n_mels] f32 (log-mel, time-major), energy [B*T] f32.
   T = (n_samples + n_fft - hop - n_fft)/hop + 1 (bit-exact frame count, utils/mel.py:148-167).
   utt_samples (host int64 [B] or NULL): ragged batch, utterance b's samples (<= n_samples); its T_b frames as above. */
svc_status svc_mel_energy(svc_ctx* ctx, const float* wav24k, int B, int64_t n_samples, const int64_t* utt_samples,
                          float* mel, float* energy, void* stream);

/* A3-F0: Praat autocorrelation pitch (to_pitch_ac, voicing 0.6, floor f0_min, ceiling f0_max, time step hop/fs),
   padded to T frames as utils/f0.py:156-157; unvoiced = 0. f0 [B*T] float64. Uses the feature-stage workspace
   (shared with svc_mel_energy only): may run on another stream beside the content-encoder calls. */
svc_status svc_f0_ac(svc_ctx* ctx, const float* wav24k, int B, int64_t n_samples, const int64_t* utt_samples, int T,
                     double* f0, void* stream);

/* F4: pYIN F0, utils/f0.py:95-117 get_f0_features_using_pyin(audio, fs, win_length, hop_length,
   f0_min, f0_max) = librosa.pyin with its defaults (frame_length 2048, centred frames, 100 beta(2, 18) thresholds,
   0.1-semitone bins, Viterbi decoding) and the unvoiced frames set to 0. wav [B][n_samples] f32 -> f0 [B*T] float64,
   utterance b's frames 1 + utt_samples[b] / hop_length, the rest of its T rows 0 (T >= 1 + n_samples / hop_length
   when every utterance is full length). Uses the feature-stage workspace, like svc_f0_ac; the context need not be
   finalized. Parity is unpinned (librosa is absent here): tests/test_f0.py holds it to oracle/pyin.py, which restates
   librosa 0.10.1 (its parabolic-interpolation shift and pyin's pad_mode="constant" default; librosa 0.9 / 0.10.0
   compute the parabolic shift differently, and the reference pins no librosa version). The device tables are built
   once per (fs, f0_min, f0_max, win_length, hop_length) and kept in the context. */
svc_status svc_f0_pyin(svc_ctx* ctx, const float* wav, int B, int64_t n_samples, const int64_t* utt_samples, double fs,
                       int win_length, int hop_length, double f0_min, double f0_max, int T, double* f0, void* stream);

/* A4: in place, f0 [B*T] float64 *= target_median / median(voiced f0 of that utterance)
   (utils/acoustic_feature_extraction.py:33-52; np.median semantics, NaN when no frame is voiced). */
svc_status svc_pitch_shift(svc_ctx* ctx, double* f0, int B, int T, double target_median, void* stream);

/* A5+A6: wav16k [B][n_samples] f32 (int16-quantised, <= 480000 samples; zero-padded to 30 s)
   -> Whisper encoder output feats [B*n_ctx][n_state] f32.
   Non-finite input: the attention kernel is compiled with -fno-honor-nans (its softmax max tree skips NaN
   canonicalisation), so a NaN reaching q / k / v gives undefined feats (possibly finite) instead of a propagated
   NaN. The log-mel front end and LayerNorm keep finite audio finite; a NaN / inf sample in wav16k is the caller's
   error. The same holds for svc_hubert_encode and svc_op_attention. */
svc_status svc_whisper_encode(svc_ctx* ctx, const float* wav16k, int B, int64_t n_samples, float* feats, void* stream);

/* A7: feats [B*src_rows][D] f32 -> content [B*T][D] f16 (IEEE binary16 bits), 15:8 repeat/average. T <= 2812. */
svc_status svc_map_content(svc_ctx* ctx, const float* feats, int B, int src_rows, int T, int D, void* content_f16,
                           void* stream);

/* A7/A8 mapping with an output row stride: feats [B*src_rows][D] f32 -> out f16 [B*T] rows of ld_out halves
   (columns 0..D-1 written; pass a column-offset pointer to fill one content type of a concatenated buffer).
   mode 0: Whisper rule (utils/whisper.py:31-81, T <= 2812, source truncated to T*8/15+1 rows);
   mode 1: HuBERT rule (utils/hubert.py:83-134, all src_rows frames, <= 3 missing rows repeat the last mapped
   row; |T - src_rows*15/8| > 3 is SVC_ERR_INVALID where the reference calls exit()). */
svc_status svc_map_content_ex(svc_ctx* ctx, const float* feats, int B, int src_rows, int T, int D, int mode,
                              void* out_f16, int ld_out, void* stream);

/* A8 (variant): HuBERT/ContentVec content encoder, replacing utils/hubert.py:31-47 get_hubert_content
   (fairseq HubertModel.extract_features(output_layer = config "hubert.output_layer", default 9) + final_proj).
   wav16k [B][n_samples] f32 (librosa-loaded 16 kHz float audio, utils/hubert.py:55) -> feats
   [B*svc_hubert_frames(n)][final_dim] f32. Parameters are added as "hubert." + fairseq state_dict keys. */
svc_status svc_hubert_encode(svc_ctx* ctx, const float* wav16k, int B, int64_t n_samples, float* feats, void* stream);
/* frames of the conv feature extractor for n samples (499 for 160 000) */
int64_t svc_hubert_frames(int64_t n_samples);
svc_status svc_hubert_dims(svc_ctx* ctx, int* final_dim, int* embed_dim);

/* A10: content f16 [B*T][D], f0 f64 [B*T], energy f32 [B*T], singer int32 [B] -> cond f32 [B*T][384].
   With several content types (config mapper.content_feature) D is the sum of their widths and the
   content columns are concatenated in ascending type-name order (e.g. contentvec | whisper); the
   per-type Linear layers (modules/encoder.py:144-148) are summed as one GEMM. */
svc_status svc_condition(svc_ctx* ctx, const void* content_f16, const double* f0, const float* energy,
                         const int32_t* singer, int B, int T, float* cond, void* stream);

/* A10's integer half, exported for bit-exact testing: the melody / loudness embedding indices the conditioner uses,
   torch.bucketize(f0 f64, melody bins f32) and torch.bucketize(energy f32, loudness bins f32) with right=False and
   torch's NaN placement (past the last bin) — modules/encoder.py:47-57,70 and :93-102,115. Bins are the context's
   (checkpoint) bins. f0 [n] f64, energy [n] f32 -> melody_idx, loudness_idx [n] int32 in [0, n_bins - 1]. */
svc_status svc_condition_indices(svc_ctx* ctx, const double* f0, const float* energy, int n, int32_t* melody_idx,
                                 int32_t* loudness_idx, void* stream);

/* A11+A12: cond f32 [B*T][384] -> x_0 f32 [B*T][n_mel] (normalised mel, time-major). frames: see Ragged batches.
   mode SVC_MODE_DDPM: `interval` ignored, 1000 steps; SVC_MODE_PLMS: reference speedup (e.g. 10).
   x_T f32 [B*T][n_mel] or NULL (then drawn on device from `seed` and `utt_ids`).
   noise (DDPM only) f32 [steps][B*T][n_mel] (already in time-major order) or NULL (device Philox noise keyed by
   `seed` and `utt_ids`). utt_ids int32 [B] may be NULL only when nothing is drawn on the device: x_T given and,
   for DDPM, `noise` given; otherwise a NULL utt_ids is SVC_ERR_INVALID. */
svc_status svc_diffsvc_sample(svc_ctx* ctx, const float* cond, int B, int T, const int32_t* frames, int mode,
                              int interval, const float* x_T, const float* noise, uint64_t seed,
                              const int32_t* utt_ids, float* x0, void* stream);

/* single epsilon prediction (DiffSVC.forward, modules/diffsvc.py:284-321) for testing: x f32 [B*T][n_mel], step t */
svc_status svc_diffsvc_eps(svc_ctx* ctx, const float* cond, const float* x, int B, int T, const int32_t* frames, int t,
                           float* eps, void* stream);

/* A13+A14+A15: x0 f32 [B*T][n_mel] (normalised) -> wav [B][T*256] f32 (denorm, Generator, tanh, fade-out).
   frames (host int32 [B] or NULL): ragged batch, utterance b's waveform is frames[b]*256 samples (fade-out at its end,
   zeros after).
   mel_denorm_out (optional, f32 [B*T][n_mel]) receives the de-normalised mel. */
svc_status svc_bigvgan(svc_ctx* ctx, const float* x0, int B, int T, const int32_t* frames, float* wav,
                       float* mel_denorm_out, void* stream);

/* ---------------- op-level entry points (used by the parity tests; weights are unpacked f32 device arrays) */
/* y[B*T_out][Cout] = conv1d(x[B*T_in][Cin]) ; w [Cout][Cin][k] ; act 0 none / 1 gelu / 2 relu */
svc_status svc_op_conv1d(const float* x, int B, int T_in, int Cin, const float* w, const float* bias, int Cout, int k,
                         int stride, int dilation, int pad, int act, float* y, void* stream);
/* ConvTranspose1d, w [Cin][Cout][k]; T_out = (T_in-1)*stride - 2*pad + k */
svc_status svc_op_conv_transpose1d(const float* x, int B, int T_in, int Cin, const float* w, const float* bias,
                                   int Cout, int k, int stride, int pad, float* y, void* stream);
/* Rational-ratio resampler (F1; replaces librosa.resample in utils/audio.py:49-53 and ffmpeg's 16 kHz decode in
 * utils/whisper_extractor/audio.py:41-49). x f32 [B][n_in] -> y f32 [B][svc_resample_len(n_in, sr_in, sr_out)],
 * scipy.signal.resample_poly's Kaiser(5) polyphase FIR; quantize16 = 1 rounds to int16 / 32768 (s16le decode). */
int64_t svc_resample_len(int64_t n_in, int sr_in, int sr_out);
svc_status svc_resample(const float* x, int B, int64_t n_in, int sr_in, int sr_out, int quantize16, float* y,
                        void* stream);
/* host-only: the designed taps (cap >= *n, or h = NULL to query *n) and the plan's up/down/pre_remove */
svc_status svc_resample_filter(int sr_in, int sr_out, double* h, int cap, int* n, int* up, int* down,
                               int* pre_remove);
/* BigVGAN AMP step for small channel counts: y = conv_k,d(Activation1d(x)) + bias (+ add_row), fused.
 * x, add_row, y f32 [B*L][C] time-major; w f32 [C][C][k] (effective weight); C in {24, 48, 96}.
 * Replaces modules/bigvgan.py:427-431 (a1/c1, a2/c2 pairs) for the late generator stages. */
svc_status svc_op_amp_conv(const float* x, int B, int L, int C, const float* alpha_log, const float* beta_log,
                           const float* filt, const float* w, const float* bias, int k, int d, const float* add_row,
                           float* y, void* stream);
/* Activation1d(SnakeBeta, logscale): x f32 [B*L][C] -> y f32 [B*L][C] */
svc_status svc_op_activation1d(const float* x, int B, int L, int C, const float* alpha_log, const float* beta_log,
                               const float* filt12, float* y, void* stream);
/* the same on an f16 input x16 [B*L][C] (binary16; the AMPBlock1 convs1 outputs in the product path) */
svc_status svc_op_activation1d_x16(const void* x16, int B, int L, int C, const float* alpha_log, const float* beta_log,
                                   const float* filt12, float* y, void* stream);
/* attention on f32 q,k,v [B*L][D] (already projected; scaled inside by dh^-1/4 each) -> out f32 [B*L][D] */
svc_status svc_op_attention(const float* q, const float* k, const float* v, int B, int L, int D, float* out,
                            void* stream);
svc_status svc_op_layernorm(const float* x, const float* g, const float* b, int rows, int D, float* y, void* stream);
/* live per-kernel timing: enable(1) clears and starts recording (hipEvents around each launch),
   read(idx, ...) synchronises and returns kernel idx's name, total ms, launches, algorithmic FLOPs/bytes;
   n_kernels receives the number of distinct kernels. */
svc_status svc_profile_enable(int enable);
/* Restrict live profiling to kernels whose name starts with kernel_prefix ("" or NULL = all): bench.py times
 * only the dominant kernel in its timed region, so the other ~4 000 launches per step carry no events. */
svc_status svc_profile_filter(const char* kernel_prefix);
svc_status svc_profile_read(int idx, char* name, int name_len, double* total_ms, int64_t* launches, double* flops,
                            double* bytes, int* n_kernels);
/* GEMM microbenchmark on synthetic operands: average ms per launch of one implicit-GEMM configuration
   (10-14 = conv_gemm3 tiles, 15 = the production choice, 20 / 24 = conv_gemm4 with the LDS-staged / register
   gate epilogue; see run_gemm in engine.hip); epi 0 = f16 store, 1 = paired gate, 2 / 6 = f32 / split-fp16 residual
   read-modify-write, 3-5 = gate diagnostics (variant 24: 3 no cp read and no store, 4 no cp read, 5 no store);
   iters < 0: |iters| launches, each after a 1 GiB memset (operands evicted from the caches) */
svc_status svc_gemm_bench(int M, int N, int Cin, int taps, int epi, int variant, int iters, double* ms_out);
/* slaney mel filterbank (librosa.filters.mel, htk=False, norm='slaney') computed natively, host output */
svc_status svc_mel_filterbank(int sr, int n_fft, int n_mels, double fmin, double fmax, float* out_host);

#ifdef __cplusplus
}
#endif
#endif
