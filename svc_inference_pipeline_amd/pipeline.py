"""Batched counterpart of the reference's infer.py (infer.py:44-90), on one GPU.

    mel, energy = acoutic_feature_extractor(...)        infer.py:53   -> SVCEngine.mel_energy + f0
    f0 = pitch_shift(f0, cfg)                           infer.py:59   -> SVCEngine.pitch_shift
    whisper_feature = whisper_feature_extractor(...)    infer.py:64   -> whisper_encode + map_content
    contentVec_feature = contentVec_feature_extractor   infer.py:65   -> hubert_encode + map_content(rule="hubert")
    y_pred = svc_model_inference(...)                   infer.py:79   -> condition + diffsvc_sample
    y_pred = denormalize_mel_channel(y_pred, cfg)       infer.py:80   -> fused into bigvgan
    audio = synthesis_audios(...)                       infer.py:86   -> bigvgan (Generator, trim, fade)

Inputs are device tensors of B equal-length utterances (24 kHz f32 and the 16 kHz int16-quantised
copy Whisper consumes); every stage runs in libsvc_hip.so on the current stream.

Long inputs (SURVEY.md §5 "Long-context", BASELINE config 4). The reference pads/trims Whisper's input
to one 30 s window and caps the mapped content at 2812 frames (utils/whisper.py:52-56), so for clips
longer than ~29.99 s its `torch.cat` in modules/encoder.py:197 raises. Here, when T > 2812, Whisper runs
on consecutive windows of 478 720 samples (29.92 s = 1496 encoder frames = exactly 2805 mel frames, so
the 15:8 map stays integral and every window starts on a mel frame). Each window is encoded in its own
zero-padded 30 s context and mapped with the reference's own 15:8 rule. Parity for such clips is per
window (tests/test_gpu_long.py). Mel, F0, the sampler and BigVGAN run over the whole length in one pass:
a 180 s song needs ~0.4 GB per vocoder stage buffer, far below 288 GB of HBM, so the vocoder needs no
overlap-add seams.
"""
from dataclasses import dataclass

import torch

from .runtime import SVCEngine, mel_frames

WHISPER_WINDOW = 478720       # 16 kHz samples per long-input window (29.92 s)
WINDOW_MEL_FRAMES = 2805      # = 1496 encoder frames * 15 / 8
MAX_MAPPED = 2812             # utils/whisper.py:56 (1500 * 15 // 8)
HUBERT_CONTENT_TYPES = ("contentvec", "content_vector", "hubert")  # config/config.json:35 names it content_vector


@dataclass
class ConvertResult:
    wav: torch.Tensor        # f32 [B, T*hop] converted audio (before save_audio's peak normalisation)
    mel: torch.Tensor        # f32 [B, T, n_mels] source log-mel
    f0: torch.Tensor         # f64 [B, T] pitch-shifted F0
    x0: torch.Tensor         # f32 [B, T, n_mel] normalised mel from the sampler


class SVCPipeline:
    def __init__(self, engine: SVCEngine, f0_side=True, f0_method="parselmouth"):
        """f0_side: run the 24 kHz features (mel / energy, F0, pitch shift) on the context's sub-stream 2 beside the
        content encoder (default; measured +0.4 %) instead of on the caller's stream.
        f0_method: "parselmouth" (utils/f0.py:120-161, what utils/acoustic_feature_extraction.py:53 uses) or "pyin"
        (utils/f0.py:95-117 get_f0_features_using_pyin, svc_f0_pyin; its 1 + N // hop frames cut to the mel frames)."""
        if f0_method not in ("parselmouth", "pyin"):
            raise ValueError(f"f0_method {f0_method!r}: 'parselmouth' or 'pyin'")
        self.engine = engine
        self.f0_side = f0_side
        self.f0_method = f0_method

    def extract_f0(self, wav24, T, n_samples=None, T_b=None):
        """F0 by the configured method -> f64 [B, T] (rows past an utterance's T_b frames 0)."""
        e = self.engine
        if self.f0_method == "parselmouth":
            return e.f0(wav24, T, n_samples=n_samples)
        N = wav24.shape[1]
        f0 = e.f0_pyin(wav24, n_samples=n_samples, T=max(T, 1 + N // e.cfg.hop_length))[:, :T].contiguous()
        if T_b is not None:
            for b, tb in enumerate(T_b):
                f0[b, tb:] = 0
        return f0

    def content(self, wav16, T, wav16_float=None):
        """Content features of every type in cfg.mapper.content_feature mapped to T mel frames -> [B, T, sum of
        widths] in the engine's content_dtype (f16, or bf16 with operands="bf16"), the types' columns concatenated in ascending name order (the order in which the
        native conditioner packs their ContentEncoder Linears). "whisper" runs Whisper on the int16-quantised
        16 kHz audio (utils/whisper.py:96-103); "contentvec" runs HuBERT/ContentVec on float 16 kHz audio
        (utils/hubert.py:137-143; `wav16_float`, defaulting to wav16)."""
        e = self.engine
        m = e.cfg.mapper
        types = sorted(m.content_feature)
        if types == ["whisper"]:
            return self.whisper_content(wav16, T)
        widths = [int(m.input_content_dim[t]) for t in types]
        B = wav16.shape[0]
        out = torch.empty(B, T, sum(widths), device=wav16.device, dtype=e.content_dtype)
        col = 0
        for t, w in zip(types, widths):
            view = out[:, :, col:col + w]
            if t == "whisper":
                view.copy_(self.whisper_content(wav16, T))
            elif t in HUBERT_CONTENT_TYPES:
                feats = e.hubert_encode(wav16 if wav16_float is None else wav16_float)
                e.map_content(feats, T, rule="hubert", out=view)
            else:
                raise ValueError(f"content feature {t!r} is not supported (whisper, {', '.join(HUBERT_CONTENT_TYPES)})")
            col += w
        return out

    def whisper_content(self, wav16, T):
        """Whisper content features mapped to T mel frames -> f16 [B, T, D]."""
        e = self.engine
        B = wav16.shape[0]
        if T <= MAX_MAPPED:
            return e.map_content(e.whisper_encode(wav16), T)
        n_win = -(-T // WINDOW_MEL_FRAMES)
        need = n_win * WHISPER_WINDOW
        w = wav16
        if w.shape[1] < need:
            w = torch.nn.functional.pad(w, (0, need - w.shape[1]))
        wins = w[:, :need].reshape(B * n_win, WHISPER_WINDOW).contiguous()
        feats = e.whisper_encode(wins)                      # [B*n_win, 1500, D]
        D = feats.shape[-1]
        out = torch.empty(B, n_win * WINDOW_MEL_FRAMES, D, device=wav16.device, dtype=e.content_dtype)
        full = e.map_content(feats, WINDOW_MEL_FRAMES)     # every window mapped to 2805 frames
        out.copy_(full.view(B, n_win * WINDOW_MEL_FRAMES, D))
        return out[:, :T].contiguous()

    def _side_stream(self, device):
        if getattr(self, "_side", None) is None:
            self._side = self.engine.aux_stream(2)  # the context's own stream: no extra hardware-queue pressure
        return self._side

    def convert(self, wav24, wav16, singer, fast_inference=True, speedup=10, seed=0, utt_ids=None, x_T=None,
                noise=None, f0=None, wav16_float=None):
        """infer.py's sequence for B equal-length clips -> ConvertResult. `f0` (optional, f64 [B, T]) replaces the
        Praat extraction; it is pitch-shifted on a copy (the caller's tensor is not modified)."""
        with self.engine.lock:
            return self._convert(wav24, wav16, singer, fast_inference, speedup, seed, utt_ids, x_T, noise, f0,
                                 wav16_float)

    def _convert(self, wav24, wav16, singer, fast_inference, speedup, seed, utt_ids, x_T, noise, f0, wav16_float):
        e = self.engine
        T = mel_frames(wav24.shape[1], e.cfg.n_fft, e.cfg.hop_length)  # utils/mel.py:130-174 frame count
        # The 24 kHz features (mel / energy, and F0: Praat AC + pitch shift, latency-bound serial work on few CUs)
        # run on the context's sub-stream 2 beside the content encoder (they use their own workspace), joined before
        # the conditioner needs them
        main = torch.cuda.current_stream(wav24.device)
        side = self._side_stream(wav24.device) if self.f0_side else main
        side.wait_stream(main)
        with torch.cuda.stream(side):
            mel, energy = e.mel_energy(wav24)
            # a caller-supplied f0 is shifted on a copy (svc_pitch_shift works in place)
            f0 = self.extract_f0(wav24, T) if f0 is None else f0.to(torch.float64).contiguous().clone()
            e.pitch_shift(f0)
        assert mel.shape[1] == T
        content = self.content(wav16, T, wav16_float)
        main.wait_stream(side)
        for t in (mel, energy, f0):
            t.record_stream(main)
        cond = e.condition(content, f0, energy, singer)
        if utt_ids is None and x_T is None:
            utt_ids = torch.arange(wav24.shape[0], device=wav24.device, dtype=torch.int32)
        x0 = e.diffsvc_sample(cond, fast_inference=fast_inference, speedup=speedup, x_T=x_T, noise=noise, seed=seed,
                              utt_ids=utt_ids)
        wav = e.bigvgan(x0)
        return ConvertResult(wav=wav, mel=mel, f0=f0, x0=x0)

    def convert_many(self, wavs24, wavs16, singers, wavs16_float=None, fast_inference=True, speedup=10, seed=0,
                     utt_ids=None, bucketed=False):
        """Ragged requests: lists of per-utterance device tensors (24 kHz f32 [N_i],
        16 kHz [N16_i], optional float 16 kHz for ContentVec) and singer ids -> list of waveforms f32 [T_i*hop] in
        input order, each bit-identical to converting that clip alone with the same utterance id
        (tests/test_gpu_ragged.py). utt_ids (default: list positions) key the device noise, as in convert().

        Default: ONE padded batch with per-utterance lengths (convert_ragged): every kernel that looks across time
        (STFT, Praat frames, convolutions, anti-aliased activations, fade-out) stops at each utterance's own end.
        bucketed=True instead runs one batch per distinct length."""
        n = len(wavs24)
        if not (len(wavs16) == n == len(singers)) or (wavs16_float is not None and len(wavs16_float) != n):
            raise ValueError("convert_many: wavs24, wavs16, singers (and wavs16_float) must have one entry per utterance")
        ids = list(range(n)) if utt_ids is None else [int(u) for u in utt_ids]
        if not bucketed:
            return self.convert_ragged(wavs24, wavs16, singers, wavs16_float=wavs16_float,
                                       fast_inference=fast_inference, speedup=speedup, seed=seed, utt_ids=ids)
        buckets = {}
        for i in range(n):
            key = (int(wavs24[i].shape[-1]), int(wavs16[i].shape[-1]),
                   int(wavs16_float[i].shape[-1]) if wavs16_float is not None else 0)
            buckets.setdefault(key, []).append(i)
        out = [None] * n
        dev = wavs24[0].device
        for key in sorted(buckets):
            idx = buckets[key]
            w24 = torch.stack([wavs24[i].reshape(-1) for i in idx]).contiguous()
            w16 = torch.stack([wavs16[i].reshape(-1) for i in idx]).contiguous()
            w16f = torch.stack([wavs16_float[i].reshape(-1) for i in idx]).contiguous() if wavs16_float is not None else None
            sing = torch.tensor([int(singers[i]) for i in idx], device=dev, dtype=torch.int32)
            uid = torch.tensor([ids[i] for i in idx], device=dev, dtype=torch.int32)
            res = self.convert(w24, w16, sing, fast_inference=fast_inference, speedup=speedup, seed=seed,
                               utt_ids=uid, wav16_float=w16f)
            for j, i in enumerate(idx):
                out[i] = res.wav[j]
        return out

    @staticmethod
    def _pad_stack(tensors):
        """list of 1-D device tensors -> zero-padded [B, max_len] and the host lengths"""
        lens = [int(t.shape[-1]) for t in tensors]
        out = torch.zeros(len(tensors), max(lens), dtype=tensors[0].dtype, device=tensors[0].device)
        for i, t in enumerate(tensors):
            out[i, :lens[i]] = t.reshape(-1)
        return out, lens

    def ragged_content(self, wavs16, T_b, T, wavs16_float=None):
        """Content features for a ragged batch -> f16 [B, T, D]; rows [b, :T_b[b]] equal convert()'s for that clip
        alone. Whisper runs on zero-padded 16 kHz audio (pad_or_trim pads with zeros, so the padding is exact), in two
        groups: clips the reference maps in one 30 s window (T_b <= 2812) and long clips (per-window, see
        whisper_content). HuBERT / ContentVec attends over every frame and normalises over time, so it runs per
        exact-length bucket."""
        e = self.engine
        m = e.cfg.mapper
        types = sorted(m.content_feature)
        widths = [int(m.input_content_dim[t]) for t in types]
        B = len(wavs16)
        dev = wavs16[0].device
        out = torch.zeros(B, T, sum(widths), device=dev, dtype=e.content_dtype)
        col = 0
        for t, w in zip(types, widths):
            if t == "whisper":
                for group in ([i for i in range(B) if T_b[i] <= MAX_MAPPED], [i for i in range(B) if T_b[i] > MAX_MAPPED]):
                    if not group:
                        continue
                    w16, _ = self._pad_stack([wavs16[i] for i in group])
                    Tg = max(T_b[i] for i in group)
                    c = self.whisper_content(w16, Tg)
                    for j, i in enumerate(group):
                        out[i, :T_b[i], col:col + w] = c[j, :T_b[i]]
            elif t in HUBERT_CONTENT_TYPES:
                src = wavs16 if wavs16_float is None else wavs16_float
                buckets = {}
                for i in range(B):
                    buckets.setdefault((int(src[i].shape[-1]), T_b[i]), []).append(i)
                for (_, tb), idx in sorted(buckets.items()):
                    feats = e.hubert_encode(torch.stack([src[i].reshape(-1) for i in idx]).contiguous())
                    c = e.map_content(feats, tb, rule="hubert")
                    for j, i in enumerate(idx):
                        out[i, :tb, col:col + w] = c[j]
            else:
                raise ValueError(f"content feature {t!r} is not supported (whisper, {', '.join(HUBERT_CONTENT_TYPES)})")
            col += w
        return out

    def convert_ragged(self, wavs24, wavs16, singers, wavs16_float=None, fast_inference=True, speedup=10, seed=0,
                       utt_ids=None):
        """infer.py's sequence for B clips of different lengths as ONE padded batch: the C-ABI stages take the
        per-utterance lengths (include/svc_hip.h, "Ragged batches") and compute each clip exactly as alone.
        -> list of waveforms f32 [T_b * hop]."""
        with self.engine.lock:
            return self._convert_ragged(wavs24, wavs16, singers, wavs16_float, fast_inference, speedup, seed, utt_ids)

    def _convert_ragged(self, wavs24, wavs16, singers, wavs16_float, fast_inference, speedup, seed, utt_ids):
        e = self.engine
        n = len(wavs24)
        ids = list(range(n)) if utt_ids is None else [int(u) for u in utt_ids]
        w24, n24 = self._pad_stack(wavs24)
        dev = w24.device
        T_b = [mel_frames(k, e.cfg.n_fft, e.cfg.hop_length) for k in n24]
        T = max(T_b)
        main = torch.cuda.current_stream(dev)
        side = self._side_stream(dev) if self.f0_side else main
        side.wait_stream(main)
        with torch.cuda.stream(side):
            mel, energy = e.mel_energy(w24, n_samples=n24)
            f0 = self.extract_f0(w24, T, n_samples=n24, T_b=T_b)
            e.pitch_shift(f0)
        content = self.ragged_content(list(wavs16), T_b, T, wavs16_float)
        main.wait_stream(side)
        for t in (mel, energy, f0):
            if t.is_cuda:
                t.record_stream(main)
        sing = torch.tensor([int(s) for s in singers], device=dev, dtype=torch.int32)
        cond = e.condition(content, f0, energy, sing)
        uid = torch.tensor(ids, device=dev, dtype=torch.int32)
        x0 = e.diffsvc_sample(cond, fast_inference=fast_inference, speedup=speedup, seed=seed, utt_ids=uid, frames=T_b)
        wav = e.bigvgan(x0, frames=T_b)
        hop = e.cfg.hop_length
        return [wav[i, :T_b[i] * hop] for i in range(n)]
