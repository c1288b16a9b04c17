"""Batched counterpart of the reference's infer.py (infer.py:44-90), on one GPU.

    mel, energy = acoutic_feature_extractor(...)        infer.py:53   -> SVCEngine.mel_energy + f0
    f0 = pitch_shift(f0, cfg)                           infer.py:59   -> SVCEngine.pitch_shift
    whisper_feature = whisper_feature_extractor(...)    infer.py:64   -> whisper_encode + map_content
    y_pred = svc_model_inference(...)                   infer.py:79   -> condition + diffsvc_sample
    y_pred = denormalize_mel_channel(y_pred, cfg)       infer.py:80   -> fused into bigvgan
    audio = synthesis_audios(...)                       infer.py:86   -> bigvgan (Generator, trim, fade)

Inputs are device tensors of B equal-length utterances (24 kHz f32 and the 16 kHz int16-quantised
copy Whisper consumes); every stage runs in libsvc_hip.so on the current stream.
"""
from dataclasses import dataclass

import torch

from .runtime import SVCEngine


@dataclass
class ConvertResult:
    wav: torch.Tensor        # f32 [B, T*hop] converted audio (before save_audio's peak normalisation)
    mel: torch.Tensor        # f32 [B, T, n_mels] source log-mel
    f0: torch.Tensor         # f64 [B, T] pitch-shifted F0
    x0: torch.Tensor         # f32 [B, T, n_mel] normalised mel from the sampler


class SVCPipeline:
    def __init__(self, engine: SVCEngine):
        self.engine = engine

    def convert(self, wav24, wav16, singer, fast_inference=True, speedup=10, seed=0, utt_ids=None, x_T=None,
                noise=None, f0=None):
        e = self.engine
        mel, energy = e.mel_energy(wav24)
        T = mel.shape[1]
        if f0 is None:
            f0 = e.f0(wav24, T)
        e.pitch_shift(f0)
        feats = e.whisper_encode(wav16)
        content = e.map_content(feats, T)
        cond = e.condition(content, f0, energy, singer)
        if utt_ids is None and x_T is None:
            utt_ids = torch.arange(wav24.shape[0], device=wav24.device, dtype=torch.int32)
        x0 = e.diffsvc_sample(cond, fast_inference=fast_inference, speedup=speedup, x_T=x_T, noise=noise, seed=seed,
                              utt_ids=utt_ids)
        wav = e.bigvgan(x0)
        return ConvertResult(wav=wav, mel=mel, f0=f0, x0=x0)
