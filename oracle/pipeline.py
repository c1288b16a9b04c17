"""ORACLE (test infrastructure only) — the whole infer.py path on the CPU (torch-CPU fp32 / numpy f64),
one utterance: the CPU baseline `bench.py` times, and the end-to-end reference for parity tests.

infer.py:53 features -> :59 pitch shift -> :64 Whisper (or :65 ContentVec) content -> :79 DiffSVC sampler ->
:80 de-normalisation -> :86 BigVGAN synthesis (fade). Pitch: oracle.praat_ac (parity unpinned).
"""
import numpy as np
import torch

from svc_inference_pipeline_amd import config as C
from svc_inference_pipeline_amd import weights as W

from . import features as OF
from . import models as OM
from . import noise as ON
from . import praat_ac as PA


WHISPER_WINDOW = 478720      # svc_inference_pipeline_amd/pipeline.py: 29.92 s windows for T > 2812
WINDOW_MEL_FRAMES = 2805


def whisper_content(ws, wav16, T):
    """utils/whisper.py:22-81 for one utterance -> f32 [T, D]. Up to 2812 frames this is exactly the
    reference's path; longer clips (where the reference raises) are encoded per 29.92 s window, each
    padded to Whisper's 30 s context and mapped 15:8 onto its 2805 mel frames."""
    dims = W.whisper_dims_from_state(ws)
    wav16 = np.asarray(wav16, np.float32)

    def enc(w):
        lm = OF.whisper_log_mel(torch.from_numpy(OF.pad_or_trim(w))[None])
        return OM.whisper_encoder(ws, lm, dims["n_audio_head"])[0].numpy()

    if T <= 2812:
        return OF.map_whisper_features(enc(wav16), T)
    parts = []
    for c in range(-(-T // WINDOW_MEL_FRAMES)):
        tl = min(WINDOW_MEL_FRAMES, T - c * WINDOW_MEL_FRAMES)
        parts.append(OF.map_whisper_features(enc(wav16[c * WHISPER_WINDOW:(c + 1) * WHISPER_WINDOW]), tl))
    return np.concatenate(parts, 0)


def hubert_content(hs, wav16, T, output_layer=9):
    """utils/hubert.py:137-143 (contentVec_feature_extractor) for one utterance -> f32 [T, final_dim]."""
    feats = OM.hubert_content(hs, torch.from_numpy(np.asarray(wav16, np.float32))[None], output_layer)[0].numpy()
    return OF.map_hubert_features(feats, T)


def convert(cfg, ws, ms, vs, wav24, wav16, singer, speedup=10, seed=0, fast_inference=True, x_T=None, f0=None,
            hs=None, wav16_float=None, hubert_output_layer=9):
    """Returns dict(wav f32[T*hop], mel, f0, x0). Content types follow cfg.mapper.content_feature: "whisper"
    uses ws on wav16, "contentvec" uses the HuBERT state hs on wav16_float (default wav16)."""
    mel = OF.mel_spectrogram(torch.from_numpy(np.asarray(wav24, np.float32))[None], cfg)  # [1,100,T]
    energy = OF.energy_from_mel(mel)
    T = mel.shape[-1]
    if f0 is None:
        f0 = PA.f0_features(wav24, T, fs=cfg.fs, hop=cfg.hop_length, floor=cfg.f0_min, ceiling=cfg.f0_max)
    f0 = OF.pitch_shift(f0, C.load_stats(cfg)["target_f0_median"])
    content = {}
    for ct in cfg.mapper.content_feature:
        if ct == "whisper":
            c = whisper_content(ws, wav16, T)
        else:
            c = hubert_content(hs, wav16 if wav16_float is None else wav16_float, T, hubert_output_layer)
        content[ct] = torch.from_numpy(np.asarray(c, np.float32))[None]
    cond = OM.conditioner(ms, content, torch.from_numpy(f0)[None], energy, torch.tensor([[int(singer)]]))
    table = W.step_embedding_table(len(C.noise_schedule(cfg.mapper)))
    consts = OM.schedule_constants(C.noise_schedule(cfg.mapper))
    den = lambda x, t: OM.diffsvc_forward(ms, cfg.mapper, x, cond, t, table)
    xT = torch.from_numpy(ON.x_T(seed, 1, T) if x_T is None else np.asarray(x_T, np.float32))
    steps = len(C.noise_schedule(cfg.mapper))
    if fast_inference:
        x0 = OM.sample_plms(den, xT, 1, T, steps, speedup, consts)
    else:
        x0 = OM.sample_ddpm(den, xT, 1, T, steps, consts, lambda i: torch.from_numpy(ON.step_noise(seed, i, 1, T)))
    stats = C.load_stats(cfg)
    mel_d = OF.denormalize_mel_channel(x0[0].numpy().T, stats["mel_min"], stats["mel_max"]).astype(np.float32)
    wav = OM.bigvgan_forward(vs, cfg.vocoder, torch.from_numpy(mel_d)[None])
    wav = OF.synthesis_fade(wav[0, 0], T)
    return {"wav": wav.numpy(), "mel": mel[0].numpy(), "f0": f0, "x0": x0[0].numpy()}
