"""The north-star tolerance check shared by tests/test_gpu_headline.py and tests/test_gpu_configs.py: one clip through
SVCPipeline.convert with DDPM-1000 and shared x_T / per-step noise (oracle/noise.py), against the fp32 oracle's
chain; the metric is the mean |delta| of the de-normalised natural-log mel (utils/acoustic_feature_extraction.py:83-97,
the sampler's output as modules/diffsvcrepo_inference.py:233-235 returns it, de-normalised)."""
import numpy as np
import torch

from gpu_util import dev
from oracle import features as OF
from oracle import models as OM
from oracle import noise as ON
from oracle import pipeline as OP
from svc_inference_pipeline_amd import config as C
from svc_inference_pipeline_amd import weights as W
from svc_inference_pipeline_amd.pipeline import SVCPipeline

MEL_L1_TARGET = 1e-3   # BASELINE.json north_star: "<= 1e-3 mel-L1 vs the CPU reference"
SEED = 17


def clip(content, seconds):
    """(24 kHz wav, 16 kHz wav, T, synthetic F0, x_T) of the test clip"""
    w24 = ON.synth_clip(7, seconds, 24000).astype(np.float32)
    if content == "whisper":
        w16 = ON.synth_clip_16k_quantised(7, seconds)
    else:
        w16 = ON.synth_clip(7, seconds, 16000).astype(np.float32)
    T = OF.mel_frames(len(w24))
    return w24, w16, T, ON.synth_f0(4, T), ON.x_T(SEED, 1, T)


def gpu_mel(engine, content, seconds):
    """the de-normalised ln-mel [n_mel, T] of the GPU conversion (the engine's precision mode)"""
    w24, w16, T, f0, xT = clip(content, seconds)
    noise = dev(np.stack([ON.step_noise(SEED, i, 1, T) for i in reversed(range(1000))]))
    res = SVCPipeline(engine).convert(dev(w24[None]), dev(w16[None]), dev(np.array([2]), torch.int32),
                                      fast_inference=False, x_T=dev(xT), noise=noise,
                                      f0=dev(f0[None], torch.float64),
                                      wav16_float=dev(w16[None]) if content != "whisper" else None)
    _, mel = engine.bigvgan(res.x0, return_mel=True)
    assert bool(torch.isfinite(res.wav).all())
    return mel[0].cpu().numpy().T


def oracle_mel(cfg, states, content, seconds, operand_dtype=None):
    """the oracle's de-normalised ln-mel [n_mel, T]: fp32, or with every conv / linear / attention matmul rounding its
    operands to `operand_dtype` (oracle.models.OperandRounding, fp32 accumulation)"""
    stats = C.load_stats(cfg)
    w24, w16, T, f0, xT = clip(content, seconds)
    ms = states["mapper"]
    rounding = OM.OperandRounding(operand_dtype, linear=True) if operand_dtype is not None else None
    if rounding:
        rounding.__enter__()
    try:
        with torch.no_grad():
            mel = OF.mel_spectrogram(torch.from_numpy(w24)[None], cfg)
            en = OF.energy_from_mel(mel)
            f0s = torch.from_numpy(OF.pitch_shift(f0, stats["target_f0_median"]))[None]
            if content == "whisper":
                feats = OP.whisper_content(states["whisper"], w16, T)
            else:
                feats = OP.hubert_content(states["hubert"], w16, T)
            feats = torch.from_numpy(np.asarray(feats, np.float32))[None]
            cond = OM.conditioner(ms, {content: feats}, f0s, en, torch.tensor([[2]]))
            table = W.step_embedding_table(1000)
            consts = OM.schedule_constants(C.noise_schedule(cfg.mapper))
            cache = {}  # the conditioner projections of `cond`, computed once (bit-identical, ~40 % of each call)
            den = lambda x, t: OM.diffsvc_forward(ms, cfg.mapper, x, cond, t, table, cache)  # noqa: E731
            x0 = OM.sample_ddpm(den, torch.from_numpy(xT), 1, T, 1000, consts,
                                lambda i: torch.from_numpy(ON.step_noise(SEED, i, 1, T)))
    finally:
        if rounding:
            rounding.__exit__(None, None, None)
    return OF.denormalize_mel_channel(x0[0].numpy().T, stats["mel_min"], stats["mel_max"])


def ddpm1000_mel_l1(engine, cfg, states, content, seconds):
    """content "whisper" (states["whisper"], int16-quantised 16 kHz input) or "contentvec" (states["hubert"], float
    16 kHz input). Returns the mel-L1 of the GPU conversion against the fp32 oracle (default precision mode of
    `engine`)."""
    g = gpu_mel(engine, content, seconds)
    ref = oracle_mel(cfg, states, content, seconds)
    assert g.shape == ref.shape == (cfg.mapper.n_mel, g.shape[1])
    return float(np.mean(np.abs(g - ref)))
