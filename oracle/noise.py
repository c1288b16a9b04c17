"""ORACLE (test infrastructure only) — deterministic inputs shared by the golden generator and tests.

Synthetic clips follow SURVEY.md §8(d): a voiced harmonic tone (f0 in [110, 440] Hz, 5.5 Hz vibrato
±3 %, 8 harmonics with amplitude 1/h, peak 0.3) with ~10 % unvoiced gaps, generated analytically at
24 kHz (f32) and 16 kHz (int16-quantised /32768, utils/whisper_extractor/audio.py:41-49) from the same
continuous-time formula, so no resampler is involved.

Sampler noise replaces the reference's unseeded torch RNG (modules/diffsvcrepo_inference.py:22-27,
208-214): x_T ~ N(0, (1/1.2)^2) in [B,T,100] and per-step z ~ N(0,1) drawn in the reference's
[B,1,100,T] order and handed over transposed to [B,T,100].
"""
import numpy as np


def _rng(seed, tag):
    return np.random.Generator(np.random.PCG64([int(seed) & 0xFFFFFFFF, tag]))


from svc_inference_pipeline_amd.synth import clip_params, synth_clip, synth_clip_16k_quantised  # noqa: E402,F401


def x_T(seed, B, T, n_mel=100):
    return (_rng(seed, 3).standard_normal((B, T, n_mel), dtype=np.float32) * np.float32(1 / 1.2)).astype(np.float32)


def step_noise(seed, i, B, T, n_mel=100):
    """z for DDPM step i, reference order [B,1,n_mel,T] -> returned [B,T,n_mel]."""
    z = _rng(seed, 1000 + i).standard_normal((B, 1, n_mel, T), dtype=np.float32)
    return np.ascontiguousarray(z[:, 0].transpose(0, 2, 1))


def synth_f0(seed, T, voiced_frac=0.85):
    """Synthetic f0 contour (f64) with unvoiced zeros, for conditioner tests."""
    r = _rng(seed, 4)
    f0 = 220.0 * np.exp(0.3 * np.sin(np.arange(T) / 17.0)) * (1 + 0.01 * r.standard_normal(T))
    f0[r.uniform(size=T) > voiced_frac] = 0.0
    return f0.astype(np.float64)
