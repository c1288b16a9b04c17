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


def clip_params(k):
    r = _rng(k, 1)
    return dict(f0=float(r.uniform(110.0, 440.0)), phase=float(r.uniform(0, 2 * np.pi)),
                gap_start=float(r.uniform(0.2, 0.7)))


def synth_clip(k, seconds, fs):
    """Continuous-time tone sampled at fs; returns f32[round(seconds*fs)]."""
    p = clip_params(k)
    n = int(round(seconds * fs))
    t = np.arange(n, dtype=np.float64) / fs
    f0 = p["f0"] * (1.0 + 0.03 * np.sin(2 * np.pi * 5.5 * t))
    phase = 2 * np.pi * np.cumsum(f0) / fs + p["phase"]
    y = np.zeros(n)
    for h in range(1, 9):
        y += np.sin(h * phase) / h
    # ~10% unvoiced gap: replace by low-level deterministic noise
    g0, g1 = p["gap_start"] * seconds, p["gap_start"] * seconds + 0.1 * seconds
    gap = (t >= g0) & (t < g1)
    y[gap] = 0.02 * _rng(k, 2).standard_normal(int(gap.sum()))
    # raised-cosine 5 ms edges so the edges are not silent but not clicking
    y *= 0.3 / np.max(np.abs(y))
    return y.astype(np.float32)


def synth_clip_16k_quantised(k, seconds):
    y = synth_clip(k, seconds, 16000).astype(np.float64)
    q = np.clip(np.round(y * 32768.0), -32768, 32767).astype(np.int16)
    return q.astype(np.float32) / 32768.0


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
