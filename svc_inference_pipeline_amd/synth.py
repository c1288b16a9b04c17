"""Synthetic singing-like input clips for benchmarks and tests.

A voiced harmonic tone (f0 uniform in [110, 440] Hz, 5.5 Hz vibrato +-3 %, 8 harmonics with amplitude
1/h, peak 0.3) with a 10 % unvoiced gap, generated analytically at 24 kHz (f32) and at 16 kHz
(int16-quantised / 32768 as the reference's ffmpeg decode, utils/whisper_extractor/audio.py:41-49)
from the same continuous-time formula, so no resampler is involved. Clip k is seeded by k.
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
    y *= 0.3 / np.max(np.abs(y))
    return y.astype(np.float32)


def synth_clip_16k_quantised(k, seconds):
    y = synth_clip(k, seconds, 16000).astype(np.float64)
    q = np.clip(np.round(y * 32768.0), -32768, 32767).astype(np.int16)
    return q.astype(np.float32) / 32768.0
