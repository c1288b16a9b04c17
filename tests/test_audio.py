"""Audio I/O and resampling (F1) on the CPU: the WAV reader/writer against the stdlib `wave` module and the
reference's own files, and the resampler's filter design + index arithmetic against scipy.signal.resample_poly
(the GPU kernel evaluates exactly this arithmetic; tests/test_gpu_audio.py checks the device results).

Parity notes: the reference resamples with librosa/soxr and decodes Whisper's input with ffmpeg, neither of
which is installed; resampling parity is pinned to scipy's polyphase algorithm and is "unpinned" against
soxr / ffmpeg. save_audio's int16 conversion is pinned by gen/1100000814_svcc_CDF1.wav (peak -29491).
"""
import ctypes
import os
import wave

import numpy as np
import pytest
import scipy.signal as ss

from oracle import features as OF
from svc_inference_pipeline_amd import _lib
from svc_inference_pipeline_amd import audio as A

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
RATIOS = [(44100, 24000), (44100, 16000), (24000, 16000), (48000, 24000), (22050, 24000), (16000, 24000)]


def _taps(si, so):
    n, up, dn, pr = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    refs = [ctypes.byref(v) for v in (n, up, dn, pr)]
    _lib.call("svc_resample_filter", si, so, None, 0, *refs)
    h = np.zeros(n.value)
    _lib.call("svc_resample_filter", si, so, ctypes.c_void_p(h.ctypes.data), n.value, *refs)
    return h, up.value, dn.value, pr.value


def _kernel_emulation(x, si, so):
    """resample_kernel's per-output arithmetic (csrc/resample.hip), evaluated in numpy f64."""
    h, up, dn, pr = _taps(si, so)
    n_in = len(x)
    n_out = _lib.load().svc_resample_len(n_in, si, so)
    y = np.zeros(n_out)
    for n in range(n_out):
        j = (n + pr) * dn
        k0, i0 = j % up, j // up
        r = np.arange(max(0, i0 - (n_in - 1)), min((len(h) - 1 - k0) // up, i0) + 1)
        y[n] = np.sum(h[k0 + up * r] * x[i0 - r])
    return y


@pytest.mark.parametrize("si,so", RATIOS)
def test_resample_filter_is_scipy_firwin(si, so):
    h, up, dn, pr = _taps(si, so)
    R = max(up, dn)
    half = 10 * R
    ref = ss.firwin(2 * half + 1, 1.0 / R, window=("kaiser", 5.0)) * up
    pad = dn - half % dn
    assert len(h) == pad + len(ref) and pr == (half + pad) // dn
    assert np.all(h[:pad] == 0)
    np.testing.assert_allclose(h[pad:], ref, rtol=0, atol=1e-14)


@pytest.mark.parametrize("si,so", RATIOS)
def test_resample_arithmetic_is_resample_poly(si, so):
    for n_in in (1, 2, 7, 300, 1001):
        x = np.random.default_rng(n_in).standard_normal(n_in)
        y = _kernel_emulation(x, si, so)
        ref = ss.resample_poly(x, so, si)
        assert y.shape == ref.shape
        np.testing.assert_allclose(y, ref, rtol=0, atol=1e-12)


def _write_pcm(path, samples, width, sr=22050, channels=1):
    with wave.open(path, "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(width)
        w.setframerate(sr)
        w.writeframes(samples.tobytes())


@pytest.mark.parametrize("width", [1, 2, 3, 4])
def test_read_wav_pcm_scaling(tmp_path, width):
    rng = np.random.default_rng(width)
    n, ch = 257, 2
    if width == 1:
        raw = rng.integers(0, 256, n * ch).astype(np.uint8)
        exp = (raw.astype(np.float64) - 128) / 128
        data = raw
    elif width == 3:
        v = rng.integers(-(1 << 23), 1 << 23, n * ch)
        b = (v & 0xFFFFFF).astype(np.uint32)
        data = np.stack([(b & 0xFF), (b >> 8) & 0xFF, (b >> 16) & 0xFF], 1).astype(np.uint8)
        exp = v / float(1 << 23)
    else:
        dt = {2: "<i2", 4: "<i4"}[width]
        v = rng.integers(np.iinfo(dt).min, np.iinfo(dt).max, n * ch).astype(dt)
        data = v
        exp = v.astype(np.float64) / float(1 << (8 * width - 1))
    p = str(tmp_path / "x.wav")
    _write_pcm(p, data, width, channels=ch)
    x, sr = A.read_wav(p)
    assert sr == 22050 and x.shape == (n, ch)
    np.testing.assert_array_equal(x, exp.reshape(n, ch))


def test_read_reference_test_clip(golden):
    """The reference's input clip (test_set/1100000814.wav): 44.1 kHz PCM16 mono, read like soundfile."""
    g = golden("format_golden")
    path = os.path.join(GOLDEN, "test_set_1100000814.wav")
    x, sr = A.read_wav(path)
    assert sr == int(g["in_sr"]) and x.shape == (int(g["in_len"]), 1)
    with wave.open(path, "rb") as w:
        ref = np.frombuffer(w.readframes(w.getnframes()), "<i2").astype(np.float64) / 32768.0
    np.testing.assert_array_equal(x[:, 0], ref)
    # 24 kHz length through the resampler -> 379 mel frames, as the reference's output file has
    n24 = _lib.load().svc_resample_len(x.shape[0], sr, 24000)
    assert OF.mel_frames(n24) == 379 and 1200 + 256 * 379 + 1200 == int(g["out_len"])


def test_save_audio_matches_reference_format(tmp_path, golden):
    w = np.random.default_rng(0).uniform(-0.4, 0.3, 5000).astype(np.float32)
    pcm = A.to_pcm16(w, 24000)
    np.testing.assert_array_equal(pcm, OF.save_audio_pcm16(w, 24000))
    assert len(pcm) == 5000 + 2 * 1200 and max(pcm.max(), -pcm.min()) == 29491
    p = str(tmp_path / "o.wav")
    A.save_audio(p, w, 24000)
    with wave.open(p, "rb") as f:
        assert (f.getnchannels(), f.getsampwidth(), f.getframerate()) == (1, 2, 24000)
        back = np.frombuffer(f.readframes(f.getnframes()), "<i2")
    np.testing.assert_array_equal(back, pcm)


def test_normalisation_classes():
    """utils/audio.py:36-42: float data is divided by 1, 2^15+1 or 2^31+1 depending on its peak."""
    x = np.array([0.5, -1.0], np.float64)
    np.testing.assert_array_equal(A._normalise(x), x.astype(np.float32))
    y = np.array([300.0, -2.0])
    np.testing.assert_allclose(A._normalise(y), (y / 32769.0).astype(np.float32), rtol=1e-7)
    z = np.array([70000.0, 1.0])
    np.testing.assert_allclose(A._normalise(z), (z / 2147483649.0).astype(np.float32), rtol=1e-7)
