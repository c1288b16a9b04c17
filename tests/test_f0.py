"""F0 (Praat to_pitch_ac, utils/f0.py:120-161). PARITY UNPINNED: parselmouth/Praat is absent, so the
oracle (oracle/praat_ac.py, a restatement of Praat's published algorithm) is checked with known-answer
tests on synthetic tones (CPU), and the HIP kernel is checked against the oracle (GPU): frame count and
voicing decisions exact, frequencies to 2e-7 relative (Brent tolerance; the kernel's own f64 radix-4/2 FFT
autocorrelation vs numpy's FFT: the same transform, rounded differently)."""
import numpy as np
import pytest

from oracle import praat_ac as PA
from svc_inference_pipeline_amd.synth import clip_params, synth_clip

FS = 24000


def tone(f, seconds=1.0, harmonics=5):
    t = np.arange(int(FS * seconds)) / FS
    return (sum(np.sin(2 * np.pi * f * h * t) / h for h in range(1, harmonics + 1)) * 0.3).astype(np.float32)


@pytest.mark.parametrize("f", [70.0, 110.0, 220.0, 440.0, 780.0])
def test_known_tones(f):
    f0 = PA.to_pitch_ac(tone(f), FS, 256 / FS)
    v = f0[f0 > 0]
    assert len(v) == len(f0)  # a steady periodic tone is voiced everywhere
    assert np.max(np.abs(v / f - 1)) < (1e-3 if f < 100 else 2e-4)  # ~3 periods per window near the floor


def test_silence_and_noise_unvoiced():
    assert np.all(PA.to_pitch_ac(np.zeros(FS, np.float32), FS, 256 / FS) == 0)
    x = (np.random.default_rng(0).standard_normal(FS) * 0.01).astype(np.float32)
    assert np.mean(PA.to_pitch_ac(x, FS, 256 / FS) > 0) < 0.05


def test_frame_count_and_padding():
    """10 s at 24 kHz: Praat fits 934 frames; utils/f0.py:156-157 pads (2, 1) to 937 mel frames."""
    P = PA.analysis_params(240000, FS, 256 / FS, 65.0, 800.0)
    assert P["n_frames"] == 934 and P["nsamp_window"] == 1104 and P["brent_ixmax"] == 552 and P["nfft"] == 2048
    f0 = PA.f0_features(tone(200.0, 10.0), 937)
    assert len(f0) == 937 and f0[0] == 0 and f0[1] == 0 and f0[-1] == 0 and f0[2] > 0


def test_synthetic_clip_tracks_vibrato():
    x = synth_clip(3, 2.0, FS)
    f0 = PA.f0_features(x, (len(x) + 768 - 1024) // 256 + 1)
    p = clip_params(3)
    v = f0[f0 > 0]
    assert 0.75 < len(v) / len(f0) < 0.95
    assert abs(np.median(v) / p["f0"] - 1) < 0.01


@pytest.mark.gpu
def test_gpu_f0_matches_oracle():
    import torch
    from svc_inference_pipeline_amd import config as C
    from svc_inference_pipeline_amd.runtime import SVCEngine
    cfg = C.load_config()
    eng = SVCEngine(cfg, 0)
    clips = [synth_clip(5, 3.0, FS), tone(150.0, 3.0), (np.random.default_rng(1).standard_normal(3 * FS) * 0.05).astype(np.float32),
             np.concatenate([tone(300.0, 1.5), np.zeros(int(1.5 * FS), np.float32)])]
    wav = torch.from_numpy(np.stack(clips)).cuda()
    T = (wav.shape[1] + 768 - 1024) // 256 + 1
    f0 = eng.f0(wav, T).cpu().numpy()
    for b, x in enumerate(clips):
        ref = PA.f0_features(x, T)
        assert np.array_equal(f0[b] > 0, ref > 0), b
        # Brent stops at tol_act = 1.5e-8*lag + 3e-11 (NUMminimize_brent): frequencies agree to ~1e-7;
        # on flat autocorrelation maxima (onsets/offsets) the stopping point moves within that flat
        # region, so <= 1 % of frames may differ by up to 1e-5 relative.
        rel = np.abs(f0[b] - ref) / np.maximum(np.abs(ref), 1e-300)
        assert np.all(rel <= 1e-5), (b, rel.max())
        assert np.mean(rel > 2e-7) <= 0.01, (b, np.mean(rel > 2e-7))
    # pitch shift: np.median semantics
    f0d = torch.from_numpy(f0.copy()).cuda()
    eng.pitch_shift(f0d, 223.25784012425046)
    for b in range(len(clips)):
        v = f0[b] != 0
        if v.any():
            exp = f0[b] * (223.25784012425046 / np.median(f0[b][v]))
            np.testing.assert_array_equal(f0d[b].cpu().numpy(), exp)
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("fs,floor", [(24000, 250.0), (16000, 150.0), (24000, 150.0), (44100, 65.0)])
def test_gpu_f0_fft_sizes(fs, floor):
    """The autocorrelation FFT at every size the frame kernel has a plan for (nfft = the power of two >= 1.5 x the
    3-period window): 512 (24 kHz with a 250 Hz floor, 16 kHz with 150 Hz), 1024 (24 kHz, 150 Hz) and 4096 (44.1 kHz,
    65 Hz); the default configuration (2048) is test_gpu_f0_matches_oracle. Same bar as there, except that a frame on a
    flat maximum (the tone's offset into silence) may move by up to 5e-5 relative at 44.1 kHz (measured 1.8e-5 on one
    frame, r06a: the 2034-sample window's autocorrelation is flatter around its peak, so Brent's stopping point moves
    further for the same rounding difference)."""
    import torch
    from svc_inference_pipeline_amd import config as C
    from svc_inference_pipeline_amd.runtime import SVCEngine
    P = PA.analysis_params(3 * fs, fs, 256 / fs, floor, 800.0)
    cfg = C.load_config()
    cfg.fs, cfg.f0_min = fs, floor
    eng = SVCEngine(cfg, 0)
    t = np.arange(3 * fs) / fs
    clips = [(0.3 * np.sin(2 * np.pi * 330.0 * t * (1 + 0.03 * np.sin(2 * np.pi * 5.5 * t)))).astype(np.float32),
             np.concatenate([np.sin(2 * np.pi * 420.0 * t[:fs]) * 0.2, np.zeros(2 * fs)]).astype(np.float32),
             (np.random.default_rng(2).standard_normal(3 * fs) * 0.05).astype(np.float32)]
    wav = torch.from_numpy(np.stack(clips)).cuda()
    T = 3 * fs // 256 + 1
    f0 = eng.f0(wav, T).cpu().numpy()
    for b, x in enumerate(clips):
        ref = PA.f0_features(x, T, fs=fs, floor=floor)
        assert np.array_equal(f0[b] > 0, ref > 0), (P["nfft"], b)
        rel = np.abs(f0[b] - ref) / np.maximum(np.abs(ref), 1e-300)
        assert np.all(rel <= (5e-5 if fs > 24000 else 1e-5)), (P["nfft"], b, rel.max())
        assert np.mean(rel > 2e-7) <= 0.01, (P["nfft"], b)
    eng.close()


# ---------------------------------------------------------------------------- pYIN (utils/f0.py:95-117)
# PARITY UNPINNED: librosa is absent, so oracle/pyin.py (a restatement of librosa 0.10's pyin) is pinned only by
# known-answer tones and silence; the HIP kernels (csrc/pyin.hip) are held to the oracle.
from oracle import pyin as PY  # noqa: E402

PY_ARGS = dict(fs=FS, win_length=1024, hop_length=256, f0_min=65.0, f0_max=800.0)  # config/config.json values


def test_pyin_params():
    p = PY.pyin_params(FS, 65.0, 800.0, 2048, 1024, 256)
    # min/max period from the f0 range, the window limit 2048 - 1024 - 1 = 1023 not binding; 435 bins of 0.1 semitone;
    # transition width round(35.92 * 12 * 256 / 24000) = 5 semitones -> 51 bins
    assert (p["min_period"], p["max_period"], p["n_bins"], p["width"]) == (30, 370, 435, 51)
    t = PY.transition_local(p["n_bins"], p["width"])
    np.testing.assert_allclose(t.sum(axis=1), 1.0, rtol=1e-12)
    assert np.count_nonzero(t[200]) == 51 and np.count_nonzero(t[0]) == 26  # centred band, cut at the edges


@pytest.mark.parametrize("f", [82.0, 110.0, 220.0, 440.0, 700.0])
def test_pyin_known_tones(f):
    f0 = PY.f0_pyin(tone(f, 0.8), **PY_ARGS)
    assert len(f0) == 1 + int(0.8 * FS) // 256
    v = f0[f0 > 0]
    assert len(v) >= 0.9 * len(f0)
    # bins are 0.1 semitone (0.58 %) apart; the parabolic period estimate of a 5-harmonic tone lands within a bin
    assert np.median(np.abs(v / f - 1)) < 0.006


def test_pyin_silence_unvoiced():
    assert np.all(PY.f0_pyin(np.zeros(FS // 2, np.float32), **PY_ARGS) == 0)


def _pyin_clips():
    rng = np.random.default_rng(3)
    return [
        synth_clip(5, 1.5, FS),
        tone(150.0, 1.5),
        (rng.standard_normal(int(1.5 * FS)) * 0.05).astype(np.float32),
        np.concatenate([tone(300.0, 0.7), np.zeros(int(0.8 * FS), np.float32)]),
    ]


@pytest.mark.gpu
def test_gpu_pyin_matches_oracle():
    """HIP pYIN vs the oracle: the decoded path agrees on >= 99 % of frames (voicing and bin) per clip. The kernels sum
    the lag products directly in f64 where librosa (and the oracle) use an FFT, so a CMND value that sits on a trough /
    threshold decision boundary may flip; everything downstream is the same f64 arithmetic. A bin's frequency
    fmin * 2^(k / 120) is compared to 1e-14 relative, not bit for bit: the library's table comes from C pow, numpy's
    from its own vectorised power, and the two differ by 1 ulp on 24 of the 435 bins (first GPU run, r04i: every
    mismatching frame was such a bin; bins are 0.58 % apart, so the tolerance cannot confuse two)."""
    import torch
    from svc_inference_pipeline_amd import config as C
    from svc_inference_pipeline_amd.runtime import SVCEngine
    eng = SVCEngine(C.load_config(), 0)
    clips = _pyin_clips()
    wav = torch.from_numpy(np.stack(clips)).cuda()
    f0 = eng.f0_pyin(wav).cpu().numpy()
    assert f0.shape == (len(clips), 1 + wav.shape[1] // 256)
    for b, x in enumerate(clips):
        ref = PY.f0_pyin(x, **PY_ARGS)
        same = np.isclose(f0[b], ref, rtol=1e-14, atol=0)
        assert np.mean(same) >= 0.99, (b, np.mean(same), np.nonzero(~same)[0][:10])
        assert np.array_equal(f0[b] > 0, ref > 0) or np.mean((f0[b] > 0) != (ref > 0)) <= 0.01, b
    # ragged batch: each utterance as a clip of its own length, rows past its frames 0
    lens = [int(1.5 * FS), int(0.9 * FS), int(0.4 * FS) + 77, int(1.2 * FS)]
    f0r = eng.f0_pyin(wav, n_samples=lens).cpu().numpy()
    for b, n in enumerate(lens):
        Fb = 1 + n // 256
        alone = eng.f0_pyin(wav[b:b + 1, :n].contiguous()).cpu().numpy()[0]
        np.testing.assert_array_equal(f0r[b, :Fb], alone)
        assert np.all(f0r[b, Fb:] == 0)
    eng.close()
