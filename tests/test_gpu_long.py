"""GPU parity for long clips (BASELINE config 4, SURVEY.md §5 "Long-context").

The reference cannot run clips over ~30 s (utils/whisper.py:52-56 pads/trims to one window; the mapped
2812-frame content then fails to concatenate in modules/encoder.py:197), so parity here is per window:
the GPU's windowed Whisper content (svc_inference_pipeline_amd/pipeline.py) must match the oracle's
per-window restatement (oracle/pipeline.whisper_content), and mel/energy/F0 — which the reference
computes over the whole clip — must match the oracle over the whole clip.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from gpu_util import dev, rel_l2  # noqa: E402
from oracle import features as OF  # noqa: E402
from oracle import noise as ON  # noqa: E402
from oracle import pipeline as OP  # noqa: E402
from oracle import praat_ac as PA  # noqa: E402
from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402
from svc_inference_pipeline_amd.pipeline import SVCPipeline  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402

TINY = W.WHISPER_DIMS["tiny-test"]
SECONDS = 65.0   # three Whisper windows (2805 + 2805 + 484 mel frames)


@pytest.fixture(scope="module")
def cfg():
    c = C.load_config()
    c.mapper.input_content_dim["whisper"] = TINY["n_audio_state"]
    return c


@pytest.fixture(scope="module")
def states(cfg):
    return dict(whisper=W.make_whisper_state(TINY, 0), mapper=W.make_mapper_state(cfg.mapper, 0),
                vocoder=W.make_vocoder_state(cfg.vocoder, 0))


@pytest.fixture(scope="module")
def engine(cfg, states):
    e = SVCEngine(cfg, 0, whisper_state=states["whisper"], mapper_state=states["mapper"], vocoder_state=states["vocoder"])
    yield e
    e.close()


@pytest.fixture(scope="module")
def clip():
    wav24 = ON.synth_clip(11, SECONDS, 24000)
    wav16 = ON.synth_clip_16k_quantised(11, SECONDS)
    return wav24, wav16


def test_long_content_windows(engine, states, clip):
    wav24, wav16 = clip
    T = OF.mel_frames(len(wav24))
    assert T > 2 * 2805
    content = SVCPipeline(engine).content(dev(wav16[None]), T)[0].float().cpu().numpy()
    ref = OP.whisper_content(states["whisper"], wav16, T)
    assert content.shape == ref.shape == (T, TINY["n_audio_state"])
    # same bound as the single-window encoder test, per window
    for c in range(3):
        sl = slice(c * 2805, min(T, (c + 1) * 2805))
        assert rel_l2(content[sl], ref[sl]) < 5e-3, c


def test_long_mel_f0(engine, cfg, clip):
    wav24, _ = clip
    mel, en = engine.mel_energy(dev(wav24[None]))
    T = mel.shape[1]
    ref = OF.mel_spectrogram(torch.from_numpy(wav24)[None], cfg)[0].numpy()
    assert np.mean(np.abs(mel[0].cpu().numpy().T - ref)) < 3e-5
    f0 = engine.f0(dev(wav24[None]), T)[0].cpu().numpy()
    f0_ref = PA.f0_features(wav24, T, fs=cfg.fs, hop=cfg.hop_length, floor=cfg.f0_min, ceiling=cfg.f0_max)
    assert np.array_equal(f0 > 0, f0_ref > 0)
    rel = np.abs(f0 - f0_ref) / np.maximum(f0_ref, 1.0)
    assert rel.max() < 1e-5 and np.mean(rel > 2e-7) < 0.01


def test_long_convert_runs_full_length(engine, cfg, clip):
    wav24, wav16 = clip
    r = SVCPipeline(engine).convert(dev(wav24[None]), dev(wav16[None]), dev(np.array([1]), torch.int32),
                                    speedup=250)
    T = r.mel.shape[1]
    assert r.wav.shape == (1, T * cfg.hop_length)
    assert torch.isfinite(r.wav).all()
