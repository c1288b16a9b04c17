"""GPU: resampler vs scipy.signal.resample_poly, config-1 plumbing through the infer.py counterpart, and the
reference checkpoint formats (F2) end to end.

Tolerances: the resampler accumulates in f64 and stores f32, so it must match scipy (f64) to f32 rounding
(|err| <= 2e-7 * max|y| + 1e-9); the 16 kHz int16 quantisation may differ by one LSB where f32 rounding
crosses a rounding boundary (<= 0.1 % of samples). Checkpoint-loaded and state-loaded engines must agree
bit-exactly.
"""
import os
import wave

import numpy as np
import pytest
import scipy.signal as ss
import torch

pytestmark = pytest.mark.gpu

from svc_inference_pipeline_amd import audio as A  # noqa: E402
from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import infer as I  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CLIP = os.path.join(GOLDEN, "test_set_1100000814.wav")


@pytest.mark.parametrize("si,so", [(44100, 24000), (44100, 16000), (48000, 24000), (22050, 24000), (16000, 24000)])
@pytest.mark.parametrize("n_in", [1, 5, 1000, 178598])
def test_resample_matches_scipy(si, so, n_in):
    x = (np.random.default_rng(n_in).standard_normal((2, n_in)) * 0.3).astype(np.float32)
    y = A.resample(x, si, so).cpu().numpy()
    ref = ss.resample_poly(x.astype(np.float64), so, si, axis=1)
    assert y.shape == ref.shape
    assert np.max(np.abs(y - ref)) <= 2e-7 * max(np.max(np.abs(ref)), 1e-3) + 1e-9


def test_resample_int16_quantisation():
    x = (np.random.default_rng(1).standard_normal(44100) * 0.2).astype(np.float32)
    y = A.resample(x, 44100, 16000, quantize16=True).cpu().numpy()
    q = np.clip(np.round(ss.resample_poly(x.astype(np.float64), 16000, 44100) * 32768.0), -32768, 32767)
    d = np.abs(y * 32768.0 - q)
    assert d.max() <= 1.0 and np.mean(d > 0) <= 1e-3
    assert np.array_equal(y * 32768.0, np.round(y * 32768.0))  # on the int16 grid


def test_infer_cli_plumbing(tmp_path, golden):
    """BASELINE config 1 counterpart: test_set/1100000814.wav -> svcc_CDF1 through the CLI (seeded weights,
    PLMS). The output file has the reference's format (gen/1100000814_svcc_CDF1.wav): 24 kHz 16-bit mono,
    1200 + 379*256 + 1200 samples, peak 29491, 50 ms of silence each side."""
    g = golden("format_golden")
    out = str(tmp_path / "gen" / "out.wav")
    assert I.main(["--wav", CLIP, "--singer", "svcc_CDF1", "--out", out, "--random-weights", "tiny-test", "--fast",
                   "--speedup", "250"]) == 0
    with wave.open(out, "rb") as f:
        assert (f.getnchannels(), f.getsampwidth(), f.getframerate()) == (1, 2, int(g["out_sr"]))
        pcm = np.frombuffer(f.readframes(f.getnframes()), "<i2")
    assert len(pcm) == int(g["out_len"])
    assert max(int(pcm.max()), -int(pcm.min())) == int(g["out_peak"])
    assert np.all(pcm[:1200] == 0) and np.all(pcm[-1200:] == 0)


def test_infer_cli_several_files(tmp_path):
    """Several --wav files run as ONE ragged batch (convert_many): each written file equals the single-file CLI's
    (file 0 has utterance id 0 in both runs; a second file of another length rides in the same batch)."""
    with wave.open(CLIP, "rb") as f:
        params, pcm = f.getparams(), f.readframes(f.getnframes())
    short = str(tmp_path / "short.wav")
    with wave.open(short, "wb") as f:
        f.setparams(params)
        f.writeframes(pcm[:len(pcm) * 3 // 5 // 2 * 2])
    common = ["--singer", "svcc_CDF1", "--random-weights", "tiny-test", "--fast", "--speedup", "250"]
    one = str(tmp_path / "one.wav")
    assert I.main(["--wav", CLIP, "--out", one] + common) == 0
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        assert I.main(["--wav", CLIP, short] + common) == 0
    finally:
        os.chdir(cwd)
    stem = os.path.splitext(os.path.basename(CLIP))[0]
    outs = [tmp_path / "gen" / f"{stem}_svcc_CDF1.wav", tmp_path / "gen" / "short_svcc_CDF1.wav"]
    read = lambda p: wave.open(str(p), "rb").readframes(10 ** 9)  # noqa: E731
    assert read(outs[0]) == read(one)
    assert 0 < len(read(outs[1])) < len(read(outs[0]))


@pytest.fixture(scope="module")
def tiny_states():
    cfg = C.load_config()
    cfg.mapper.input_content_dim["whisper"] = W.WHISPER_DIMS["tiny-test"]["n_audio_state"]
    return cfg, dict(whisper=W.make_whisper_state(W.WHISPER_DIMS["tiny-test"], 3), mapper=W.make_mapper_state(cfg.mapper, 3),
                     vocoder=W.make_vocoder_state(cfg.vocoder, 3))


def _outputs(engine, cfg):
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.uniform(-1, 1, (1, 40, 100)).astype(np.float32)).cuda()
    cond = torch.from_numpy(rng.standard_normal((1, 40, 384)).astype(np.float32)).cuda()
    wav16 = torch.from_numpy(rng.uniform(-0.3, 0.3, (1, 16000)).astype(np.float32)).cuda()
    return [engine.bigvgan(x).cpu().numpy(), engine.diffsvc_eps(cond, x, 321).cpu().numpy(),
            engine.whisper_encode(wav16).cpu().numpy()]


def test_checkpoint_formats_roundtrip(tmp_path, tiny_states):
    cfg, st = tiny_states
    paths = W.save_checkpoints(str(tmp_path), st["mapper"], st["vocoder"], st["whisper"], module_prefix=True)
    loaded = W.load_checkpoints(paths["mapper"], paths["vocoder"], paths["whisper"])
    for k in ("mapper", "vocoder", "whisper"):
        assert set(loaded[k]) == set(st[k])
        for name in st[k]:
            np.testing.assert_array_equal(loaded[k][name], st[k][name])
    e1 = SVCEngine(cfg, 0, whisper_state=st["whisper"], mapper_state=st["mapper"], vocoder_state=st["vocoder"])
    e2 = I.build_engine(cfg, 0, paths["mapper"], paths["vocoder"], paths["whisper"])
    for a, b in zip(_outputs(e1, cfg), _outputs(e2, cfg)):
        assert np.array_equal(a, b)
    e1.close()
    e2.close()


def test_checkpoint_missing_key_fails_loudly(tmp_path, tiny_states):
    """The reference keeps random init for a missing key (utils/load_models.py:34-43); here finalize fails."""
    cfg, st = tiny_states
    voc = dict(st["vocoder"])
    voc.pop(next(k for k in voc if k.startswith("resblocks.0.convs1.0")))
    paths = W.save_checkpoints(str(tmp_path), st["mapper"], voc, st["whisper"])
    with pytest.raises(Exception):
        I.build_engine(cfg, 0, paths["mapper"], paths["vocoder"], paths["whisper"])
