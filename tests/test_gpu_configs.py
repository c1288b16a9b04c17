"""GPU parity for BASELINE.json configs[3] and configs[4] at their real dimensions.

configs[3] — one 180 s song (T = 16 875 mel frames) through the headline engine (Whisper-medium). The reference cannot
run it (utils/whisper.py:52-56 pads / trims to one 30 s window, and the 2812-frame mapped content then fails to
concatenate in modules/encoder.py:197), so, as in tests/test_gpu_long.py, content parity is per 29.92 s window
against oracle.pipeline.whisper_content (7 windows), mel / energy / F0 parity is over the whole clip, and the converted
waveform must be finite and full length.

configs[4] — the HuBERT / ContentVec content encoder (fairseq layer 9 + final_proj, utils/hubert.py:31-47,83-134) at
the real ContentVec dims with the 1000-step DDPM schedule: the north-star mel-L1 tolerance (<= 1e-3 of the
de-normalised ln-mel, utils/acoustic_feature_extraction.py:83-97) against the fp32 oracle with shared x_T and step
noise, in the engine's default precision mode.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from gpu_util import dev, rel_l2  # noqa: E402
from mel_l1 import MEL_L1_TARGET, ddpm1000_mel_l1, gpu_mel, oracle_mel  # noqa: E402
from oracle import features as OF  # noqa: E402
from oracle import noise as ON  # noqa: E402
from oracle import pipeline as OP  # noqa: E402
from oracle import praat_ac as PA  # noqa: E402
from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402
from svc_inference_pipeline_amd.pipeline import WINDOW_MEL_FRAMES, SVCPipeline  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402

MEDIUM = W.WHISPER_DIMS["medium"]


@pytest.fixture(scope="module")
def long_setup():
    torch.set_num_threads(16)
    cfg = C.load_config()
    cfg.mapper.input_content_dim["whisper"] = MEDIUM["n_audio_state"]
    ws = W.make_whisper_state(MEDIUM, 0)
    e = SVCEngine(cfg, 0, whisper_state=ws, mapper_state=W.make_mapper_state(cfg.mapper, 0),
                  vocoder_state=W.make_vocoder_state(cfg.vocoder, 0))
    wav24 = ON.synth_clip(21, 180.0, 24000)
    wav16 = ON.synth_clip_16k_quantised(21, 180.0)
    yield cfg, ws, e, wav24, wav16
    e.close()


def test_config4_180s_content_per_window(long_setup):
    cfg, ws, e, wav24, wav16 = long_setup
    T = OF.mel_frames(len(wav24))
    assert T == 16875
    n_win = -(-T // WINDOW_MEL_FRAMES)
    assert n_win == 7
    content = SVCPipeline(e).content(dev(wav16[None]), T)[0].float().cpu().numpy()
    with torch.no_grad():
        ref = OP.whisper_content(ws, wav16, T)
    assert content.shape == ref.shape == (T, MEDIUM["n_audio_state"])
    for c in range(n_win):  # the headline encoder's bound (tests/test_gpu_headline.py), per window
        sl = slice(c * WINDOW_MEL_FRAMES, min(T, (c + 1) * WINDOW_MEL_FRAMES))
        assert rel_l2(content[sl], ref[sl]) < 2e-3, (c, rel_l2(content[sl], ref[sl]))


def test_config4_180s_mel_f0_and_full_length_convert(long_setup):
    cfg, ws, e, wav24, wav16 = long_setup
    mel, en = e.mel_energy(dev(wav24[None]))
    T = mel.shape[1]
    ref = OF.mel_spectrogram(torch.from_numpy(wav24)[None], cfg)[0].numpy()
    assert ref.shape[-1] == T  # bit-exact frame count
    assert np.mean(np.abs(mel[0].cpu().numpy().T - ref)) < 3e-5
    np.testing.assert_allclose(en[0].cpu().numpy(), OF.energy_from_mel(torch.from_numpy(ref)[None])[0].numpy(),
                               rtol=2e-5, atol=1e-7)
    f0 = e.f0(dev(wav24[None]), T)[0].cpu().numpy()
    f0_ref = PA.f0_features(wav24, T, fs=cfg.fs, hop=cfg.hop_length, floor=cfg.f0_min, ceiling=cfg.f0_max)
    assert np.array_equal(f0 > 0, f0_ref > 0)
    rel = np.abs(f0 - f0_ref) / np.maximum(f0_ref, 1.0)
    assert rel.max() < 1e-5 and np.mean(rel > 2e-7) < 0.01
    r = SVCPipeline(e).convert(dev(wav24[None]), dev(wav16[None]), dev(np.array([3]), torch.int32), speedup=10,
                               seed=5)
    assert r.wav.shape == (1, T * cfg.hop_length) and r.x0.shape == (1, T, 100)
    assert bool(torch.isfinite(r.wav).all()) and bool(torch.isfinite(r.x0).all())


@pytest.mark.parametrize("seconds", [1.0, pytest.param(10.0, marks=pytest.mark.timeout(900))])
def test_config5_contentvec_ddpm1000_mel_l1(seconds):
    """ContentVec (768 wide, 12 layers used up to output_layer 9, final_proj 256) + DDPM-1000, shared x_T and per-step
    noise, default precision mode: de-normalised ln-mel L1 <= 1e-3 against the fp32 oracle, at 1 s (T = 93) and at the
    headline 10 s (T = 937)."""
    torch.set_num_threads(16)
    cfg = C.load_config()
    cfg.mapper.content_feature = ["contentvec"]
    cfg.mapper.input_content_dim["contentvec"] = W.HUBERT_DIMS["contentvec"]["final_dim"]
    states = dict(hubert=W.make_hubert_state(W.HUBERT_DIMS["contentvec"], 0), mapper=W.make_mapper_state(cfg.mapper, 0))
    e = SVCEngine(cfg, 0, mapper_state=states["mapper"], vocoder_state=W.make_vocoder_state(cfg.vocoder, 0),
                  hubert_state=states["hubert"])
    try:
        l1 = ddpm1000_mel_l1(e, cfg, states, "contentvec", seconds)
    finally:
        e.close()
    print(f"mel-L1 contentvec DDPM-1000 {seconds:g} s: {l1:.4e}")
    assert l1 <= MEL_L1_TARGET, l1


def test_config5_fp16_vs_bf16_operands():
    """BASELINE configs[4]'s fp16-vs-bf16 tolerance sweep on the MI355X kernels (ContentVec + DDPM-1000, 1 s clip, shared
    x_T / noise): the bf16 operand variant (SVCEngine(operands="bf16"): the content encoder, conditioner and DiffSVC
    GEMMs and attention on v_mfma_f32_16x16x32_bf16) against the fp32 oracle and against the oracle with every operand
    rounded to bf16 (the same precision class, fp32 accumulation). Plain bf16 operands track the bf16 emulation
    (within 2x its distance from fp32) and miss the 1e-3 target by an order of magnitude, where plain fp16 misses it by
    ~1.6x and the default split-fp16 mode meets it (DESIGN.md precision sweep, profiles/r03*_precision_sweep.json)."""
    torch.set_num_threads(16)
    cfg = C.load_config()
    cfg.mapper.content_feature = ["contentvec"]
    cfg.mapper.input_content_dim["contentvec"] = W.HUBERT_DIMS["contentvec"]["final_dim"]
    states = dict(hubert=W.make_hubert_state(W.HUBERT_DIMS["contentvec"], 0), mapper=W.make_mapper_state(cfg.mapper, 0))
    vs = W.make_vocoder_state(cfg.vocoder, 0)
    mel = {}
    for name, operands, split, head in (("bf16", "bf16", 0, False), ("bf16-split", "bf16", 2, True),
                                        ("fp16", "fp16", 0, False)):
        e = SVCEngine(cfg, 0, mapper_state=states["mapper"], vocoder_state=vs, hubert_state=states["hubert"],
                      content_split=split, head_split=head, operands=operands)
        try:
            mel[name] = gpu_mel(e, "contentvec", 1.0)
        finally:
            e.close()
    ref = oracle_mel(cfg, states, "contentvec", 1.0)
    emu = oracle_mel(cfg, states, "contentvec", 1.0, torch.bfloat16)
    l1 = {k: float(np.mean(np.abs(v - ref))) for k, v in mel.items()}
    l1_emu = float(np.mean(np.abs(emu - ref)))
    print(f"mel-L1 vs fp32: {l1}, bf16 emulation {l1_emu:.4e}, GPU bf16 vs emulation "
          f"{float(np.mean(np.abs(mel['bf16'] - emu))):.4e}")
    assert l1["bf16"] <= 2.0 * l1_emu + 1e-3, (l1, l1_emu)
    assert l1["bf16"] > l1["fp16"] and l1["bf16-split"] < l1["bf16"], l1
    assert l1["bf16"] > MEL_L1_TARGET  # the reason the build runs fp16 (DESIGN.md precision sweep)
