"""GPU parity for the HuBERT/ContentVec variant (BASELINE config 5), through the C-ABI.

Encoder: the HIP path (conv extractor as implicit GEMMs + GroupNorm, pos_conv per group, post-LN layers) vs
the oracle (tests/test_oracle_golden.py pins it to transformers.HubertModel, fairseq being absent) and vs that
fixture directly; fp16 MFMA operands, so relative L2 <= 5e-3. Mapping: bit-exact against the reference's own
get_mapped_features outputs (after the f16 store), and the >3-frame mismatch is a loud error. Conditioner with
several content types: against the reference's EncoderFramework fixture, relative L2 <= 5e-3.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from gpu_util import dev, rel_l2  # noqa: E402
from oracle import models as OM  # noqa: E402
from oracle import noise as ON  # noqa: E402
from svc_inference_pipeline_amd import _lib  # noqa: E402
from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402

HT = W.HUBERT_DIMS["tiny-test"]


@pytest.fixture(scope="module")
def hsd():
    return W.make_hubert_state(HT, 0)


@pytest.fixture(scope="module")
def engine(hsd):
    e = SVCEngine(C.load_config(), 0, hubert_state=hsd, hubert_output_layer=HT["output_layer"])
    yield e
    e.close()


def test_hubert_encoder_golden(engine, golden):
    g = golden("hubert_encoder_tiny")
    feats = engine.hubert_encode(dev(g["wav16"]))
    assert tuple(feats.shape) == g["feats"].shape
    assert rel_l2(feats.cpu().numpy(), g["feats"]) < 5e-3


@pytest.mark.parametrize("n", [400, 16000 * 3 + 123, 160000])
def test_hubert_encoder_vs_oracle(engine, hsd, n):
    """Ragged tails (n not a multiple of the 320-sample hop), the shortest clip giving one frame, and 10 s."""
    B = 2
    wav = np.stack([ON.synth_clip(10 + b, n / 16000.0, 16000)[:n] for b in range(B)]).astype(np.float32)
    feats = engine.hubert_encode(dev(wav))
    F = W.hubert_frames(n)
    assert feats.shape[1] == F == int(_lib.load().svc_hubert_frames(n))
    with torch.no_grad():
        ref = OM.hubert_content(hsd, torch.from_numpy(wav), HT["output_layer"]).numpy()
    assert ref.shape == tuple(feats.shape)
    assert rel_l2(feats.cpu().numpy(), ref) < 5e-3


def test_hubert_batch_independence(engine):
    """Utterances of a batch never mix (GroupNorm statistics and convolutions are per utterance)."""
    n = 16000
    wav = np.stack([ON.synth_clip(20 + b, 1.0, 16000) for b in range(3)]).astype(np.float32)
    both = engine.hubert_encode(dev(wav)).cpu()
    one = engine.hubert_encode(dev(wav[1:2])).cpu()
    assert torch.equal(both[1], one[0])


def test_hubert_map_exact(engine, golden):
    g = golden("hubert_map")
    for s, t in g["cases"]:
        raw = dev(g[f"raw_{s}_{t}"][None])
        out = engine.map_content(raw, int(t), rule="hubert")[0].cpu().numpy()
        exp = g[f"out_{s}_{t}"].astype(np.float32).astype(np.float16)
        assert np.array_equal(out, exp), (s, t)
    for s, t, _ in g["exits"]:
        with pytest.raises(_lib.SVCError, match="utils/hubert.py"):
            engine.map_content(dev(np.zeros((1, int(s), 4), np.float32)), int(t), rule="hubert")


def test_map_into_column_slice(engine, golden):
    """Mapping writes only its column slice of a concatenated content buffer."""
    g = golden("hubert_map")
    raw = dev(g["raw_499_937"][None])
    buf = torch.full((1, 937, 40), 7.0, device="cuda", dtype=torch.float16)
    engine.map_content(raw, 937, rule="hubert", out=buf[:, :, 8:32])
    exp = g["out_499_937"].astype(np.float32).astype(np.float16)
    b = buf[0].cpu().numpy()
    assert np.array_equal(b[:, 8:32], exp)
    assert np.all(b[:, :8] == 7.0) and np.all(b[:, 32:] == 7.0)


@pytest.mark.parametrize("types", [["whisper", "contentvec"], ["contentvec"]])
def test_conditioner_multi_content(golden, types):
    g = golden("conditioner_multi_content")
    cfg = C.load_config()
    cfg.mapper.content_feature = types
    cfg.mapper.input_content_dim["whisper"] = 128
    cfg.mapper.input_content_dim["contentvec"] = 32
    e = SVCEngine(cfg, 0, mapper_state=W.make_mapper_state(cfg.mapper, 0))
    try:
        content = np.concatenate([g[f"content_{t}"] for t in sorted(types)], axis=-1)
        cond = e.condition(dev(content, torch.float16), dev(g["f0"], torch.float64), dev(g["energy"]),
                           dev(g["singer"][0], torch.int32))
        tag = "multi" if len(types) == 2 else "cv"
        assert rel_l2(cond.cpu().numpy(), g[f"cond_{tag}"]) < 5e-3
    finally:
        e.close()


def test_contentvec_pipeline_plms(hsd):
    """Config-5 plumbing at small size: content_feature ["contentvec"] (HuBERT -> hubert map -> conditioner)
    -> PLMS-4 -> x0, against the oracle chain on the same weights, x_T and F0."""
    from svc_inference_pipeline_amd.pipeline import SVCPipeline
    from oracle import features as OF
    cfg = C.load_config()
    cfg.mapper.content_feature = ["contentvec"]
    cfg.mapper.input_content_dim["contentvec"] = HT["final_dim"]
    ms = W.make_mapper_state(cfg.mapper, 0)
    e = SVCEngine(cfg, 0, mapper_state=ms, vocoder_state=W.make_vocoder_state(cfg.vocoder, 0), hubert_state=hsd,
                  hubert_output_layer=HT["output_layer"])
    try:
        secs = 1.0
        w24 = ON.synth_clip(5, secs, 24000)[None]
        w16 = ON.synth_clip(5, secs, 16000)[None].astype(np.float32)
        T = OF.mel_frames(w24.shape[1])
        f0 = ON.synth_f0(3, T)[None]
        xT = ON.x_T(13, 1, T)
        res = SVCPipeline(e).convert(dev(w24), dev(w16), dev(np.array([2]), torch.int32), fast_inference=True,
                                     speedup=250, x_T=dev(xT), f0=dev(f0, torch.float64), wav16_float=dev(w16))
        torch.cuda.synchronize()
        # oracle chain
        mel = OF.mel_spectrogram(torch.from_numpy(w24), cfg)
        en = OF.energy_from_mel(mel)
        st = C.load_stats(cfg)
        f0s = torch.from_numpy(OF.pitch_shift(f0[0], st["target_f0_median"]))[None]
        with torch.no_grad():
            hf = OM.hubert_content(hsd, torch.from_numpy(w16), HT["output_layer"])[0].numpy()
        content = torch.from_numpy(OF.map_hubert_features(hf, T).astype(np.float32))[None]
        cond = OM.conditioner(ms, {"contentvec": content}, f0s, en, torch.tensor([[2]]))
        table = W.step_embedding_table(1000)
        consts = OM.schedule_constants(C.noise_schedule(cfg.mapper))
        den = lambda x, t: OM.diffsvc_forward(ms, cfg.mapper, x, cond, t, table)  # noqa: E731
        ref_x0 = OM.sample_plms(den, torch.from_numpy(xT), 1, T, 1000, 250, consts)
        assert rel_l2(res.x0.cpu().numpy(), ref_x0.numpy()) < 2e-2
        assert bool(torch.isfinite(res.wav).all())
    finally:
        e.close()


def test_contentvec_full_dims():
    """The real ContentVec shapes (512-channel extractor, 768-wide, 12 heads, 16 pos_conv groups of 48,
    output_layer 9, final 256) on a 2 s clip, B=2, against the oracle."""
    d = W.HUBERT_DIMS["contentvec"]
    sd = W.make_hubert_state(d, 1)
    e = SVCEngine(C.load_config(), 0, hubert_state=sd, hubert_output_layer=d["output_layer"])
    try:
        wav = np.stack([ON.synth_clip(30 + b, 2.0, 16000) for b in range(2)]).astype(np.float32)
        feats = e.hubert_encode(dev(wav)).cpu().numpy()
        with torch.no_grad():
            ref = OM.hubert_content(sd, torch.from_numpy(wav), d["output_layer"]).numpy()
        assert feats.shape == ref.shape == (2, W.hubert_frames(32000), 256)
        assert rel_l2(feats, ref) < 5e-3
    finally:
        e.close()


def test_content_split_precision(hsd, golden):
    """content_split: the HuBERT and Whisper GEMMs on split-fp16 operands land an order of magnitude closer to the
    oracle than the fp16 path (measured 3.5e-4 vs 1.1e-3 HuBERT, 1.5e-4 vs 4.1e-4 Whisper-tiny; the attention path
    stays fp16 and bounds the gain)."""
    cfg = C.load_config()
    d = W.HUBERT_DIMS["contentvec"]
    sd = W.make_hubert_state(d, 1)
    wd = W.WHISPER_DIMS["tiny-test"]
    wsd = W.make_whisper_state(wd, 0)
    wav = np.stack([ON.synth_clip(30 + b, 2.0, 16000) for b in range(2)]).astype(np.float32)
    with torch.no_grad():
        ref = OM.hubert_content(sd, torch.from_numpy(wav), d["output_layer"]).numpy()
    g = golden("whisper_logmel")
    wref = golden("whisper_encoder_tiny")["feats"]
    errs = {}
    for split in (False, True):
        e = SVCEngine(cfg, 0, hubert_state=sd, whisper_state=wsd, hubert_output_layer=d["output_layer"],
                      content_split=split)
        try:
            errs[split] = (rel_l2(e.hubert_encode(dev(wav)).cpu().numpy(), ref),
                           rel_l2(e.whisper_encode(dev(g["wav16"][None]))[0].cpu().numpy(), wref))
        finally:
            e.close()
    assert errs[False][0] < 5e-3 and errs[False][1] < 5e-3
    assert errs[True][0] < 5e-4 and errs[True][1] < 5e-4, errs
    assert errs[True][0] < errs[False][0] / 2.5 and errs[True][1] < errs[False][1] / 2, errs
