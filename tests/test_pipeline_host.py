"""CPU: host logic of the pipeline without a GPU — ragged bucketing (F3) and content-type column order."""
import types

import pytest
import torch

from svc_inference_pipeline_amd.pipeline import SVCPipeline


def test_convert_many_bucketed_by_length_and_keeps_order():
    calls = []
    pipe = SVCPipeline.__new__(SVCPipeline)

    def fake_convert(w24, w16, singer, fast_inference=True, speedup=10, seed=0, utt_ids=None, wav16_float=None, **kw):
        calls.append((tuple(w24.shape), singer.tolist(), utt_ids.tolist()))
        T = (w24.shape[1] + 768 - 1024) // 256 + 1
        wav = torch.stack([torch.full((T * 256,), float(u)) for u in utt_ids.tolist()])
        return types.SimpleNamespace(wav=wav)

    pipe.convert = fake_convert
    lens = [2400, 4800, 2400, 1000, 4800]
    w24 = [torch.zeros(n) for n in lens]
    w16 = [torch.zeros(n * 2 // 3) for n in lens]
    outs = pipe.convert_many(w24, w16, [0, 1, 2, 3, 4], utt_ids=[10, 11, 12, 13, 14], bucketed=True)
    assert len(calls) == 3  # three distinct lengths
    assert sorted(c[0][0] for c in calls) == [1, 2, 2]
    for i, o in enumerate(outs):
        assert o.shape[0] == ((lens[i] + 768 - 1024) // 256 + 1) * 256
        assert float(o[0]) == 10 + i  # each output came back to its own slot
    for shape, singers, uids in calls:
        assert [u - 10 for u in uids] == singers


def test_convert_many_rejects_mismatched_lists():
    pipe = SVCPipeline.__new__(SVCPipeline)
    with pytest.raises(ValueError):
        pipe.convert_many([torch.zeros(10)], [], [0])


def test_check_supported_rejects_concat_merge_mode():
    from svc_inference_pipeline_amd import config as C
    from svc_inference_pipeline_amd.runtime import check_supported
    cfg = C.load_config()
    check_supported(cfg)  # the reference config ("add") is accepted
    cfg.mapper.merge_mode = "concat"
    with pytest.raises(ValueError, match="merge_mode"):
        check_supported(cfg)


class _FakeEngine:
    """CPU stand-in for SVCEngine that records the ragged-length tables the pipeline passes to each stage."""

    def __init__(self, types=("whisper",)):
        from svc_inference_pipeline_amd import config as C
        self.cfg = C.load_config()
        self.cfg.mapper.content_feature = list(types)
        self.calls = []
        import threading
        self.lock = threading.RLock()
        self.content_dtype = torch.float16

    def mel_energy(self, w24, n_samples=None):
        self.calls.append(("mel", tuple(w24.shape), list(n_samples)))
        B, N = w24.shape
        T = (N + 768 - 1024) // 256 + 1
        return torch.zeros(B, T, 100), torch.zeros(B, T)

    def f0(self, w24, T, n_samples=None):
        self.calls.append(("f0", T, list(n_samples)))
        return torch.zeros(w24.shape[0], T, dtype=torch.float64)

    def f0_pyin(self, w24, n_samples=None, T=None):
        self.calls.append(("f0_pyin", T, list(n_samples)))
        return torch.ones(w24.shape[0], T, dtype=torch.float64)  # every frame voiced at 1 Hz

    def pitch_shift(self, f0):
        return f0

    def whisper_encode(self, w16):
        self.calls.append(("whisper", tuple(w16.shape)))
        return w16[:, :1, None].expand(-1, 1500, 1024).float().contiguous()  # utterance marker in every row

    def hubert_encode(self, w16):
        self.calls.append(("hubert", tuple(w16.shape)))
        F = (w16.shape[1] - 400) // 320 + 1
        return w16[:, :1, None].expand(-1, F, 256).float().contiguous()

    def map_content(self, feats, T, rule="whisper", out=None):
        return feats[:, :1].expand(-1, T, -1).half()

    def condition(self, content, f0, energy, singer):
        self.calls.append(("condition", tuple(content.shape), singer.tolist()))
        return content[:, :, :384].float()

    def diffsvc_sample(self, cond, fast_inference=True, speedup=10, seed=0, utt_ids=None, frames=None, **kw):
        self.calls.append(("sample", tuple(cond.shape), list(frames), utt_ids.tolist()))
        return cond[:, :, :100].clone()

    def bigvgan(self, x0, frames=None):
        self.calls.append(("bigvgan", tuple(x0.shape), list(frames)))
        B, T, _ = x0.shape
        wav = x0[:, :, :1].repeat_interleave(256, dim=1)[:, :, 0]
        for b in range(B):
            wav[b, frames[b] * 256:] = -1.0  # never returned: the pipeline trims at frames * hop
        return wav


def test_convert_many_is_one_ragged_batch(monkeypatch):
    import contextlib
    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a: types.SimpleNamespace(wait_stream=lambda s: None))
    monkeypatch.setattr(torch.cuda, "stream", lambda s: contextlib.nullcontext())
    eng = _FakeEngine()
    pipe = SVCPipeline(eng, f0_side=False)
    lens = [2400, 4800, 24000, 1000]
    w24 = [torch.zeros(n) for n in lens]
    w16 = [torch.full((n * 2 // 3,), float(i + 1)) for i, n in enumerate(lens)]  # marker = position + 1
    outs = pipe.convert_many(w24, w16, [0, 1, 2, 3], utt_ids=[10, 11, 12, 13])
    T_b = [(n + 768 - 1024) // 256 + 1 for n in lens]
    kinds = [c[0] for c in eng.calls]
    assert kinds.count("mel") == kinds.count("sample") == kinds.count("bigvgan") == 1  # one batch, not buckets
    mel = next(c for c in eng.calls if c[0] == "mel")
    assert mel[1] == (4, 24000) and mel[2] == lens
    assert next(c for c in eng.calls if c[0] == "f0")[1:] == (max(T_b), lens)
    sample = next(c for c in eng.calls if c[0] == "sample")
    assert sample[2] == T_b and sample[3] == [10, 11, 12, 13]
    assert next(c for c in eng.calls if c[0] == "bigvgan")[2] == T_b
    for i, o in enumerate(outs):
        assert o.shape == (T_b[i] * 256,)
        assert bool((o == float(i + 1)).all())  # its own content came back to its own slot, trimmed


def test_ragged_content_whisper_groups_and_hubert_buckets(monkeypatch):
    eng = _FakeEngine(types=("contentvec", "whisper"))
    eng.cfg.mapper.input_content_dim["contentvec"] = 256
    pipe = SVCPipeline(eng)
    lens16 = [16000, 32000, 16000]
    w16 = [torch.full((n,), float(i + 1)) for i, n in enumerate(lens16)]
    T_b = [94, 188, 94]
    out = pipe.ragged_content(w16, T_b, 188)
    assert out.shape == (3, 188, 256 + 1024)
    hub = [c for c in eng.calls if c[0] == "hubert"]
    assert sorted(c[1] for c in hub) == [(1, 32000), (2, 16000)]  # per exact length
    assert [c for c in eng.calls if c[0] == "whisper"] == [("whisper", (3, 32000))]  # one zero-padded batch
    for i in range(3):
        assert bool((out[i, :T_b[i]] == float(i + 1)).all()) and not out[i, T_b[i]:].any()


def test_pyin_f0_method_cuts_to_mel_frames(monkeypatch):
    """f0_method="pyin" (utils/f0.py:95-117): librosa's 1 + N // hop frames are cut to the mel frames, and the rows
    past each utterance's own frames are zero, as the Praat path leaves them."""
    import contextlib
    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a: types.SimpleNamespace(wait_stream=lambda s: None))
    monkeypatch.setattr(torch.cuda, "stream", lambda s: contextlib.nullcontext())
    eng = _FakeEngine()
    seen = {}
    cond = eng.condition
    eng.condition = lambda content, f0, energy, singer: (seen.setdefault("f0", f0), cond(content, f0, energy, singer))[1]
    pipe = SVCPipeline(eng, f0_side=False, f0_method="pyin")
    lens = [2400, 4800, 1000]
    pipe.convert_many([torch.zeros(n) for n in lens], [torch.zeros(n * 2 // 3) for n in lens], [0, 1, 2])
    T_b = [(n + 768 - 1024) // 256 + 1 for n in lens]
    call = next(c for c in eng.calls if c[0] == "f0_pyin")
    assert call == ("f0_pyin", 1 + max(lens) // 256, lens)  # librosa's frame count for the batch length
    f0 = seen["f0"]
    assert f0.shape == (3, max(T_b))
    for b, tb in enumerate(T_b):
        assert bool((f0[b, :tb] == 1).all()) and not f0[b, tb:].any()
    with pytest.raises(ValueError, match="f0_method"):
        SVCPipeline(eng, f0_method="crepe")
