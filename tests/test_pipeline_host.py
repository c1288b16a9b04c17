"""CPU: host logic of the pipeline without a GPU — ragged bucketing (F3) and content-type column order."""
import types

import pytest
import torch

from svc_inference_pipeline_amd.pipeline import SVCPipeline


def test_convert_many_buckets_by_length_and_keeps_order():
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
    outs = pipe.convert_many(w24, w16, [0, 1, 2, 3, 4], utt_ids=[10, 11, 12, 13, 14])
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
