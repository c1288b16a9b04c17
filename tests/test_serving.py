"""F3: SVCServer, the streaming front end over SVCPipeline.convert_ragged. CPU tests drive the
batching policy with a stand-in pipeline (the GPU path is tests/test_gpu_ragged.py::test_server_matches_single_clips)."""
import threading
import time
from types import SimpleNamespace

import pytest
import torch

from svc_inference_pipeline_amd.serving import SVCServer


class FakePipeline:
    """convert_ragged stand-in: the 'waveform' of a clip is its samples * (singer + 1) + utt_id."""

    def __init__(self, fail_on=None):
        self.engine = SimpleNamespace(cfg=SimpleNamespace(n_fft=1024, hop_length=256), device=None)
        self.calls = []
        self.fail_on = fail_on

    def convert_ragged(self, wavs24, wavs16, singers, wavs16_float=None, utt_ids=None, **kw):
        self.calls.append((list(utt_ids), kw))
        if self.fail_on is not None and self.fail_on in utt_ids:
            raise RuntimeError("boom")
        return [w * (s + 1) + u for w, s, u in zip(wavs24, singers, utt_ids)]


def clip(n, v=1.0):
    return torch.full((n,), v)


def test_batches_by_length_and_resolves_in_order():
    p = FakePipeline()
    srv = SVCServer(p, max_batch=8, max_wait_s=0.3, length_ratio=2.0, speedup=250, seed=3)
    lens = [1000, 1100, 5000, 900, 5200]
    futs = [srv.submit(clip(n, 0.5), clip(n // 2), singer=i) for i, n in enumerate(lens)]
    outs = [f.result(timeout=10) for f in futs]
    srv.close()
    # mel frames 3, 4, 19, 3, 20: the oldest request's batch takes the clips within 2x of its length
    assert list(srv.batches) == [[0, 1, 3], [2, 4]]
    for i, (n, o) in enumerate(zip(lens, outs)):
        assert o.shape == (n,) and torch.equal(o, clip(n, 0.5) * (i + 1) + i)
    assert all(kw == dict(fast_inference=True, speedup=250, seed=3) for _, kw in p.calls)


def test_max_batch_and_explicit_ids():
    p = FakePipeline()
    with SVCServer(p, max_batch=2, max_wait_s=0.3) as srv:
        futs = [srv.submit(clip(2000), clip(1000), singer=0, utt_id=100 + i) for i in range(5)]
        res = [f.result(timeout=10) for f in futs]
    assert list(srv.batches) == [[100, 101], [102, 103], [104]]
    assert [float(r[0]) for r in res] == [101.0, 102.0, 103.0, 104.0, 105.0]


def test_full_batch_runs_without_waiting():
    p = FakePipeline()
    srv = SVCServer(p, max_batch=3, max_wait_s=30.0)
    t0 = time.monotonic()
    futs = [srv.submit(clip(3000), clip(1500), singer=1) for _ in range(3)]
    for f in futs:
        f.result(timeout=10)
    assert time.monotonic() - t0 < 10.0  # a full batch does not wait out max_wait_s
    srv.close()


def test_errors_reach_every_caller_of_the_batch_and_close_drains():
    p = FakePipeline(fail_on=1)
    srv = SVCServer(p, max_batch=4, max_wait_s=0.3)
    a = srv.submit(clip(1000), clip(500), singer=0)
    b = srv.submit(clip(1000), clip(500), singer=0)
    c = srv.submit(clip(9000), clip(4500), singer=0)
    srv.close()  # waits for the queue to drain
    with pytest.raises(RuntimeError, match="boom"):
        a.result(timeout=1)
    with pytest.raises(RuntimeError, match="boom"):
        b.result(timeout=1)
    assert c.result(timeout=1).shape == (9000,)
    with pytest.raises(RuntimeError, match="closed"):
        srv.submit(clip(1000), clip(500), singer=0)


def test_concurrent_submitters():
    p = FakePipeline()
    srv = SVCServer(p, max_batch=16, max_wait_s=0.05)
    results = {}

    def worker(k):
        for j in range(10):
            uid = k * 100 + j
            results[uid] = srv.submit(clip(1500 + 10 * j), clip(700), singer=k, utt_id=uid)

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for uid, f in results.items():
        k = uid // 100
        assert float(f.result(timeout=10)[0]) == (k + 1) + uid
    srv.close()
    assert sorted(u for b in srv.batches for u in b) == sorted(results)
    assert all(len(b) <= 16 for b in srv.batches)


def test_bad_arguments():
    with pytest.raises(ValueError):
        SVCServer(FakePipeline(), max_batch=0)
    srv = SVCServer(FakePipeline())
    with pytest.raises(ValueError):
        srv.submit(clip(0), clip(0), singer=0)
    srv.close()
