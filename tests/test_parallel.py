"""CPU: the per-utterance data-parallel path (svc_inference_pipeline_amd/parallel.py) with world_size 2
over gloo — sharding, the length exchange and the final gather to rank 0, max-over-ranks timing."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from svc_inference_pipeline_amd.parallel import DistContext, shard


@pytest.mark.parametrize("n,world", [(256, 8), (10, 3), (3, 4), (32, 1), (0, 2)])
def test_shard_covers_all(n, world):
    spans = [shard(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0 and a1 >= a0
    assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_items, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    d = DistContext.from_env(backend="gloo")
    a, b = shard(n_items, rank, world)
    # each utterance's "waveform" is a function of its global id only (as the sampler noise is)
    wav = torch.stack([torch.arange(16, dtype=torch.float32) + 100 * u for u in range(a, b)]) if b > a else \
        torch.zeros(0, 16)
    t = d.max_over_ranks(float(rank + 1))
    out = d.gather_waveforms(wav)
    d.barrier()
    q.put((rank, t, None if out is None else out.numpy()))
    d.close()


@pytest.mark.parametrize("n_items", [8, 5])
def test_gather_world2_gloo(n_items):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n_items, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, t, out = q.get(timeout=120)
        res[r] = (t, out)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert all(res[r][0] == 2.0 for r in res)  # max over ranks
    assert res[1][1] is None
    out = res[0][1]
    exp = np.stack([np.arange(16, dtype=np.float32) + 100 * u for u in range(n_items)])
    assert out.shape == exp.shape and np.array_equal(out, exp)
