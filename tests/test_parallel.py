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


def _worker_ragged(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    d = DistContext.from_env(backend="gloo")
    # rank 0: 3 utterances of 10 samples; rank 1: 1 utterance of 17 samples (different B and S per rank)
    n, s = (3, 10) if rank == 0 else (1, 17)
    wav = torch.stack([torch.arange(s, dtype=torch.float32) + 1000 * (rank * 10 + i) for i in range(n)])
    out, lens = d.gather_waveforms(wav, return_lengths=True)
    q.put((rank, None if out is None else out.numpy(), None if lens is None else lens.numpy()))
    d.close()


def test_gather_unequal_lengths_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_ragged, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, out, lens = q.get(timeout=120)
        res[r] = (out, lens)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert res[1] == (None, None)
    out, lens = res[0]
    assert out.shape == (4, 17) and lens.tolist() == [10, 10, 10, 17]
    for row, (rk, i, s) in enumerate([(0, 0, 10), (0, 1, 10), (0, 2, 10), (1, 0, 17)]):
        exp = np.arange(s, dtype=np.float32) + 1000 * (rk * 10 + i)
        assert np.array_equal(out[row, :s], exp) and not out[row, s:].any()


def _bench(tmp_path, gpus, name):
    """bench.py's own rank spawn (no torchrun, WORLD_SIZE unset) in --dry-run mode on the CPU over gloo."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dump = str(tmp_path / f"{name}.npy")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", str(gpus), "--dry-run", "--batch",
                        "3", "--seconds", "0.25", "--steps", "2", "--dump", dump], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    return json.loads(lines[0]), np.load(dump)


def test_bench_spawn_dry_run_world2_matches_world1(tmp_path):
    line2, out2 = _bench(tmp_path, 2, "w2")
    assert line2["dist_world"] == 2 and line2["backend"] == "gloo" and len(line2["per_rank_s"]) == 2
    # the process group's own size and each rank's gather time per step (bench.py reports both on the GPU line too)
    assert line2["rccl_world"] == 2 and len(line2["gather_ms_per_step"]) == 2
    assert all(v >= 0 for v in line2["gather_ms_per_step"])
    assert line2["gathered"][0] == 6
    # world 1 with the whole batch (6 utterances, ids 0..5) must gather identical waveforms
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dump = str(tmp_path / "w1.npy")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "1", "--dry-run", "--batch", "6",
                        "--seconds", "0.25", "--steps", "1", "--dump", dump], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out1 = np.load(dump)
    assert out1.shape == out2.shape and np.array_equal(out1, out2)


def test_bench_rejects_world_mismatch():
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "4", "--dry-run"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


@pytest.mark.parametrize("fault", ["raise", "hang"])
def test_bench_spawn_rank_failure_ends_job(tmp_path, fault):
    """A rank that raises mid-run, or hangs without exiting, ends the whole world-2 job with a non-zero status within
    the collective timeout: the raising rank exits and spawn_ranks kills its peer; with a hanging rank, the peer's
    gather times out (DistContext collective timeout), it exits non-zero, and spawn_ranks kills the hung rank."""
    import subprocess
    import sys
    import time
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry-run", "--batch", "2",
                        "--seconds", "0.25", "--steps", "3", "--fault", fault, "--dist-timeout", "15"], env=env,
                       capture_output=True, text=True, timeout=200)
    assert r.returncode != 0
    assert time.time() - t0 < 150
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]  # no result line from a failed job


def test_gather_one_dimensional_world1():
    """gather_waveforms takes a 1-D waveform as one utterance (world 1 returns it as [1, S] with its length)."""
    d = DistContext()
    out, lens = d.gather_waveforms(torch.arange(7, dtype=torch.float32), return_lengths=True)
    assert out.shape == (1, 7) and lens.tolist() == [7]
    with pytest.raises(ValueError):
        d.gather_waveforms(torch.zeros(2, 3, 4))
