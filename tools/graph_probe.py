"""Probe (GPU): the PLMS-100 sampler (B = 32 x 937 frames) launched directly vs replayed from a HIP graph captured
through torch.cuda.graph, for several kernel-switch settings: how much of the sampler's time is launch / dependency
gaps. Usage: python tools/graph_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402


def timed(fn, n=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    cfg = C.load_config()
    eng = SVCEngine(cfg, 0, mapper_state=W.make_mapper_state(cfg.mapper, seed=0))
    B, T = 32, 937
    cond = torch.randn(B, T, cfg.mapper.conditioner_size, device="cuda")
    uid = torch.arange(B, device="cuda", dtype=torch.int32)
    for sw in ({}, {"gemm4_rmw": 1}, {"sampler_streams": 1}, {"sampler_streams": 1, "gemm4_rmw": 1},
               {"sampler_streams": 2}):
        eng.tune(reset=1)
        eng.tune(**sw)
        run = lambda: eng.diffsvc_sample(cond, fast_inference=True, speedup=10, seed=7, utt_ids=uid)
        direct = timed(run)
        ref = run().clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            run()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = run()
        graph = timed(g.replay)
        same = bool(torch.equal(out, ref))
        print(f"{sw}: direct {direct:.1f} ms, graph replay {graph:.1f} ms, identical {same}", flush=True)
        del g


if __name__ == "__main__":
    main()
