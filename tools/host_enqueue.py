"""Host-side enqueue time of the sampler vs its GPU time (GPU): is the PLMS-100 sampler launch-bound?
Prints the wall time of svc_diffsvc_sample's host call (the launches are asynchronous) and of the call + a device
synchronize, for B = 32 clips x 937 frames. Usage: python tools/host_enqueue.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402


def main():
    cfg = C.load_config()
    eng = SVCEngine(cfg, 0, mapper_state=W.make_mapper_state(cfg.mapper, seed=0))
    B, T = 32, 937
    cond = torch.randn(B, T, cfg.mapper.conditioner_size, device="cuda")
    for it in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.diffsvc_sample(cond, fast_inference=True, speedup=10)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"iter {it}: host enqueue {1e3 * (t1 - t0):.1f} ms, enqueue + GPU {1e3 * (t2 - t0):.1f} ms", flush=True)


if __name__ == "__main__":
    main()
