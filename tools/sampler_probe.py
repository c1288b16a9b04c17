"""Probe (GPU): PLMS-100 sampler (B = 32 x 937 frames) wall time and per kernel@site times (live HIP-event
profiler) under kernel-switch settings given as JSON dicts on the command line, e.g.
python tools/sampler_probe.py '{}' '{"sampler_streams": 1}'"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from svc_inference_pipeline_amd import _lib  # noqa: E402
from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402


def main():
    cfg = C.load_config()
    eng = SVCEngine(cfg, 0, mapper_state=W.make_mapper_state(cfg.mapper, seed=0))
    B, T = 32, 937
    cond = torch.randn(B, T, cfg.mapper.conditioner_size, device="cuda")
    uid = torch.arange(B, device="cuda", dtype=torch.int32)
    run = lambda: eng.diffsvc_sample(cond, fast_inference=True, speedup=10, seed=7, utt_ids=uid)
    for arg in sys.argv[1:] or ["{}"]:
        sw = json.loads(arg)
        eng.tune(reset=1)
        eng.tune(**sw)
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / 3 * 1e3
        _lib.profile_enable(True)
        run()
        torch.cuda.synchronize()
        prof = _lib.profile_read()
        _lib.profile_enable(False)
        print(f"{sw}: wall {wall:.1f} ms", flush=True)
        for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"])[:8]:
            print(f"    {k:48s} {v['ms']:8.2f} ms  {v['launches']:5d} launches  {1e3 * v['ms'] / v['launches']:7.1f} us/launch",
                  flush=True)


if __name__ == "__main__":
    main()
