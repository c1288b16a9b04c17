"""DiffSVC denoiser microbenchmark (GPU): one epsilon prediction (svc_diffsvc_eps) on B clips of T frames,
fused residual-layer kernel (SVC_DIFF_FUSED=1, default) or the unfused GEMM path (=0). Prints ms per call and the
per-kernel breakdown of one profiled call. Usage: python tools/layer_bench.py [B] [T] [iters]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svc_inference_pipeline_amd import _lib  # noqa: E402
from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd import weights as W  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 937
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    cfg = C.load_config()
    cfg.mapper.input_content_dim["whisper"] = 1024
    e = SVCEngine(cfg, 0, mapper_state=W.make_mapper_state(cfg.mapper, 0))
    rng = np.random.default_rng(0)
    cond = torch.from_numpy(rng.standard_normal((B, T, 384)).astype(np.float32)).cuda()
    x = torch.from_numpy(rng.standard_normal((B, T, 100)).astype(np.float32)).cuda()
    e.diffsvc_eps(cond, x, 500)
    torch.cuda.synchronize()
    _lib.profile_enable(True)
    e.diffsvc_eps(cond, x, 500)
    torch.cuda.synchronize()
    prof = _lib.profile_read()
    _lib.profile_enable(False)
    t0 = time.time()
    for _ in range(iters):
        e.diffsvc_eps(cond, x, 500)
    torch.cuda.synchronize()
    dt = (time.time() - t0) / iters
    print(f"B={B} T={T} fused={os.environ.get('SVC_DIFF_FUSED', '1')}: {dt * 1e3:.3f} ms per eps call "
          f"(includes the hoisted conditioner projection)")
    for k, v in sorted(prof.items(), key=lambda kv: -kv[1]["ms"]):
        tf = v["flops"] / max(v["ms"], 1e-9) / 1e9 if v["flops"] else 0
        print(f"  {k:40s} {v['ms'] * 1e3 / v['launches']:9.1f} us x {v['launches']:3d}  {tf:7.1f} TF/s")
    e.close()


if __name__ == "__main__":
    main()
