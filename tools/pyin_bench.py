"""pYIN F0 on the GPU (svc_f0_pyin) for the headline batch shape (32 x 10 s at 24 kHz): launch time per batch, frames
per second, against the CPU restatement (oracle/pyin.py, one clip). Usage: python tools/pyin_bench.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402
from svc_inference_pipeline_amd.synth import synth_clip  # noqa: E402


def main():
    cfg = C.load_config()
    eng = SVCEngine(cfg, 0)
    B, secs = 32, 10.0
    wav = torch.from_numpy(np.stack([synth_clip(i, secs, cfg.fs) for i in range(B)])).cuda()
    for _ in range(2):
        eng.f0_pyin(wav)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 5
    for _ in range(n):
        f0 = eng.f0_pyin(wav)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    frames = f0.shape[0] * f0.shape[1]
    print(f"GPU svc_f0_pyin: {B} x {secs:.0f} s: {ms:.2f} ms per batch, {frames / ms * 1e3 / 1e6:.2f} M frames/s, "
          f"{B * secs / (ms / 1e3):.0f} audio-s/s", flush=True)
    from oracle import pyin as PY
    x = synth_clip(0, secs, cfg.fs)
    t0 = time.perf_counter()
    PY.f0_pyin(x, cfg.fs, cfg.win_length, cfg.hop_length, cfg.f0_min, cfg.f0_max)
    dt = time.perf_counter() - t0
    print(f"CPU oracle/pyin.py: 1 x {secs:.0f} s in {dt:.2f} s = {secs / dt:.2f} audio-s/s (1 thread, numpy)")
    eng.close()


if __name__ == "__main__":
    main()
