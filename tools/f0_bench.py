"""Praat-AC F0 on the GPU (svc_f0_ac) for the headline batch shape (32 x 10 s at 24 kHz): time per batch with HIP
events, alone on the stream.
Usage: python tools/f0_bench.py [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine, mel_frames  # noqa: E402
from svc_inference_pipeline_amd.synth import synth_clip  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    cfg = C.load_config()
    eng = SVCEngine(cfg, 0)
    B, secs = 32, 10.0
    wav = torch.from_numpy(np.stack([synth_clip(i, secs, cfg.fs) for i in range(B)])).cuda()
    T = mel_frames(wav.shape[1])
    for _ in range(3):
        f0 = eng.f0(wav, T)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f0 = eng.f0(wav, T)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    f = f0.cpu().numpy()
    print(f"svc_f0_ac {B} x {secs:.0f} s: {ms:.3f} ms per batch, "
          f"voiced {np.mean(f > 0):.3f}, checksum {float(np.sum(f)):.6f}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
