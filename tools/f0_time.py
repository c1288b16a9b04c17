"""F0 (Praat AC) kernel timing on B = 32 x 10 s synthetic clips, with the diagnostic phase cuts of the f0_dbg kernel switch
(1 = autocorrelation only, 2 = no Brent refinement). Usage: python tools/f0_time.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402
from svc_inference_pipeline_amd.synth import synth_clip  # noqa: E402


def main():
    eng = SVCEngine(C.load_config(), 0)
    wav = torch.from_numpy(np.stack([synth_clip(i, 10.0, 24000) for i in range(32)])).cuda()
    T = (wav.shape[1] + 768 - 1024) // 256 + 1
    for mode in ("", "1", "2", ""):
        eng.tune(f0_dbg=int(mode or 0))
        eng.f0(wav, T)
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(3):
            eng.f0(wav, T)
        torch.cuda.synchronize()
        print("mode", mode or "full", round((time.time() - t0) / 3 * 1000, 2), "ms", flush=True)


if __name__ == "__main__":
    main()
