"""24 kHz DFT + mel + energy kernel timing (svc_mel_energy) on B = 32 x 10 s synthetic clips, with the diagnostic
phase cuts of the dft_dbg kernel switch (1 = no DFT loop, 2 = no filterbank phase, 3 = no frame loads).
Usage: python tools/dft_time.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from svc_inference_pipeline_amd import config as C  # noqa: E402
from svc_inference_pipeline_amd.runtime import SVCEngine  # noqa: E402
from svc_inference_pipeline_amd.synth import synth_clip  # noqa: E402


def main():
    eng = SVCEngine(C.load_config(), 0)
    wav = torch.from_numpy(np.stack([synth_clip(i, 10.0, 24000) for i in range(32)])).cuda()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for mode in (0, 1, 2, 3, 0):
        eng.tune(dft_dbg=mode)
        eng.mel_energy(wav)
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(10):
            eng.mel_energy(wav)
        ev[1].record()
        torch.cuda.synchronize()
        print("dft_dbg", mode, round(ev[0].elapsed_time(ev[1]) / 10 * 1000, 1), "us", flush=True)


if __name__ == "__main__":
    main()
