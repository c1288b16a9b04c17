"""Extract the reference's normalisation / F0 statistics WITHOUT unpickling.

The reference ships three pickles of numpy arrays:
  config/mel_min.pkl, config/mel_max.pkl  -> np.float32[100]   (utils/acoustic_feature_extraction.py:66-72)
  config/f0.pkl                           -> list of np.float64[*] (utils/acoustic_feature_extraction.py:21-30)

Loading them with `pickle` would execute code from the file, so this script walks the pickle opcode
stream with `pickletools.genops` (a pure parser: nothing from the file is executed) and reads the raw
little-endian payloads of the BINBYTES opcodes. It checks that the only globals the stream names are
numpy's ndarray reconstruction helpers and that every payload has the byte-width the dtype string says.

Output: svc_inference_pipeline_amd/config/stats.json with
  mel_min[100], mel_max[100]   float32 values (as float)
  target_f0_median             float64, = np.median(voiced frames of f0.pkl)  (acoustic_feature_extraction.py:21-30)
  target_f0_voiced_count, target_f0_total_count, target_f0_n_utts

Run once in the container that has /root/reference:  python tools/extract_config_stats.py
"""
import json
import os
import pickletools
import sys

import numpy as np

REF = os.environ.get("SVC_REFERENCE", "/root/reference")
ALLOWED_STRINGS = {"numpy.core.multiarray", "_reconstruct", "numpy", "ndarray", "dtype", "f4", "f8", "<", "b"}


def payloads(path):
    data = open(path, "rb").read()
    dtype = None
    out = []
    for op, arg, _ in pickletools.genops(data):
        if op.name in ("SHORT_BINUNICODE", "BINUNICODE", "UNICODE"):
            if arg not in ALLOWED_STRINGS:
                raise ValueError(f"{path}: unexpected global/string {arg!r} in pickle stream")
            if arg in ("f4", "f8"):
                dtype = arg
        elif op.name in ("GLOBAL", "INST"):
            raise ValueError(f"{path}: unexpected opcode {op.name}")
        elif op.name in ("BINBYTES", "SHORT_BINBYTES", "BINBYTES8"):
            if len(arg) <= 1:  # the b'b' marker argument of ndarray._reconstruct
                continue
            if dtype is None:
                raise ValueError(f"{path}: payload before dtype")
            width = 4 if dtype == "f4" else 8
            if len(arg) % width:
                raise ValueError(f"{path}: payload not a multiple of {width}")
            out.append(np.frombuffer(arg, dtype="<" + dtype).copy())
    return out


def main():
    mel_min = payloads(os.path.join(REF, "config/mel_min.pkl"))
    mel_max = payloads(os.path.join(REF, "config/mel_max.pkl"))
    assert len(mel_min) == 1 and mel_min[0].shape == (100,), [a.shape for a in mel_min]
    assert len(mel_max) == 1 and mel_max[0].shape == (100,)
    f0s = payloads(os.path.join(REF, "config/f0.pkl"))
    total = np.concatenate(f0s)
    voiced = total[total != 0]
    stats = {
        "source": "extracted by tools/extract_config_stats.py from the reference's config/*.pkl via pickletools (no unpickling)",
        "mel_min": [float(v) for v in mel_min[0]],
        "mel_max": [float(v) for v in mel_max[0]],
        "target_f0_median": float(np.median(voiced)),
        "target_f0_voiced_count": int(voiced.size),
        "target_f0_total_count": int(total.size),
        "target_f0_n_utts": len(f0s),
    }
    dst = os.path.join(os.path.dirname(__file__), "..", "svc_inference_pipeline_amd", "config", "stats.json")
    with open(dst, "w") as f:
        json.dump(stats, f, indent=1)
    print({k: v for k, v in stats.items() if not isinstance(v, list)})
    print("mel_min[:3]", stats["mel_min"][:3], "mel_max range", min(stats["mel_max"]), max(stats["mel_max"]))


if __name__ == "__main__":
    sys.exit(main())
