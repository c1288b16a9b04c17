"""Activation1d microbenchmark (GPU): achieved GB/s of each activation1d kernel form (kernel switch act_variant) on the BigVGAN stage shapes
(B = 32 clips x 10 s). Algorithmic bytes = 4 (f32 in) + 2 (f16 out) per element.
Usage: python tools/act_bench.py [variant ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from svc_inference_pipeline_amd import _lib  # noqa: E402
from svc_inference_pipeline_amd._lib import call, profile_enable, profile_read  # noqa: E402

SHAPES = [(32, 3748, 768), (32, 14992, 384), (32, 29984, 192), (32, 119936, 48), (32, 239872, 24)]


def main():
    variants = sys.argv[1:] or ["0", "1", "2", "3", "4"]
    s = torch.cuda.current_stream().cuda_stream
    for B, L, C in SHAPES:
        x = torch.randn(B * L, C, device="cuda")
        y = torch.empty(B * L, C, device="cuda")
        al = torch.randn(C, device="cuda") * 0.3
        be = torch.randn(C, device="cuda") * 0.3
        f = torch.rand(12, device="cuda")
        row = []
        for v in variants:
            _lib.tune(None, act_variant=int(v))
            args = (x.data_ptr(), B, L, C, al.data_ptr(), be.data_ptr(), f.data_ptr(), y.data_ptr(), s)
            call("svc_op_activation1d", *args)
            torch.cuda.synchronize()
            profile_enable(True)  # per-launch HIP events around the activation kernel alone
            for _ in range(10):
                call("svc_op_activation1d", *args)
            torch.cuda.synchronize()
            p = {k: v for k, v in profile_read().items() if k.startswith("activation1d")}
            profile_enable(False)
            ms = sum(v["ms"] for v in p.values()) / sum(v["launches"] for v in p.values())
            row.append(f"v{v}: {ms * 1000:7.1f} us {B * L * C * 6 / ms / 1e6:6.0f} GB/s")
        print(f"L={L:6d} C={C:4d}", " | ".join(row), flush=True)
        del x, y


if __name__ == "__main__":
    main()
