"""Fused BigVGAN activation + conv (amp_conv) microbenchmark (GPU): per-launch time of each (C, k, d) on the stage
shapes (B = 32 clips x 10 s). Usage: python tools/amp_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from svc_inference_pipeline_amd._lib import call, profile_enable, profile_read  # noqa: E402

SHAPES = [(48, 119936), (24, 239872)] + ([(96, 59968)] if os.environ.get("AMP_BENCH_C96") else [])


def main():
    s = torch.cuda.current_stream().cuda_stream
    B = 32
    for C, L in SHAPES:
        x = torch.randn(B * L, C, device="cuda")
        y = torch.empty(B * L, C, device="cuda")
        al = torch.randn(C, device="cuda") * 0.3
        be = torch.randn(C, device="cuda") * 0.3
        f = torch.rand(12, device="cuda")
        bias = torch.zeros(C, device="cuda")
        for k in (3, 7, 11):
            w = torch.randn(C, C, k, device="cuda") * 0.05
            for d in ((1, 3, 5) if k > 1 else (1,)):
                row = []
                for _rep in range(2):
                    args = (x.data_ptr(), B, L, C, al.data_ptr(), be.data_ptr(), f.data_ptr(), w.data_ptr(),
                            bias.data_ptr(), k, d, None, y.data_ptr(), s)
                    call("svc_op_amp_conv", *args)
                    torch.cuda.synchronize()
                    profile_enable(True)
                    for _ in range(5):
                        call("svc_op_amp_conv", *args)
                    torch.cuda.synchronize()
                    p = {n: v for n, v in profile_read().items() if n.startswith("amp_conv")}
                    profile_enable(False)
                    us = 1000 * sum(v["ms"] for v in p.values()) / sum(v["launches"] for v in p.values())
                    row.append(f"{us:7.1f} us")
                print(f"C={C} L={L} k={k:2d} d={d}:", " | ".join(row), flush=True)
        del x, y


if __name__ == "__main__":
    main()
