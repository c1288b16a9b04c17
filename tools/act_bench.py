"""BigVGAN Activation1d microbenchmark (GPU): per-launch time of activation1d on the generator's C >= 96 stage shapes
(B = 32 clips x 10 s; f32 input = the residual stream, f16 input = an AMPBlock1 convs1 output), with the achieved
algorithmic HBM rate. Usage: python tools/act_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from svc_inference_pipeline_amd._lib import call, profile_enable, profile_read  # noqa: E402

SHAPES = [(768, 3748), (384, 14992), (192, 29984), (96, 59968)]


def main():
    s = torch.cuda.current_stream().cuda_stream
    B = 32
    for C, L in SHAPES:
        al = torch.randn(C, device="cuda") * 0.3
        be = torch.randn(C, device="cuda") * 0.3
        f = torch.rand(12, device="cuda")
        y = torch.empty(B * L, C, device="cuda")
        for x16 in (False, True):
            x = torch.randn(B * L, C, device="cuda", dtype=torch.float16 if x16 else torch.float32)
            name = "svc_op_activation1d_x16" if x16 else "svc_op_activation1d"
            args = (x.data_ptr(), B, L, C, al.data_ptr(), be.data_ptr(), f.data_ptr(), y.data_ptr(), s)
            row = []
            for _rep in range(2):
                call(name, *args)
                torch.cuda.synchronize()
                profile_enable(True)
                for _ in range(5):
                    call(name, *args)
                torch.cuda.synchronize()
                p = profile_read()["activation1d"]
                profile_enable(False)
                us = 1000 * p["ms"] / p["launches"]
                row.append(f"{us:7.1f} us {p['bytes'] / p['launches'] / (us * 1e-6) / 1e12:4.2f} TB/s")
            print(f"C={C:4d} L={L} {'f16' if x16 else 'f32'}:", " | ".join(row), flush=True)
            del x
        del y


if __name__ == "__main__":
    main()
