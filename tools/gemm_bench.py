"""GEMM kernel microbenchmark (GPU): TFLOP/s of the implicit-GEMM variants on the hot-path shapes.
Usage: python tools/gemm_bench.py [variant ...]   (30: res_proj.hip, on the split residual shapes only)
GEMM_BENCH_WARM=1: each measurement (ours and torch.mm) follows 30 untimed launches of the same GEMM, so it is taken at
sustained clocks (the default times 10 launches after 2 warm-ups, while the clocks may still be ramping).
GEMM_BENCH_COLD=1: each launch after a 1 GiB memset (operands not cache-resident, as in the sampler)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svc_inference_pipeline_amd import _lib  # noqa: E402

SHAPES = [  # name, M, N, Cin, taps, epi
    ("diffsvc.dilated(gate)", 29984, 768, 384, 3, 1),
    ("diffsvc.dilated(store)", 29984, 768, 384, 3, 0),
    ("diffsvc.outproj(res)", 29984, 384, 384, 1, 0),
    ("diffsvc.outproj(rmw)", 29984, 384, 384, 1, 2),   # with the real epilogue: f32 residual RMW + next f16 input
    ("diffsvc.outproj(rmw,sub)", 9995, 384, 384, 1, 2),
    ("diffsvc.outproj(split)", 29984, 384, 384, 1, 6),  # the default split-fp16 residual RMW (hi / lo halves)
    ("diffsvc.outproj(split,sub)", 9995, 384, 384, 1, 6),
    ("diffsvc.outproj(split,sub2)", 14992, 384, 384, 1, 6),  # 2-stream sampler sub-batch
    ("diffsvc.skipsum", 29984, 384, 7680, 1, 0),
    ("bigvgan.s2 k11", 32 * 14992, 384, 384, 11, 0),
    ("whisper.fc1", 48000, 4096, 1024, 1, 0),
    ("whisper.fc2", 48000, 1024, 4096, 1, 0),
    ("whisper.qkv", 48000, 3072, 1024, 1, 0),
    ("whisper.out", 48000, 1024, 1024, 1, 0),
    ("bigvgan.s3 k11 (C192)", 32 * 29984, 192, 192, 11, 0),
    ("bigvgan.s4 k11 (C96)", 32 * 59968, 96, 96, 11, 0),
    ("bigvgan.s1 k11", 32 * 3748, 768, 768, 11, 0),
    ("square 8192", 8192, 8192, 8192, 1, 0),
]


def main():
    variants = [int(v) for v in sys.argv[1:]] or [-1, 15, 24]
    import torch
    torch.cuda.init()
    only = os.environ.get("GEMM_BENCH_SHAPES")
    shapes = SHAPES
    if os.environ.get("GEMM_BENCH_CUSTOM"):  # "M,N,Cin,taps,epi;..." (e.g. a K sweep)
        shapes = [(f"custom {c}",) + tuple(int(v) for v in c.split(",")) for c in os.environ["GEMM_BENCH_CUSTOM"].split(";")]
    for name, M, N, Cin, taps, epi in shapes:
        if only and not any(o in name for o in only.split(",")):
            continue
        row = []
        for v in variants:
            if v < 0 and epi == 1:  # v1 has no paired gate epilogue
                continue
            ms = ctypes.c_double()
            # GEMM_BENCH_COLD=1: each launch after a 1 GiB memset (operands not cache-resident, as in the sampler)
            iters = -10 if os.environ.get("GEMM_BENCH_COLD") == "1" else 10
            try:
                if os.environ.get("GEMM_BENCH_WARM") == "1":
                    _lib.call("svc_gemm_bench", M, N, Cin, taps, epi, v, 30, ctypes.byref(ms))
                _lib.call("svc_gemm_bench", M, N, Cin, taps, epi, v, iters, ctypes.byref(ms))
            except _lib.SVCError as err:  # the library rejects this (variant, epilogue) pair before launching
                row.append(f"v{v}: {'n/a':>27s}")
                if os.environ.get("GEMM_BENCH_VERBOSE"):
                    print(f"  (v{v} on {name}: {err})", file=sys.stderr)
                continue
            tf = 2.0 * M * N * Cin * taps / (ms.value * 1e-3) / 1e12
            row.append(f"v{v}: {ms.value * 1000:8.1f} us {tf:7.1f} TF")
        if os.environ.get("GEMM_BENCH_TORCH", "1") == "1":
            # hipBLASLt yardstick (plain GEMM, K = taps * Cin, no epilogue), same shape
            a = torch.randn(M, Cin * taps, device="cuda", dtype=torch.float16)
            b = torch.randn(Cin * taps, N, device="cuda", dtype=torch.float16)
            for _ in range(30 if os.environ.get("GEMM_BENCH_WARM") == "1" else 1):
                torch.mm(a, b)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                torch.mm(a, b)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            row.append(f"torch.mm: {ms * 1000:8.1f} us {2.0 * M * N * Cin * taps / (ms * 1e-3) / 1e12:7.1f} TF")
            del a, b
        print(f"{name:24s}", " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
