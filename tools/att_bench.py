"""Attention kernel microbenchmark (GPU): Whisper-medium shape (B = 32, L = 1500, 16 heads x 64) and HuBERT's
(L = 499, 12 heads), per-launch time of the attention kernel alone (live HIP-event profiler) and TFLOP/s (4 B L^2 D).
Timed: 5 launches right after the first (cold: the GPU's clocks still ramping, the figure of rounds 2-3) and 20 more
after ATT_BENCH_WARM (default 30) untimed warm-up launches (sustained clocks, as inside a bench step).
Usage: python tools/att_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from svc_inference_pipeline_amd import _lib  # noqa: E402


def main():
    s = torch.cuda.current_stream().cuda_stream
    for B, L, D in ((32, 1500, 1024), (32, 499, 768)):
        q, k, v = (torch.randn(B * L, D, device="cuda") for _ in range(3))
        out = torch.empty(B * L, D, device="cuda")
        args = (q.data_ptr(), k.data_ptr(), v.data_ptr(), B, L, D, out.data_ptr(), s)
        _lib.call("svc_op_attention", *args)
        torch.cuda.synchronize()

        def timed(n):
            _lib.profile_enable(True)
            for _ in range(n):
                _lib.call("svc_op_attention", *args)
            torch.cuda.synchronize()
            p = {n: x for n, x in _lib.profile_read().items() if n.startswith("attention")}
            _lib.profile_enable(False)
            return sum(x["ms"] for x in p.values()) / sum(x["launches"] for x in p.values())

        cold = timed(5)
        for _ in range(int(os.environ.get("ATT_BENCH_WARM", "30"))):
            _lib.call("svc_op_attention", *args)
        warm = timed(20)
        fl = 4.0 * B * L * L * D
        print(f"B={B} L={L} D={D}: cold {cold * 1e3:8.1f} us/launch ({fl / (cold * 1e-3) / 1e12:6.1f} TFLOP/s), "
              f"warm {warm * 1e3:8.1f} us/launch ({fl / (warm * 1e-3) / 1e12:6.1f} TFLOP/s)", flush=True)


if __name__ == "__main__":
    main()
