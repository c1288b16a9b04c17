"""(debug) gate outputs of conv_gemm4 (24) and gate_ws (argv[1], default 40) on the
same synthetic operands, compared element by element (differing elements, max |d|, max difference in f16 units)."""
import os, subprocess, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V = int(sys.argv[1]) if len(sys.argv) > 1 else 40
for M in (93, 4685, 29984):
    for dil in (1, 8):
        outs = {}
        for v in (24, V):
            path = f"/tmp/gd_{v}.bin"
            env = dict(os.environ, SVC_BENCH_DUMP=path, SVC_BENCH_DIL=str(dil), GEMM_BENCH_TORCH="0",
                       GEMM_BENCH_CUSTOM=f"{M},768,384,3,1")
            subprocess.run([sys.executable, os.path.join(R, "tools", "gemm_bench.py"), str(v)], env=env, check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            outs[v] = np.fromfile(path, dtype=np.float16).reshape(M, 384)
        d = outs[24] != outs[V]
        rows = np.nonzero(d.any(1))[0]
        cols = np.nonzero(d.any(0))[0]
        a, b = outs[24].astype(np.float32), outs[V].astype(np.float32)
        ulp = np.abs(outs[24].view(np.int16).astype(np.int32) - outs[V].view(np.int16).astype(np.int32))  # (same sign)
        print(f"M={M} dil={dil} v{V}: {d.sum()} differing elements of {d.size}, rows {rows[:12].tolist()}"
              f"{'...' if len(rows) > 12 else ''} ({len(rows)}), cols ({len(cols)}), max |d| {np.abs(a - b).max():.3e}, "
              f"max f16 units {ulp.max()}", flush=True)
