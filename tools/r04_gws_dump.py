"""(debug) gate outputs of conv_gemm4 (24) and gate_ws (40) on the same synthetic operands, compared row by row."""
import os, subprocess, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for M in (93, 4685, 29984):
    for dil in (1, 8):
        outs = {}
        for v in (24, 40):
            path = f"/tmp/gd_{v}.bin"
            env = dict(os.environ, SVC_BENCH_DUMP=path, SVC_BENCH_DIL=str(dil), GEMM_BENCH_TORCH="0",
                       GEMM_BENCH_CUSTOM=f"{M},768,384,3,1")
            subprocess.run([sys.executable, os.path.join(R, "tools", "gemm_bench.py"), str(v)], env=env, check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            outs[v] = np.fromfile(path, dtype=np.float16).reshape(M, 384)
        d = outs[24] != outs[40]
        rows = np.nonzero(d.any(1))[0]
        cols = np.nonzero(d.any(0))[0]
        print(f"M={M} dil={dil}: {d.sum()} differing elements, rows {rows[:20].tolist()}{'...' if len(rows) > 20 else ''} "
              f"({len(rows)}), cols {cols[:16].tolist()} ({len(cols)}), max |d| "
              f"{np.abs(outs[24].astype(np.float32) - outs[40].astype(np.float32)).max():.3e}", flush=True)
