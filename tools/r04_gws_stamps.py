"""(diagnostics) gate_ws step timeline: s_memtime stamps per workgroup (svc_gemm_bench variant 40, SVC_GWS_STAMPS).
Stamp 0: kernel start (second wave), 1: after its W / cp prologue loads were issued, 2: prologue barrier, 3: end of
step 0, 4 + j: end of the step that finished block j."""
import os, subprocess, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for M in [int(v) for v in (sys.argv[1:] or ["29984", "14992"])]:
    path = "/tmp/gws_stamps.bin"
    env = dict(os.environ, SVC_GWS_STAMPS=path, GEMM_BENCH_TORCH="0", GEMM_BENCH_CUSTOM=f"{M},768,384,3,1")
    subprocess.run([sys.executable, os.path.join(R, "tools", "gemm_bench.py"), "40"], env=env, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    st = np.fromfile(path, dtype=np.uint64).reshape(256, 128).astype(np.int64)
    live = st[:, 0] > 0
    st = st[live]
    t0 = st[:, 0].min()
    rel = np.where(st > 0, st - t0, -1)
    n = (rel >= 0).sum(1)
    print(f"M={M}: {live.sum()} workgroups, stamps per wg {n.min()}..{n.max()} (clock ticks of s_memtime = shader clock)")
    print("  start spread:", np.percentile(rel[:, 0], [0, 50, 100]))
    print("  prologue loads issued:", np.percentile(rel[:, 1] - rel[:, 0], [0, 50, 100]))
    print("  prologue barrier:", np.percentile(rel[:, 2] - rel[:, 0], [0, 50, 100]))
    print("  step 0:", np.percentile(rel[:, 3] - rel[:, 2], [0, 50, 100]))
    steps = []
    for w in range(len(rel)):
        k = n[w]
        d = np.diff(rel[w, 3:k])
        steps.append(d)
    alls = np.concatenate(steps)
    print("  per step (ticks) pctl 10/50/90/max:", np.percentile(alls, [10, 50, 90, 100]))
    print("  first 12 steps median:", [int(np.median([s[i] for s in steps if len(s) > i])) for i in range(12)])
    print("  end (last stamp) spread:", np.percentile([rel[w, n[w] - 1] for w in range(len(rel))], [0, 50, 100]))
