"""(diagnostics) gate_ws step timeline: s_memtime stamps per workgroup (svc_gemm_bench variant 40, SVC_GWS_STAMPS).
Kind 0 (second wave): 0 kernel start, 1 after its W / cp prologue loads were issued, 2 prologue barrier, 3 + k after the
barrier of step k. Kind 1 / 2 (first wave): step k before / after its ring vmcnt wait; kind 3 (second wave): step k
before its barrier."""
import os, subprocess, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for M in [int(v) for v in (sys.argv[1:] or ["29984", "14992"])]:
    path = "/tmp/gws_stamps.bin"
    env = dict(os.environ, SVC_GWS_STAMPS=path, GEMM_BENCH_TORCH="0", GEMM_BENCH_CUSTOM=f"{M},768,384,3,1")
    subprocess.run([sys.executable, os.path.join(R, "tools", "gemm_bench.py"), os.environ.get("GWS_V", "40")], env=env, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    full = np.fromfile(path, dtype=np.uint64).reshape(256, 4, 128).astype(np.int64)
    live = full[:, 0, 0] > 0
    full = full[live]
    st = full[:, 0]
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
    # per step roles: D_{k-1} = end of the previous barrier (kind 0 index 2 + k)
    fw, wt, sw, bw = [], [], [], []
    by3 = {0: [], 1: [], 2: []}  # second wave's step time by k mod 3 (its steady loop is unrolled by 3 from k = 2)
    late = {0: [], 1: [], 2: []}  # (second-wave arrival - first-wave arrival) at the step's barrier, by k mod 3
    for w in range(len(full)):
        nsub = n[w] - 4  # stamps 3..3+nsub
        for k in range(1, nsub):
            d0 = full[w, 0, 2 + k]
            a1, b2, c3, d1 = full[w, 1, k], full[w, 2, k], full[w, 3, k], full[w, 0, 3 + k]
            if min(a1, b2, c3, d1, d0) <= 0:
                continue
            fw.append(a1 - d0); wt.append(b2 - a1); sw.append(c3 - d0); bw.append(d1 - max(b2, c3))
            if k >= 2:
                by3[k % 3].append(c3 - d0)
                late[k % 3].append(c3 - b2)
    for name, v in (("first wave: MFMAs + partial write", fw), ("first wave: ring vmcnt wait", wt),
                    ("second wave: cp load + MFMAs + epilogue", sw), ("barrier release after the later arrival", bw)):
        print(f"  {name}: pctl 10/50/90", np.percentile(v, [10, 50, 90]).astype(int))
    for r in range(3):
        if by3[r]:
            print(f"  k % 3 == {r}: second wave step median {int(np.median(by3[r]))}, second minus first arrival "
                  f"median {int(np.median(late[r]))}")
