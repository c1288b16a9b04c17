"""Per-stream idle time inside the DiffSVC sampler from a rocprofv3 kernel trace: for each stream, the summed gaps
between its consecutive kernels (all, and those > 200 us), between the first and the last gate-GEMM launch.
Usage: python tools/stream_gaps.py <rocprofv3 -d directory>"""
import collections
import csv
import glob
import os
import sys


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows)
    g4 = [e for e in ev if "conv_gemm4" in e[3] or "gate_ws" in e[3]]
    t0, t1 = g4[0][0], g4[-1][1]
    by = collections.defaultdict(list)
    for s, e, q, _ in ev:
        if t0 <= s <= t1:
            by[q].append((s, e))
    print(f"sampler span {(t1 - t0) / 1e6:.1f} ms")
    for q, lst in sorted(by.items()):
        busy = sum(e - s for s, e in lst)
        gaps = [lst[i + 1][0] - lst[i][1] for i in range(len(lst) - 1)]
        big = [g for g in gaps if g > 200_000]
        print(f"stream {q}: {len(lst)} kernels, busy {busy / 1e6:.1f} ms, gaps {sum(gaps) / 1e6:.1f} ms "
              f"({len(big)} over 200 us: {sum(big) / 1e6:.1f} ms)")


if __name__ == "__main__":
    main()
