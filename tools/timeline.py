"""Kernel-trace timeline of bench steps (rocprofv3 --kernel-trace CSV): per step wall time, the GPU-busy union
(time with at least one kernel running), the idle gaps, and per-kernel-family busy time, to see whether a step is
bound by kernels or by host launch gaps. Usage: python tools/timeline.py run_kernel_trace.csv [gap_ms]"""
import collections
import csv
import re
import sys


def family(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"<.*", "", n)
    return n.split("::")[-1]


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot, gaps


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    gap_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    k = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # split into segments at host-side gaps longer than gap_ms (synchronize between steps / passes)
    segs, cur, last_end = [], [], None
    for s, e, n in k:
        if last_end is not None and s - last_end > gap_ms * 1e6:
            segs.append(cur)
            cur = []
        cur.append((s, e, n))
        last_end = e if last_end is None else max(last_end, e)
    segs.append(cur)
    for i, sg in enumerate(segs):
        wall = (max(e for _, e, _ in sg) - sg[0][0]) / 1e6
        busy, gaps = union([(s, e) for s, e, _ in sg])
        big = sorted(gaps, reverse=True)[:3]
        print(f"segment {i}: {len(sg)} kernels, wall {wall:.2f} ms, busy {busy / 1e6:.2f} ms ({100 * busy / 1e6 / max(wall, 1e-9):.1f} %), "
              f"idle gaps {len(gaps)} (sum {sum(gaps) / 1e6:.2f} ms, largest {[round(g / 1e6, 3) for g in big]})")
        if len(sg) > 1000:
            fam = collections.defaultdict(list)
            for s, e, n in sg:
                fam[family(n)].append((s, e))
            out = []
            for f, iv in fam.items():
                u, _ = union(iv)
                out.append((u, f, len(iv), sum(e - s for s, e in iv)))
            for u, f, n, tot in sorted(out, reverse=True)[:14]:
                print(f"    {f:40s} launches {n:6d}  busy-union {u / 1e6:8.2f} ms  summed {tot / 1e6:8.2f} ms")


if __name__ == "__main__":
    main()
