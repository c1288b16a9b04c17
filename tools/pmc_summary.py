"""Summarise a tools/gpu_profile.sh run into profiles/: kernel stats CSV + per-launch HBM traffic.

HBM bytes per dispatch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: on gfx950 FETCH_SIZE reports exactly
half of the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md, HBM section), WRITE_SIZE is
exact for 16-B/lane stores (our epilogue stores are narrower: treat it as an estimate), both in KiB.
Infinity-Cache hits are counted as fetches, so the figure is an upper bound on DRAM traffic.
One kernel can serve launches of different sizes (conv_gemm4<128,128,pair> runs both the sampler's sub-batch
launches and the full-batch launches of bench.py's single-stream roofline pass), so traffic and the rocprof trace
durations are also split by grid size; a kernel's headline `hbm_bytes_per_launch` is that of its LARGEST grid, which
is the roofline pass's full-batch launch. (gate_ws<16x128> runs a fixed 256-workgroup grid at every size: with one
sampler stream every launch of it is a full batch.)
Usage: python tools/pmc_summary.py gpurun_out/<tag> profiles/<round-prefix>
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

NAME_MAP = {
    "attention_kernel": "attention",
    "activation1d_kernel": "activation1d",
}


def short(name):
    """Demangled kernel name -> the tag bench.py's live profile uses (libsvc_hip prof_begin names)."""
    m = re.search(r"conv_gemm3_kernel<(\d+), (\d+), (true|false), (true|false)", name)
    if m:
        return f"conv_gemm3<{m.group(1)},{m.group(2)}{',pair' if m.group(4) == 'true' else ''}>"
    m = re.search(r"conv_gemm3_kernelILi(\d+)ELi(\d+)ELb([01])ELb([01])E", name)  # rocprof keeps these mangled
    if m:
        return f"conv_gemm3<{m.group(1)},{m.group(2)}{',pair' if m.group(4) == '1' else ''}>"
    m = re.search(r"conv_gemm4_kernel<(true|false), (true|false), (true|false)", name)
    if m:
        return f"conv_gemm4<128,128{',gate' if m.group(3) == 'true' else ',pair' if m.group(2) == 'true' else ''}>"
    m = re.search(r"conv_gemm4_kernelILb([01])ELb([01])ELb([01])E", name)
    if m:
        return f"conv_gemm4<128,128{',gate' if m.group(3) == '1' else ',pair' if m.group(2) == '1' else ''}>"
    m = re.search(r"activation1d_rs_kernel", name)
    if m:
        return "activation1d"
    if "res_proj_kernel" in name:
        return "res_proj<16x192>"
    if "gate_ws_kernel" in name:
        return "gate_ws<16x128>"
    for k, v in NAME_MAP.items():
        if k in name:
            return v
    return name


def counter_rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


WG_SIZE = {}  # kernel tag -> threads per workgroup, from the counter rows


def per_kernel(rows, counter):
    """{kernel tag: {grid size in threads: [counter value per dispatch]}}"""
    acc = {}
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        k = short(r.get("Kernel_Name", ""))
        WG_SIZE[k] = int(r.get("Workgroup_Size") or 256)
        acc.setdefault(k, {}).setdefault(int(r.get("Grid_Size", 0)), []).append(float(r["Counter_Value"]))
    return acc


def trace_by_grid(src):
    """{kernel tag: {grid: (dispatches, average ns)}} from the rocprofv3 kernel trace."""
    files = glob.glob(os.path.join(src, "trace", "**", "*kernel_trace.csv"), recursive=True)
    acc = {}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
                acc.setdefault(k, {}).setdefault(g, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {k: {g: (len(v), sum(v) / len(v)) for g, v in d.items()} for k, d in acc.items()}


def mean(v):
    return sum(v) / len(v) if v else 0.0


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], dst + "_kernel_stats.csv")
    fetch = per_kernel(counter_rows(os.path.join(src, "pmc_fetch")), "FETCH_SIZE")
    write = per_kernel(counter_rows(os.path.join(src, "pmc_write")), "WRITE_SIZE")
    out = {"method": __doc__.strip().splitlines()[2:5], "kernels": {}}
    trace = trace_by_grid(src)
    for k in sorted(set(fetch) | set(write)):
        grids = sorted(set(fetch.get(k, {})) | set(write.get(k, {})))
        by_grid = {}
        for g in grids:
            f, w = fetch.get(k, {}).get(g, []), write.get(k, {}).get(g, [])
            fk, wk = mean(f), mean(w)
            e = {"workgroups": g // WG_SIZE.get(k, 256), "dispatches": max(len(f), len(w)), "fetch_kib_per_launch": fk,
                 "write_kib_per_launch": wk, "hbm_bytes_per_launch": (2 * fk + wk) * 1024.0}
            if g in trace.get(k, {}):
                e["rocprof_trace_dispatches"], ns = trace[k][g]
                e["rocprof_trace_avg_us"] = ns / 1000.0
            by_grid[str(g)] = e
        top = by_grid[str(grids[-1])]
        out["kernels"][k] = dict(top, grid_threads=grids[-1], by_grid=by_grid)
    out["source_run"] = os.path.basename(os.path.normpath(src))
    for path in (dst + "_pmc_traffic.json", os.path.join(os.path.dirname(dst) or ".", "pmc_traffic.json")):
        with open(path, "w") as fh:
            json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
