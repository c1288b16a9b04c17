"""Summarise tools/pmc_kernels.sh: per kernel (and grid size) the mean of each counter per dispatch, MFMA utilisation
and HBM bytes. MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs): the share of SIMD
cycles with the matrix core busy (MI355X_MICROARCH.md: the MFMA counter counts cycles, GRBM_GUI_ACTIVE is summed over the
8 XCDs). HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (the gfx950 FETCH_SIZE 1/2 correction). LDS bank conflicts as a
share of LDS-active cycles; VALU instructions per MFMA (MFMAs estimated as busy cycles / 16). Usage: python tools/pmc_kernels.py gpurun_out/<tag> [json_out]"""
import collections
import csv
import glob
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from tools.pmc_summary import short  # noqa: E402


def main():
    root = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(root + "/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0) // max(1, int(r.get("Workgroup_Size", r.get("Workgroup_Size_X", 1)) or 1))
            key = (short(r["Kernel_Name"]), grid)
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    rows = []
    for (k, g), cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        d = {"workgroups": g, "dispatches": n}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
            d["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
            d["gpu_cycles"] = m["GRBM_GUI_ACTIVE"] / 8
        d["kernel"] = k
        if m.get("SQ_VALU_MFMA_BUSY_CYCLES") and "SQ_INSTS_VALU" in m:
            # MFMA instructions ~ busy cycles / 16 (v_mfma_f32_16x16x32_f16 / _bf16 keep the matrix pipe 16 cycles);
            # SQ_INSTS_VALU counts them too
            n_mfma = m["SQ_VALU_MFMA_BUSY_CYCLES"] / 16.0
            d["mfma_insts_est"] = n_mfma
            d["valu_per_mfma"] = (m["SQ_INSTS_VALU"] - n_mfma) / n_mfma
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict_share"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            d["hbm_bytes"] = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
        d["counters"] = m
        out[f"{k}@{g}"] = d
        rows.append((d.get("gpu_cycles", 0) * n, k, g, d))
    for _, k, g, d in sorted(rows, key=lambda r: -r[0]):
        print(f"{k:34s} wg={g:6d} n={d['dispatches']:5d} mfma_busy={d.get('mfma_busy', float('nan')):.3f} "
              f"cycles={d.get('gpu_cycles', 0):9.0f} valu/mfma={d.get('valu_per_mfma', float('nan')):5.2f} "
              f"lds_conflict={d.get('lds_conflict_share', float('nan')):.3f} "
              f"hbm_MB={d.get('hbm_bytes', 0) / 1e6:8.1f}")
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
