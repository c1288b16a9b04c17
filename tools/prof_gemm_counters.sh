#!/bin/bash
# SQ/LDS/L2 counters of one conv_gemm3 launch shape (run from the repo root via gpurun). rocprofv3 records
# template kernels with bool parameters under their mangled names, so KRE matches the mangled symbol.
#   SHAPE: tools/gemm_bench.py shape-name filter; VAR: SVC_GEMM_VARIANT; KRE: kernel regex
set -uo pipefail
R=$(pwd); O=$R/gpurun_out/gemmprof; mkdir -p $O; export TMPDIR=/tmp
SHAPE=${SHAPE:-dilated(gate)}; VAR=${VAR:-15}; KRE=${KRE:-conv_gemm3_kernelILi128ELi384ELb1ELb1E}
export GEMM_BENCH_SHAPES="$SHAPE" GEMM_BENCH_TORCH=0
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "$KRE" -f csv -d $O/p$i -o run -- \
    python3 $R/tools/gemm_bench.py $VAR > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:28s} n={len(v):3d} mean={sum(v) / len(v):.4g}")
PY
