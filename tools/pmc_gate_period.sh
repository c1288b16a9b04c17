# gate_ws period-3 step: the same counters per dispatch at M = 29 984 (one step in three runs
# ~350 ticks long) and M = 14 992 (two in three), each pass its own rocprofv3 run (run from the repo root via gpurun).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06c}/gate_period; mkdir -p $O
i=0
for set in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCC_TAG_STALL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_REQ_sum TCC_READ_sum TA_BUFFER_READ_WAVEFRONTS_sum TA_BUFFER_WRITE_WAVEFRONTS_sum SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for M in 29984 14992; do
    GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM=$M,768,384,3,1 timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "gate_ws_kernel" -f csv -d $O/M$M/p$i -o run -- python3 tools/gemm_bench.py 40 > $O/p${i}_$M.log 2>&1 || { echo "pass $i M$M failed"; tail -5 $O/p${i}_$M.log; exit 1; }
  done
  echo "pass $i done"
done
python3 - $O <<'PY'
import csv, glob, sys, collections
root = sys.argv[1]
res = {}
for M in (29984, 14992):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{root}/M{M}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    res[M] = {k: sum(v) / len(v) for k, v in acc.items()}
print(f"{'counter (mean per dispatch)':44s} {'M=29984':>14s} {'M=14992':>14s} {'per-row ratio 14992/29984':>26s}")
for k in sorted(res[29984]):
    a, b = res[29984][k], res[14992].get(k, float('nan'))
    r = (b / 14992) / (a / 29984) if a else float('nan')
    print(f"{k:44s} {a:14.4g} {b:14.4g} {r:26.3f}")
PY
