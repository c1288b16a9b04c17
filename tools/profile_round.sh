#!/bin/bash
# profile of record: bench line (with the CPU baseline) + rocprofv3 trace + FETCH / WRITE passes on the
# headline kernel (tools/gpu_profile.sh), per-kernel PMC passes (tools/pmc_kernels.sh), and one issue-accounting pass
# on gate_ws (counters checked against rocprofv3 -L first)
set -o pipefail
TAG=${TAG:-prof}
mkdir -p gpurun_out/$TAG
timeout -k 10 60 rocprofv3 -L > gpurun_out/$TAG/counters.txt 2>&1 || true
bash tools/gpu_profile.sh $TAG > gpurun_out/${TAG}_profile.log 2>&1 || { tail -20 gpurun_out/${TAG}_profile.log; exit 1; }
tail -5 gpurun_out/${TAG}_profile.log
TAG=${TAG}_pmc bash tools/pmc_kernels.sh > gpurun_out/${TAG}_pmc.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc.log; exit 1; }
head -40 gpurun_out/${TAG}_pmc.log
SET="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU GRBM_GUI_ACTIVE"
ok=1
for c in $SET; do grep -q "\b$c\b" gpurun_out/$TAG/counters.txt || { echo "counter $c not listed"; ok=0; }; done
if [ $ok = 1 ]; then
  O=gpurun_out/${TAG}_issue; mkdir -p $O
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "gate_ws_kernel" -f csv -d $O/p5 -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/p5.log 2>&1 && echo "issue pass done"
  python3 tools/pmc_kernels.py $O $O/summary.json > $O/summary.txt; cat $O/summary.txt
fi
