#!/bin/bash
# round 4: gate_ws diagnostics (SVC_GWS_DBG modes, timing only) and one SQ counter pass per kernel
set -o pipefail
O=gpurun_out/${TAG:-r04c}; mkdir -p $O; export TMPDIR=/tmp
export GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="29984,768,384,3,1"; SH="29984,768,384,3,1;14992,768,384,3,1"
for dbg in 0 1 2 4 8 16 32 6 14; do
  SVC_GWS_DBG=$dbg GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="$SH" timeout -k 10 120 python3 tools/gemm_bench.py 40 > $O/d$dbg.txt 2>&1 || exit $?
  grep -v amdgpu $O/d$dbg.txt | sed "s/^/dbg $dbg: /"
done
GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="$SH" timeout -k 10 120 python3 tools/gemm_bench.py 24 40 | grep -v amdgpu
for v in 24 40; do
  timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -f csv -d $O/pmc$v -o run -- python3 tools/gemm_bench.py $v > $O/pmc$v.log 2>&1 || { tail -5 $O/pmc$v.log; exit 1; }
done
find $O -name "*counter_collection.csv" | head
