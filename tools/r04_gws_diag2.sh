#!/bin/bash
# round 4: gate_ws latency diagnostics + the headline-shape PLMS-100 parity test
set -o pipefail
O=gpurun_out/${TAG:-r04d}; mkdir -p $O; export TMPDIR=/tmp
SH="29984,768,384,3,1;14992,768,384,3,1"
for dbg in 0 64 128 256 192 448 450; do
  SVC_GWS_DBG=$dbg GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="$SH" timeout -k 10 120 python3 tools/gemm_bench.py 40 > $O/d$dbg.txt 2>&1 || exit $?
  grep -v amdgpu $O/d$dbg.txt | sed "s/^/dbg $dbg: /"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py -m gpu -x -q -s --timeout 500 --timeout-method thread -k "headline_shape" > $O/tests.log 2>&1
rc=$?; grep -E "PLMS-100|passed|failed|Error" $O/tests.log | tail -8; exit $rc
