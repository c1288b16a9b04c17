#!/bin/bash
# One gpurun call: GPU parity tests, GEMM variant table, short bench. Each GPU step has its own limit;
# the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_gpu_ops.py tests/test_gpu_stages.py tests/test_gpu_long.py"}
timeout -k 10 700 python -m pytest $TESTS -m gpu -q --timeout 500 > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$ACT" ]; then
  timeout -k 10 300 python3 tools/act_bench.py > gpurun_out/act_bench.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/act_bench.log
fi
timeout -k 10 300 python3 tools/gemm_bench.py ${VARIANTS:--1 10 11 12 13 14 15 20 24} > gpurun_out/gemm_bench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/gemm_bench.log
if [ -n "$BENCH" ]; then
  # BENCH_ENVS: space-separated "VAR=val,VAR=val" settings, one quick bench each ("-" = defaults)
  i=0
  for cfg in ${BENCH_ENVS:--}; do
    i=$((i+1))
    envs=""; [ "$cfg" != "-" ] && envs=$(echo "$cfg" | tr ',' ' ')
    echo "bench[$i] $cfg"
    env $envs timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_quick_$i.log 2>&1 || exit $?
    tail -1 gpurun_out/bench_quick_$i.log | cut -c1-300
  done
fi
