#!/bin/bash
# One gpurun call: optional GPU tests ($TESTS), then one quick bench per "VAR=val,VAR=val" setting in $BENCH_ENVS
# ("-" = defaults). Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
fi
i=0
for cfg in ${BENCH_ENVS:--}; do
  i=$((i+1))
  envs=""; [ "$cfg" != "-" ] && envs=$(echo "$cfg" | tr ',' ' ')
  env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps ${STEPS:-3} --warmup 1 > gpurun_out/ab_$i.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/ab_$i.log "$cfg"
done
