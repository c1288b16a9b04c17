#!/bin/bash
# round 4: gate_ws static priority placement (SVC_GWS_PRIO 0: second waves, 1: first waves, 2: none): alone, end to end
set -o pipefail
O=gpurun_out/${TAG:-r04s}; mkdir -p $O; export TMPDIR=/tmp
SVC_GWS_PRIO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 240 --timeout-method thread -k "gate_ws_bit_identical" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log
[ $rc -ne 0 ] && { tail -40 $O/tests.log; exit $rc; }
SH="29984,768,384,3,1"
for r in 1 2; do
  for p in 0 1 2; do
    SVC_GWS_PRIO=$p GEMM_BENCH_WARM=1 GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="$SH" timeout -k 10 120 python3 tools/gemm_bench.py 40 > $O/g.txt 2>&1 || exit $?
    grep -v amdgpu $O/g.txt | sed "s/^/prio $p: /"
  done
done
for r in 1 2 3; do
  for p in 0 1 2; do
    SVC_GWS_PRIO=$p timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b.json 2> $O/b.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('prio $p', d['value'], d['ms_per_step'], r['avg_launch_us'])"
  done
done
