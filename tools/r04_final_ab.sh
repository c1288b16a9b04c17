#!/bin/bash
# round 4: K split 22 / 23 / 24 end to end, parity at the default (22), PLMS-100 headline rel-L2 (printed), pYIN timing
set -o pipefail
O=gpurun_out/${TAG:-r04p}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_headline.py -m gpu -x -q -s --timeout 300 --timeout-method thread -k "gate_ws_bit_identical or plms100_headline" > $O/tests.log 2>&1; rc=$?; grep -E "PLMS|passed|failed" $O/tests.log | tail -5
[ $rc -ne 0 ] && { tail -60 $O/tests.log; exit $rc; }
for ka in 20 23 24; do
  SVC_GWS_KA=$ka timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 240 --timeout-method thread -k "gate_ws_bit_identical" > $O/t$ka.log 2>&1; rc=$?; tail -1 $O/t$ka.log
  [ $rc -ne 0 ] && { tail -40 $O/t$ka.log; exit $rc; }
done
timeout -k 10 300 python3 tools/pyin_bench.py > $O/pyin.txt 2>&1 || exit $?
grep -v amdgpu $O/pyin.txt
for r in 1 2; do
  for cfg in "SVC_NOOP=1" "SVC_GWS_KA=20" "SVC_GWS_KA=23" "SVC_GWS_KA=24"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b.json 2> $O/b.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'])"
  done
done
