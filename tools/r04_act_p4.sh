#!/bin/bash
# round 4: activation1d on f16 input in 4-row blocks (82 VGPRs, 6 waves per SIMD; SVC_ACT_P4=1) vs 8-row blocks (96)
set -o pipefail
O=gpurun_out/${TAG:-r04af}; mkdir -p $O; export TMPDIR=/tmp
SVC_ACT_P4=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 200 --timeout-method thread -k "activation" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log
[ $rc -ne 0 ] && { tail -40 $O/tests.log; exit $rc; }
for r in 1 2; do
  for p4 in 0 1; do
    SVC_ACT_P4=$p4 timeout -k 10 180 python3 tools/act_bench.py > $O/a.txt 2>&1 || { cat $O/a.txt; exit 1; }
    grep -v amdgpu $O/a.txt | grep f16 | sed "s/^/p4=$p4 act: /"
  done
done
for r in 1 2; do
  for p4 in 0 1; do
    SVC_ACT_P4=$p4 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); k=d['kernels']; print('p4=$p4', d['value'], d['ms_per_step'], 'act', round(sum(v['ms_per_step'] for kk, v in k.items() if kk.startswith('activation1d')), 2))"
  done
done
