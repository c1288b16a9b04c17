#!/bin/bash
# round 4: amp_conv epilogue over whole rows (C tile staged through LDS) vs the register epilogue (SVC_AMP_DBG=8):
# parity, alone timings, end to end alternating
set -o pipefail
O=gpurun_out/${TAG:-r04v}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_stages.py tests/test_gpu_ragged.py -m gpu -x -q --timeout 300 --timeout-method thread -k "activation or amp_conv or bigvgan or vocoder or ragged" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log
[ $rc -ne 0 ] && { tail -60 $O/tests.log; exit $rc; }
for dbg in 0 8 0 8; do
  SVC_AMP_DBG=$dbg timeout -k 10 180 python3 tools/amp_bench.py > $O/m.txt 2>&1 || { cat $O/m.txt; exit 1; }
  grep -v amdgpu $O/m.txt | grep -E "d=1|d=5" | sed "s/^/dbg$dbg amp: /"
done
for r in 1 2 3; do
  for dbg in 8 0; do
    SVC_AMP_DBG=$dbg timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); k=d['kernels']; print('dbg$dbg', d['value'], d['ms_per_step'], 'bigvgan', round(sum(v['ms_per_step'] for kk, v in k.items() if 'bigvgan' in kk), 2), 'amp', round(sum(v['ms_per_step'] for kk, v in k.items() if kk.startswith('amp_conv')), 2), 'act', round(sum(v['ms_per_step'] for kk, v in k.items() if kk.startswith('activation1d')), 2))"
  done
done
