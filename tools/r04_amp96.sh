#!/bin/bash
# round 4: amp_conv on the packed activation for every C; the C = 96 stage fused (SVC_AMP_MAXC=96) vs activation1d +
# conv_gemm3 (48, default): parity, alone timings, end to end alternating
set -o pipefail
O=gpurun_out/${TAG:-r04w}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_stages.py tests/test_gpu_ragged.py -m gpu -x -q --timeout 300 --timeout-method thread -k "activation or amp_conv or bigvgan or vocoder or ragged" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log
[ $rc -ne 0 ] && { tail -60 $O/tests.log; exit $rc; }
SVC_AMP_MAXC=96 timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_ragged.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bigvgan or vocoder or ragged" > $O/tests96.log 2>&1; rc=$?; tail -2 $O/tests96.log
[ $rc -ne 0 ] && { tail -60 $O/tests96.log; exit $rc; }
AMP_BENCH_C96=1 timeout -k 10 240 python3 tools/amp_bench.py > $O/m.txt 2>&1 || { cat $O/m.txt; exit 1; }
grep -v amdgpu $O/m.txt
for r in 1 2 3; do
  for mc in 48 96; do
    SVC_AMP_MAXC=$mc timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); k=d['kernels']; print('maxc$mc', d['value'], d['ms_per_step'], 'bigvgan', round(sum(v['ms_per_step'] for kk, v in k.items() if 'bigvgan' in kk), 2), 'amp', round(sum(v['ms_per_step'] for kk, v in k.items() if kk.startswith('amp_conv')), 2), 'act', round(sum(v['ms_per_step'] for kk, v in k.items() if kk.startswith('activation1d')), 2))"
  done
done
