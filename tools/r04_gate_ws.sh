#!/bin/bash
# round 4: gate_ws parity (bit identity with conv_gemm4) and microbenchmarks, then the default bench as a baseline
set -o pipefail
O=gpurun_out/${TAG:-r04b}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gate_ws_bit_identical or gate_gemm_ragged" > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -ne 0 ] && { tail -60 $O/tests.log; exit $rc; }
for d in 1 8; do
  SVC_BENCH_DIL=$d GEMM_BENCH_CUSTOM="29984,768,384,3,1;14992,768,384,3,1" timeout -k 10 120 python3 tools/gemm_bench.py 24 40 > $O/gemm_d$d.txt 2>&1 || exit $?
  sed "s/^/dil $d: /" $O/gemm_d$d.txt
  SVC_BENCH_DIL=$d GEMM_BENCH_WARM=1 GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="29984,768,384,3,1;14992,768,384,3,1" timeout -k 10 120 python3 tools/gemm_bench.py 24 40 > $O/gemm_warm_d$d.txt 2>&1 || exit $?
  sed "s/^/warm dil $d: /" $O/gemm_warm_d$d.txt
done
for v in 0 1; do
  SVC_GATE_WS=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/bench_gws$v.json 2> $O/bench_gws$v.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench_gws$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('gate_ws=$v', d['value'], d['ms_per_step'], {kk: round(vv['ms_per_step'],2) for kk,vv in k.items() if 'dilated' in kk or 'outproj' in kk})"
done
