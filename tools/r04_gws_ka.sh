#!/bin/bash
# round 4: gate_ws K split between the wave pair (SVC_GWS_KA 18 / 20 / 22) and gate_ws32 with the pinned K-loop:
# parity, alone timings, step timeline, end-to-end alternating A/B (timed region without events)
set -o pipefail
O=gpurun_out/${TAG:-r04n}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 240 --timeout-method thread -k "gate_ws_bit_identical or gate_ws32_close" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && { tail -60 $O/tests.log; exit $rc; }
for v in 40 41; do timeout -k 10 300 python3 tools/r04_gws_dump.py $v > $O/dump$v.txt 2>&1 || exit $?; cat $O/dump$v.txt; done
SH="29984,768,384,3,1;14992,768,384,3,1"
for r in 1 2; do
  for ka in 18 20 22; do
    SVC_GWS_KA=$ka GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="$SH" timeout -k 10 120 python3 tools/gemm_bench.py 40 > $O/g.txt 2>&1 || exit $?
    grep -v amdgpu $O/g.txt | sed "s/^/KA $ka: /"
  done
  GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="$SH" timeout -k 10 120 python3 tools/gemm_bench.py 41 > $O/g.txt 2>&1 || exit $?
  grep -v amdgpu $O/g.txt | sed "s/^/ws32: /"
done
timeout -k 10 200 python3 tools/r04_gws_stamps.py > $O/stamps.txt 2>&1 || exit $?
cat $O/stamps.txt
for r in 1 2; do
  for cfg in "SVC_GWS_KA=18" "SVC_GWS_KA=20" "SVC_GWS_KA=22" "SVC_GATE_WS=2"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b.json 2> $O/b.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'])"
  done
done
