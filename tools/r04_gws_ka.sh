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
# res_proj ring depth (SVC_RP_DEPTH) and write-through row-stream stores (SVC_STORE_WT)
for d in 4 5; do
  SVC_RP_DEPTH=$d timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 240 --timeout-method thread -k "res_proj" > $O/rtests$d.log 2>&1; rc=$?; tail -1 $O/rtests$d.log
  [ $rc -ne 0 ] && { tail -40 $O/rtests$d.log; exit $rc; }
done
SVC_STORE_WT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 240 --timeout-method thread -k "res_proj or gate_ws_bit" > $O/wtests.log 2>&1; rc=$?; tail -1 $O/wtests.log
[ $rc -ne 0 ] && { tail -40 $O/wtests.log; exit $rc; }
for d in 3 4 5; do
  SVC_RP_DEPTH=$d GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="29984,384,384,1,6" timeout -k 10 120 python3 tools/gemm_bench.py 30 > $O/g.txt 2>&1 || exit $?
  grep -v amdgpu $O/g.txt | sed "s/^/rp depth $d: /"
done
for r in 1 2; do
  for cfg in "SVC_NOOP=1" "SVC_STORE_WT=1" "SVC_RP_DEPTH=4" "SVC_RP_DEPTH=5"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b.json 2> $O/b.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$cfg', d['value'], d['ms_per_step'], {kk: round(vv['ms_per_step'],2) for kk,vv in k.items() if 'outproj' in kk or 'dilated' in kk})"
  done
done
