#!/bin/bash
# round 4: res_proj ring depth (SVC_RP_DEPTH 3 / 4 / 5) with one sampler stream: parity, alone, end-to-end A/B
set -o pipefail
O=gpurun_out/${TAG:-r04o}; mkdir -p $O; export TMPDIR=/tmp
for d in 4 5; do
  SVC_RP_DEPTH=$d timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 240 --timeout-method thread -k "res_proj" > $O/tests$d.log 2>&1; rc=$?; tail -2 $O/tests$d.log
  [ $rc -ne 0 ] && { tail -60 $O/tests$d.log; exit $rc; }
done
for r in 1 2; do
  for d in 3 4 5; do
    SVC_RP_DEPTH=$d GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="29984,384,384,1,6" timeout -k 10 120 python3 tools/gemm_bench.py 30 > $O/g.txt 2>&1 || exit $?
    grep -v amdgpu $O/g.txt | sed "s/^/depth $d: /"
  done
done
for r in 1 2 3; do
  for d in 3 4 5; do
    SVC_RP_DEPTH=$d timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b.json 2> $O/b.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); k=d['kernels']; print('depth $d', d['value'], d['ms_per_step'], {kk: round(vv['ms_per_step'],2) for kk,vv in k.items() if 'outproj' in kk})"
  done
done
