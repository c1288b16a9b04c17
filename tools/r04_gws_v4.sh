#!/bin/bash
# round 4: gate_ws v4 (deeper A-fragment prefetch, steady step as one basic block, static priority) against the
# previous build (ab/libsvc_hip_base.so): parity, step timeline, alone timings, end-to-end alternating A/B
set -o pipefail
O=gpurun_out/${TAG:-r04k}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 240 --timeout-method thread -k "gate_ws_bit_identical" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && { tail -60 $O/tests.log; exit $rc; }
timeout -k 10 300 python3 tools/r04_gws_dump.py > $O/dump.txt 2>&1 || exit $?
cat $O/dump.txt
timeout -k 10 200 python3 tools/r04_gws_stamps.py > $O/stamps.txt 2>&1 || exit $?
cat $O/stamps.txt
SH="29984,768,384,3,1;14992,768,384,3,1"
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/ab/libsvc_hip_base.so; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    SVC_HIP_LIB=$L GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="$SH" timeout -k 10 120 python3 tools/gemm_bench.py 24 40 > $O/g.txt 2>&1 || exit $?
    grep -v amdgpu $O/g.txt | sed "s/^/$lib: /"
  done
done
for dbg in 2 4; do
  SVC_GWS_DBG=$dbg GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="$SH" timeout -k 10 120 python3 tools/gemm_bench.py 40 > $O/d$dbg.txt 2>&1 || exit $?
  grep -v amdgpu $O/d$dbg.txt | sed "s/^/dbg $dbg: /"
done
for r in 1 2 3; do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/ab/libsvc_hip_base.so; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    SVC_HIP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b_$lib.json 2> $O/b_$lib.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b_$lib.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$lib', d['value'], d['ms_per_step'], {kk: round(vv['ms_per_step'],2) for kk,vv in k.items() if 'dilated' in kk or 'outproj' in kk})"
  done
done
