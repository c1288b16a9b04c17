#!/bin/bash
# round 4: gate_ws with the K-loop pinned per K-step (reads 4 ahead, epilogue spread over the segments) against the
# previous build (ab/libsvc_hip_base.so): bit identity, timeline, alone timings, end-to-end alternating A/B, the
# event-marker cost and the host enqueue time
set -o pipefail
O=gpurun_out/${TAG:-r04m}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 240 --timeout-method thread -k "gate_ws_bit_identical or gate_ws32_close" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && { tail -60 $O/tests.log; exit $rc; }
timeout -k 10 300 python3 tools/r04_gws_dump.py 40 > $O/dump.txt 2>&1 || exit $?
cat $O/dump.txt
timeout -k 10 200 python3 tools/r04_gws_stamps.py > $O/stamps.txt 2>&1 || exit $?
cat $O/stamps.txt
SH="29984,768,384,3,1;14992,768,384,3,1"
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/ab/libsvc_hip_base.so; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    SVC_HIP_LIB=$L GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="$SH" timeout -k 10 120 python3 tools/gemm_bench.py 40 41 > $O/g.txt 2>&1 || exit $?
    grep -v amdgpu $O/g.txt | sed "s/^/$lib: /"
  done
done
for r in 1 2 3; do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/ab/libsvc_hip_base.so; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    SVC_HIP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b_$lib.json 2> $O/b_$lib.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b_$lib.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$lib', d['value'], d['ms_per_step'], {kk: round(vv['ms_per_step'],2) for kk,vv in k.items() if 'dilated' in kk or 'outproj' in kk})"
  done
done
for r in 1 2; do
  for ev in 1 0; do
    BENCH_TIMED_EVENTS=$ev timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/e_$ev.json 2> $O/e_$ev.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/e_$ev.json').read().strip().splitlines()[-1]); r=d['roofline']; print('timed events=$ev', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'])"
  done
done
timeout -k 10 300 python3 tools/host_enqueue.py > $O/enqueue.txt 2>&1 || exit $?
grep -v amdgpu $O/enqueue.txt
