#!/bin/bash
# round 4: BigVGAN activation on packed channel pairs (activation1d: buffer offsets, clamp-free interior runs;
# amp_conv: the same arithmetic, whole runs) against the previous build (ab/libsvc_hip_base.so): parity, alone
# timings (tools/act_bench.py, tools/amp_bench.py), end to end alternating
set -o pipefail
O=gpurun_out/${TAG:-r04t}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_stages.py tests/test_gpu_ragged.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "activation or amp_conv or bigvgan or vocoder or ragged or mel_l1" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log
[ $rc -ne 0 ] && { tail -60 $O/tests.log; exit $rc; }
grep -E "mel-L1|mel_l1" $O/tests.log | tail -4
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/ab/libsvc_hip_base.so; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    SVC_HIP_LIB=$L timeout -k 10 180 python3 tools/act_bench.py > $O/a.txt 2>&1 || { cat $O/a.txt; exit 1; }
    grep -v amdgpu $O/a.txt | sed "s/^/$lib act: /"
    SVC_HIP_LIB=$L timeout -k 10 180 python3 tools/amp_bench.py > $O/m.txt 2>&1 || { cat $O/m.txt; exit 1; }
    grep -v amdgpu $O/m.txt | sed "s/^/$lib amp: /"
  done
done
for r in 1 2 3; do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/ab/libsvc_hip_base.so; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    SVC_HIP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$lib', d['value'], d['ms_per_step'], 'bigvgan', round(sum(v['ms_per_step'] for kk, v in k.items() if 'bigvgan' in kk), 2), 'amp', round(sum(v['ms_per_step'] for kk, v in k.items() if kk.startswith('amp_conv')), 2), 'act', round(sum(v['ms_per_step'] for kk, v in k.items() if kk.startswith('activation1d')), 2))"
  done
done
