#!/bin/bash
# round 4: amp_conv activation runs of RUN = 1 / 2 mod 8 rows (conflict-free LDS stores) against the previous build
# (ab/libsvc_hip_base.so): parity, LDS conflicts (PMC), alone timings, end to end
set -o pipefail
O=gpurun_out/${TAG:-r04q}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_stages.py -m gpu -x -q --timeout 300 --timeout-method thread -k "amp_conv or bigvgan" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log
[ $rc -ne 0 ] && { tail -60 $O/tests.log; exit $rc; }
for lib in base new; do
  if [ $lib = base ]; then L=$PWD/ab/libsvc_hip_base.so; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
  SVC_HIP_LIB=$L timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex amp_conv -f csv -d $O/pmc_$lib -o run -- python3 tools/amp_bench.py > $O/pmc_$lib.log 2>&1 || exit $?
  python3 - $O/pmc_$lib $lib <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = "amp_conv<24>" if "<24" in r["Kernel_Name"] else "amp_conv<48>"
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(acc.items()):
    print(sys.argv[2], k, "LDS conflict share", round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 3))
PY
done
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/ab/libsvc_hip_base.so; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    SVC_HIP_LIB=$L timeout -k 10 180 python3 tools/amp_bench.py > $O/m.txt 2>&1 || exit $?
    grep -v amdgpu $O/m.txt | sed "s/^/$lib amp: /"
  done
done
for r in 1 2 3; do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/ab/libsvc_hip_base.so; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    SVC_HIP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b.json 2> $O/b.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$lib', d['value'], d['ms_per_step'], 'bigvgan', round(sum(v['ms_per_step'] for kk, v in k.items() if 'bigvgan' in kk), 2), 'amp', round(sum(v['ms_per_step'] for kk, v in k.items() if kk.startswith('amp_conv')), 2))"
  done
done
