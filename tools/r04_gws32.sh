#!/bin/bash
# round 4: gate_ws32 (32x32x16 MFMA form, tune.gate_ws = 2) against gate_ws (v4): closeness, timeline, timings, A/B
set -o pipefail
O=gpurun_out/${TAG:-r04l}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gate_ws32_close or gate_ws_bit_identical" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && { tail -60 $O/tests.log; exit $rc; }
timeout -k 10 300 python3 tools/r04_gws_dump.py 41 > $O/dump.txt 2>&1 || exit $?
cat $O/dump.txt
GWS_V=41 timeout -k 10 200 python3 tools/r04_gws_stamps.py > $O/stamps.txt 2>&1 || exit $?
cat $O/stamps.txt
SH="29984,768,384,3,1;14992,768,384,3,1"
for r in 1 2; do
  GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="$SH" timeout -k 10 120 python3 tools/gemm_bench.py 40 41 > $O/g.txt 2>&1 || exit $?
  grep -v amdgpu $O/g.txt
done
for dbg in 2 4; do
  SVC_GWS_DBG=$dbg GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="$SH" timeout -k 10 120 python3 tools/gemm_bench.py 41 > $O/d$dbg.txt 2>&1 || exit $?
  grep -v amdgpu $O/d$dbg.txt | sed "s/^/dbg $dbg: /"
done
for r in 1 2 3; do
  for v in 1 2; do
    SVC_GATE_WS=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b_$v.json 2> $O/b_$v.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('gate_ws=$v', d['value'], d['ms_per_step'], {kk: round(vv['ms_per_step'],2) for kk,vv in k.items() if 'dilated' in kk or 'outproj' in kk})"
  done
done
# HIP-event vs rocprof per-launch time of the same gate_ws launches: batched events (one pair around
# 10 launches) and per-launch event pairs (as bench.py's live profile), each also under rocprofv3 --kernel-trace
for mode in batched perlaunch; do
  PL=""; [ $mode = perlaunch ] && PL=1
  SVC_BENCH_PERLAUNCH=$PL GEMM_BENCH_WARM=1 GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="29984,768,384,3,1" timeout -k 10 120 python3 tools/gemm_bench.py 40 > $O/rec_$mode.txt 2>&1 || exit $?
  grep -v amdgpu $O/rec_$mode.txt | sed "s/^/events $mode: /"
  SVC_BENCH_PERLAUNCH=$PL GEMM_BENCH_WARM=1 GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="29984,768,384,3,1" timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/rp_$mode -o run -- python3 tools/gemm_bench.py 40 > $O/rec_rp_$mode.txt 2>&1 || exit $?
  grep -v amdgpu $O/rec_rp_$mode.txt | grep custom | sed "s/^/events under rocprof $mode: /"
  python3 - $O/rp_$mode <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f)) if "gate_ws_kernel" in r["Kernel_Name"]]
print(f"rocprof trace: {len(d)} gate_ws dispatches, last 10 avg {sum(d[-10:]) / 10 / 1000:.2f} us, all avg {sum(d) / len(d) / 1000:.2f} us")
PY
done
