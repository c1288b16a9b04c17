#!/bin/bash
# round 4: gate_ws v3 parity, step timeline and timing
set -o pipefail
O=gpurun_out/${TAG:-r04i}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gate_ws_bit_identical or whisper_encoder_tiny or whisper_stream" > $O/tests.log 2>&1 && timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py -m gpu -x -q --timeout 300 --timeout-method thread -k "whisper_medium_vs_oracle" >> $O/tests.log 2>&1
rc=$?; [ $rc -eq 0 ] && { timeout -k 10 400 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_ops.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bigvgan or amp_conv" >> $O/tests.log 2>&1; rc=$?; }
tail -3 $O/tests.log; [ $rc -ne 0 ] && { tail -60 $O/tests.log; exit $rc; }
timeout -k 10 300 python3 tools/r04_gws_dump.py > $O/dump.txt 2>&1 || exit $?
cat $O/dump.txt
timeout -k 10 200 python3 tools/r04_gws_stamps.py > $O/st0.txt 2>&1 || exit $?
cat $O/st0.txt
SH="29984,768,384,3,1;14992,768,384,3,1"
for dbg in 0 2; do
  SVC_GWS_DBG=$dbg GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="$SH" timeout -k 10 120 python3 tools/gemm_bench.py 24 40 > $O/d$dbg.txt 2>&1 || exit $?
  grep -v amdgpu $O/d$dbg.txt | sed "s/^/dbg $dbg: /"
done
for v in 0 1; do
  SVC_GATE_WS=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/bench_gws$v.json 2> $O/bench_gws$v.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench_gws$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('gate_ws=$v', d['value'], d['ms_per_step'], {kk: round(vv['ms_per_step'],2) for kk,vv in k.items() if 'dilated' in kk or 'outproj' in kk})"
  SVC_SAMPLER_STREAMS=1 SVC_GATE_WS=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/bench1s_gws$v.json 2> $O/bench1s_gws$v.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench1s_gws$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('1 stream gate_ws=$v', d['value'], d['ms_per_step'], {kk: round(vv['ms_per_step'],2) for kk,vv in k.items() if 'dilated' in kk or 'outproj' in kk})"
done
for lanes in 128 160; do
  SVC_SAMPLER_STREAMS=1 SVC_GATE_WS=1 SVC_RES_PROJ=$lanes timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/bench1s_rp$lanes.json 2> $O/bench1s_rp$lanes.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench1s_rp$lanes.json').read().strip().splitlines()[-1]); k=d['kernels']; print('1 stream gate_ws res_proj lanes $lanes', d['value'], d['ms_per_step'], {kk: round(vv['ms_per_step'],2) for kk,vv in k.items() if 'dilated' in kk or 'outproj' in kk})"
done
timeout -k 10 300 python -u -m pytest tests/test_f0.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pyin.log 2>&1; echo "pyin rc=$?"; tail -30 $O/pyin.log
