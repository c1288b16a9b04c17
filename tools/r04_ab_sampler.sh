#!/bin/bash
# round 4: sampler configuration A/B (alternating), pYIN + PLMS-100 headline GPU tests
set -o pipefail
O=gpurun_out/${TAG:-r04j}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -k gate_ws_bit_identical tests/test_f0.py tests/test_gpu_headline.py -m gpu -x -q --timeout 240 --timeout-method thread -k "pyin or plms100_headline or gate_ws_bit_identical" > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log
[ $rc -ne 0 ] && { tail -60 $O/tests.log; exit $rc; }
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b_$name.json 2> $O/b_$name.err || return $?
  python3 -c "import json; d=json.loads(open('$O/b_$name.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$name', d['value'], d['ms_per_step'], {kk: round(vv['ms_per_step'],2) for kk,vv in k.items() if 'dilated' in kk or 'outproj' in kk})"
}
for i in 1 2 3; do
  run A$i SVC_NOOP=1 || exit $?
  run B$i SVC_SAMPLER_STREAMS=1 SVC_GATE_WS=1 SVC_RES_PROJ=128 || exit $?
  run C$i SVC_GATE_WS=1 || exit $?
  run D$i SVC_SAMPLER_STREAMS=1 SVC_GATE_WS=1 SVC_RES_PROJ=112 || exit $?
done
timeout -k 10 200 python3 tools/r04_gws_stamps.py > $O/stamps.txt 2>&1; cat $O/stamps.txt
