#!/bin/bash
# round 4: activation1d next-block prefetch (SVC_ACT_PF) A/B; amp_conv phase split (SVC_AMP_DBG: 1 no activation,
# 2 no conv MFMAs, 4 no epilogue)
set -o pipefail
O=gpurun_out/${TAG:-r04u}; mkdir -p $O; export TMPDIR=/tmp
SVC_ACT_PF=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -k "activation" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log
[ $rc -ne 0 ] && { tail -40 $O/tests.log; exit $rc; }
for r in 1 2; do
  for pf in 0 1; do
    SVC_ACT_PF=$pf timeout -k 10 180 python3 tools/act_bench.py > $O/a.txt 2>&1 || { cat $O/a.txt; exit 1; }
    grep -v amdgpu $O/a.txt | sed "s/^/pf$pf act: /"
  done
done
for dbg in 0 1 2 4 6 3; do
  SVC_AMP_DBG=$dbg timeout -k 10 180 python3 tools/amp_bench.py > $O/m.txt 2>&1 || { cat $O/m.txt; exit 1; }
  grep -v amdgpu $O/m.txt | grep -E "d=1|d=5" | sed "s/^/dbg$dbg amp: /"
done
