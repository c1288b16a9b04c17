#!/bin/bash
# round 4: conv_gemm3 register-epilogue mask (tune.gemm3_direct) with one sampler stream: 3 (default: F16 + RES32
# outside the sampler), 11 (+ inside the sampler), 15 (+ the split form), 1 (RES32 off: the LDS-staged residual
# epilogue): end to end alternating
set -o pipefail
O=gpurun_out/${TAG:-r04y}; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
  for m in 3 11 15 1; do
    SVC_GEMM3_DIRECT=$m timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); k=d['kernels']; print('mask$m', d['value'], d['ms_per_step'], 'bigvgan', round(sum(v['ms_per_step'] for kk, v in k.items() if 'bigvgan' in kk), 2), 'diffsvc-non-gate', round(sum(v['ms_per_step'] for kk, v in k.items() if 'diffsvc' in kk and 'gate_ws' not in kk and 'res_proj' not in kk), 2), 'whisper', round(sum(v['ms_per_step'] for kk, v in k.items() if 'whisper' in kk), 2))"
  done
done
