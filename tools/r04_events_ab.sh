#!/bin/bash
# round 4: the cost of bench.py's live HIP-event markers in the timed region (BENCH_TIMED_EVENTS 1 vs 0, alternating),
# and the sampler's host enqueue time against its GPU time (tools/host_enqueue.py)
set -o pipefail
O=gpurun_out/${TAG:-r04m}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/host_enqueue.py > $O/enqueue.txt 2>&1 || exit $?
grep -v amdgpu $O/enqueue.txt
for r in 1 2 3; do
  for ev in 1 0; do
    BENCH_TIMED_EVENTS=$ev ${EXTRA_ENV:-} timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b_$ev.json 2> $O/b_$ev.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b_$ev.json').read().strip().splitlines()[-1]); r=d['roofline']; print('events=$ev', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'])"
  done
done
