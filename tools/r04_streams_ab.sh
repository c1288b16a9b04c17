#!/bin/bash
# round 4: sub-batch streams of the vocoder and the Whisper encoder (tune.vocoder_streams / whisper_streams, default
# 1 / 1) with the round-4 kernels: end to end alternating
set -o pipefail
O=gpurun_out/${TAG:-r04aa}; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
  for vw in 1,1 2,1 1,2 2,2; do
    v=${vw%,*}; w=${vw#*,}
    SVC_VOCODER_STREAMS=$v SVC_WHISPER_STREAMS=$w timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); k=d['kernels']; print('voc$v whisper$w', d['value'], d['ms_per_step'])"
  done
done
