# Config-5 fp16-vs-bf16 precision sweep on MI355X (run from the repo root via gpurun):
# tools/precision_sweep.py --gpu --bf16 writes the JSON under gpurun_out/$TAG (copy it to profiles/).
set -o pipefail
O=gpurun_out/${TAG:-sweep}; mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1200 python3 -u tools/precision_sweep.py --content ${CONTENT:-contentvec} --gpu --bf16 --no-emu ${SWEEP_ARGS:-} \
  > $O/precision_sweep.json 2> $O/precision_sweep.err || { tail -20 $O/precision_sweep.err; exit 1; }
tail -c 2000 $O/precision_sweep.json
