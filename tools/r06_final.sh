# Round-6 record (run from the repo root via gpurun): tools/round_final.sh (full GPU suite, smoke(), bench line with the
# CPU baseline, rocprof trace, PMC passes) then the long-context throughput line (BASELINE configs[3]: one 180 s song on
# one GPU). TAG names the outputs.
set -o pipefail
T=${TAG:-r06fin}
TAG=$T bash tools/round_final.sh || exit $?
timeout -k 10 400 python3 bench.py --batch 1 --seconds 180 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$T/long180.json 2> gpurun_out/$T/long180.err || { tail -5 gpurun_out/$T/long180.err; exit 1; }
tail -c 400 gpurun_out/$T/long180.json
