# The GPU test suite in one process, then one quick bench (run from the repo root via gpurun).
# The two north-star tests at the headline 10 s clip length run the CPU oracle's DDPM-1000 (~1-2 min each).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-gpu}
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v -rA --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; grep -h "mel-L1" gpurun_out/${TAG}_tests.log | head; [ $rc -ne 0 ] && exit $rc
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
  tail -c 400 gpurun_out/${TAG}_bench.json
fi
