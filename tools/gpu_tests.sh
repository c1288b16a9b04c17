# The GPU test suite in one process, then one quick bench (run from the repo root via gpurun).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-gpu}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
  tail -c 400 gpurun_out/${TAG}_bench.json
fi
