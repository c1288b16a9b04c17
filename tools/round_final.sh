# Round-end check on the GPU box (run from the repo root via gpurun): the full GPU suite, smoke(), then the profile of
# record (tools/profile_round.sh: bench line with the CPU baseline, rocprof trace, PMC passes). TAG names the outputs.
set -o pipefail
T=${TAG:-final}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -2 gpurun_out/$T/smoke.log
TAG=$T bash tools/profile_round.sh
