set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stages.py -m gpu -k "fused_head or plms_and_ddpm" > gpurun_out/h_tests.log 2>&1 && \
for i in 1 2; do
  timeout -k 10 200 python bench.py > gpurun_out/h_b0_$i.json 2>gpurun_out/h_b0_$i.err && \
  SVC_DIFF_HEAD=1 timeout -k 10 200 python bench.py > gpurun_out/h_b1_$i.json 2>gpurun_out/h_b1_$i.err || exit 1
done && \
cd /tmp && export TMPDIR=/tmp && SVC_DIFF_HEAD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/hprof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/h_prof.log 2>&1
