# fused PLMS update (head epilogue) vs its own launch: parity tests, then alternating bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stages.py -m gpu -k "plms or fused_head or sub_streams or eps_gemm" > gpurun_out/p_tests.log 2>&1 || { tail -30 gpurun_out/p_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/p_tests.log | tail -2
for i in 1 2; do
  SVC_PLMS_FUSED=0 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/p_b0_$i.json 2>gpurun_out/p_b0_$i.err || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/p_b1_$i.json 2>gpurun_out/p_b1_$i.err || exit 1
done
