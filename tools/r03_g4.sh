# Experiment: gate GEMM variants (SVC_X_G4 = 1 interior-tile DMA without per-lane selects, 2 first fragments before
# the DMA issue, 3 both) vs the default (0)
set -o pipefail
O=gpurun_out/r03_g4; mkdir -p $O
for c in 1 3; do
  SVC_X_G4=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gate_gemm_ragged or eps_gemm_variants or plms" > $O/tests_$c.log 2>&1 || { tail -20 $O/tests_$c.log; exit 1; }
  tail -1 $O/tests_$c.log
done
for c in 0 1 2 3 0 1 2 3; do
  SVC_X_G4=$c GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM="29984,768,384,3,1;14992,768,384,3,1" timeout -k 10 120 python3 tools/gemm_bench.py 24 2>&1 | grep -v amdgpu | sed "s/^/g4=$c /"
done
for c in 0 1 2 3 0 1 2 3; do
  SVC_X_G4=$c timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); print('g4=$c', d['value'], d['roofline']['avg_launch_us'], d['roofline']['concurrent']['avg_launch_us'])"
done
