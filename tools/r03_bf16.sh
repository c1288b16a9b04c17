# Attention microbenchmark + the bf16 operand variant on MI355X: its stage tests, then the full GPU suite + bench,
# then the config-5 fp16-vs-bf16 precision sweep. Run from the repo root via gpurun.
set -o pipefail
O=gpurun_out/r03_bf16; mkdir -p $O
for i in 1 2; do timeout -k 10 120 python3 tools/att_bench.py > $O/att_$i.txt 2>&1 || exit $?; grep -v amdgpu $O/att_$i.txt; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_configs.py -m gpu -x -v -rA --timeout 300 --timeout-method thread -k "bf16" > $O/bf16_tests.log 2>&1
rc=$?; tail -5 $O/bf16_tests.log; grep -h "mel-L1\|rel" $O/bf16_tests.log | head -20; [ $rc -ne 0 ] && exit $rc
TAG=r03_bf16/full BENCH=1 bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --operands bf16 > $O/bench_bf16.json 2> $O/bench_bf16.err || exit $?
tail -c 300 $O/bench_bf16.json
timeout -k 10 900 python3 -u tools/precision_sweep.py --content contentvec --gpu --bf16 --no-emu > $O/precision_sweep.json 2> $O/precision_sweep.err || exit $?
cat $O/precision_sweep.json
