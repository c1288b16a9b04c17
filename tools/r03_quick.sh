set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err || exit $?
tail -c 300 gpurun_out/r03a/bench.json
GEMM_BENCH_SHAPES="dilated(gate),outproj(split),skipsum,fc1,fc2" timeout -k 10 300 python3 tools/gemm_bench.py 15 24 > gpurun_out/r03a/gemm.txt 2>&1 || exit $?
timeout -k 10 120 python3 tools/att_bench.py > gpurun_out/r03a/att.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r03a/gemm.txt gpurun_out/r03a/att.txt
