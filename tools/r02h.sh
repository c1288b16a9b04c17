# host enqueue vs GPU time of the sampler, and a kernel trace of one bench step (timeline / idle analysis)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r02h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python3 tools/host_enqueue.py > $O/host_enqueue.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || exit $?
find $O -name "*.csv" | head
