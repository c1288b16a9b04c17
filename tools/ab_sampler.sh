# Sampler launch-order A/B (run from the repo root via gpurun): sampler parity tests on the new build, then alternating
# quick benches of ab/libsvc_hip_base.so and the in-tree library, then (TRACE=1) a kernel trace of the new one.
set -o pipefail
O=gpurun_out/${TAG:-ab_sampler}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_ragged.py tests/test_gpu_headline.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "plms or ddpm or sub_streams or sampler or headline or ragged" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -30; exit $rc; }
TAG=${TAG:-ab_sampler} ROUNDS=${ROUNDS:-3} bash tools/ab_lib.sh || exit $?
if [ -n "${TRACE:-}" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- python3 bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline > $O/trace_bench.json 2> $O/trace_bench.err || exit $?
  python3 tools/stream_gaps.py $O/trace
fi
