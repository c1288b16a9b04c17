# (round-5 driver) full GPU suite on the new build, GEMM microbench of the given shapes, then alternating benches
# against ab/libsvc_hip_base.so. TAG names the output directory under gpurun_out/.
set -o pipefail
T=${TAG:-r05}
O=gpurun_out/$T; mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -30; exit $rc; }
fi
if [ -n "${GEMM_SHAPES:-}" ]; then
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/ab/libsvc_hip_base.so; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    SVC_HIP_LIB=$L GEMM_BENCH_WARM=1 GEMM_BENCH_TORCH=${GEMM_TORCH:-0} GEMM_BENCH_SHAPES="$GEMM_SHAPES" timeout -k 10 300 python3 tools/gemm_bench.py 15 > $O/gemm_$lib.txt 2>&1 || { tail -5 $O/gemm_$lib.txt; exit 1; }
    grep -v amdgpu $O/gemm_$lib.txt | sed "s/^/$lib: /"
  done
fi
TAG=$T MICRO=${MICRO:-} ROUNDS=${ROUNDS:-2} bash tools/ab_lib.sh > $O/ab.txt 2>&1 || { tail -30 $O/ab.txt; exit 1; }
cat $O/ab.txt
python3 - $O ${KSEL:-melpre outproj whisper.fc whisper.qkv bigvgan} <<'PY'
import json, sys
for f in ("b_base.json", "b_new.json"):
    d = json.loads(open(sys.argv[1] + "/" + f).read().strip().splitlines()[-1])
    for n, v in sorted(d["kernels"].items()):
        if any(s in n for s in sys.argv[2:]):
            print(f, n, v["ms_per_step"], v["launches_per_step"], round(1000 * v["ms_per_step"] / v["launches_per_step"], 1))
PY
