# Same-box A/B of ab/libsvc_hip_base.so (or $BASE_LIB) against the in-tree library (run from the repo root via gpurun):
# parity tests on the new build ($TESTS, -k $TESTK), then alternating microbenchmarks ($MICRO: att, gate, outproj, g3, amp)
# and quick benches (ROUNDS).
set -o pipefail
O=gpurun_out/${TAG:-ab_lib}; mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { tail -40 $O/tests.log; exit $rc; }
fi
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/${BASE_LIB:-ab/libsvc_hip_base.so}; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    for m in ${MICRO:-}; do
      case $m in
        att) SVC_HIP_LIB=$L timeout -k 10 120 python3 tools/att_bench.py > $O/m.txt 2>&1 || exit $? ;;
        gate) SVC_HIP_LIB=$L GEMM_BENCH_SHAPES="dilated(gate)" timeout -k 10 120 python3 tools/gemm_bench.py 24 > $O/m.txt 2>&1 || exit $? ;;
        outproj) SVC_HIP_LIB=$L GEMM_BENCH_TORCH=0 GEMM_BENCH_SHAPES="outproj(split" timeout -k 10 120 python3 tools/gemm_bench.py 15 30 > $O/m.txt 2>&1 || exit $? ;;
        amp) SVC_HIP_LIB=$L timeout -k 10 180 python3 tools/amp_bench.py > $O/m.txt 2>&1 || exit $? ;;
        act) SVC_HIP_LIB=$L timeout -k 10 180 python3 tools/act_bench.py > $O/m.txt 2>&1 || exit $? ;;
        g3) SVC_HIP_LIB=$L GEMM_BENCH_SHAPES="outproj(split,whisper.fc,skipsum,bigvgan.s2" timeout -k 10 180 python3 tools/gemm_bench.py 15 > $O/m.txt 2>&1 || exit $? ;;
      esac
      grep -v amdgpu $O/m.txt | sed "s/^/$lib $m: /"
    done
  done
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/${BASE_LIB:-ab/libsvc_hip_base.so}; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    SVC_HIP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/b_$lib.json 2> $O/b_$lib.err || exit $?
    python3 - $O/b_$lib.json $lib <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
pick = lambda s: round(sum(v["ms_per_step"] for kk, v in k.items() if kk.endswith("@" + s)), 3)
kind = lambda s: round(sum(v["ms_per_step"] for kk, v in k.items() if kk.startswith(s)), 3)
print(sys.argv[2], d["value"], d["ms_per_step"], "sclk", (d.get("clocks") or {}).get("sclk_mhz", {}).get("median"), "calib_us", d.get("calib_us"), "att", pick("whisper.qkv"), "dil", pick("diffsvc.dilated"), "outproj", pick("diffsvc.outproj"), "roof_us", d["roofline"].get("avg_launch_us"), "act", kind("activation1d"), "amp", kind("amp_conv"), "g3", kind("conv_gemm3"), "bigvgan", round(sum(v["ms_per_step"] for kk, v in k.items() if "@bigvgan" in kk), 2), flush=True)
PY
  done
done
