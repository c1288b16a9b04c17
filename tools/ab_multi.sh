# Same-box A/B of several libraries (run from the repo root via gpurun): LIBS = space-separated paths (first = base);
# parity tests on each non-base library (TESTS, -k TESTK), the micro benchmarks MICRO (amp, act) per library, then
# ROUNDS alternating quick benches.
set -o pipefail
O=gpurun_out/${TAG:-ab_multi}; mkdir -p $O
first=1
for L in $LIBS; do
  if [ $first = 0 ] && [ -n "${TESTS:-}" ]; then
    SVC_HIP_LIB=$PWD/$L timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > $O/tests.log 2>&1
    rc=$?; echo "$L: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { tail -40 $O/tests.log; exit $rc; }
  fi
  first=0
done
for L in $LIBS; do
  for m in ${MICRO:-}; do
    case $m in
      amp) SVC_HIP_LIB=$PWD/$L timeout -k 10 180 python3 tools/amp_bench.py > $O/m.txt 2>&1 || exit $? ;;
      act) SVC_HIP_LIB=$PWD/$L timeout -k 10 180 python3 tools/act_bench.py > $O/m.txt 2>&1 || exit $? ;;
    esac
    grep -v amdgpu $O/m.txt | sed "s#^#$(basename $L) $m: #"
  done
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in $LIBS; do
    SVC_HIP_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/b.json 2> $O/b.err || exit $?
    python3 - $O/b.json $(basename $L) <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
kind = lambda s: round(sum(v["ms_per_step"] for kk, v in k.items() if kk.startswith(s)), 3)
print(sys.argv[2], d["value"], d["ms_per_step"], "sclk", (d.get("clocks") or {}).get("sclk_mhz", {}).get("median"),
      "act", kind("activation1d"), "amp", kind("amp_conv"), "bigvgan",
      round(sum(v["ms_per_step"] for kk, v in k.items() if "@bigvgan" in kk), 2), flush=True)
PY
  done
done
