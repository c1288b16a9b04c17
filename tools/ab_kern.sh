# Alternating end-to-end A/B of environment settings with the bench line's per-kernel split (run from the repo root via
# gpurun). SETTINGS: space-separated "VAR=val,VAR=val" ("-" = defaults); ROUNDS: rounds; KPAT: regex of the `kernels`
# entries to print; TESTK: optional GPU tests (-k expression) first, under TESTENV ("VAR=val ..."). Exit codes 0 / 1 of the tests (pass / assertion
# failures) go on to the benches; anything else (a fault, an abort, a time limit) stops the script.
set -o pipefail
O=gpurun_out/${TAG:-ab_kern}; mkdir -p $O
if [ -n "${TESTK:-}" ]; then
  env ${TESTENV:-} timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTK" > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log
  [ $rc -eq 1 ] && grep -E "^E |assert" $O/tests.log | head -20
  [ $rc -gt 1 ] && exit $rc
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in ${SETTINGS:--}; do
    envs=""; [ "$cfg" != "-" ] && envs=$(echo "$cfg" | tr ',' ' ')
    env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    cp $O/b.json "$O/b_${r}_$(echo "$cfg" | tr '=,/' '__-').json"
    python3 - $O/b.json "$cfg" "${KPAT:-.}" <<'PY'
import json, re, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = {k: v["ms_per_step"] for k, v in d.get("kernels", {}).items() if re.search(sys.argv[3], k)}
print("bench", sys.argv[2], d["value"], d["ms_per_step"], "sclk", d.get("clocks", {}).get("sclk_mhz", {}).get("median"),
      "calib", d.get("calib_us"), "|", " ".join(f"{k}={v:.3f}" for k, v in sorted(ks.items())), "| sum", round(sum(ks.values()), 3))
PY
  done
done
