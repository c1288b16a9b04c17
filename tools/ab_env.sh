# Sampler probe and quick benches per environment setting, alternating (run from the repo root via gpurun).
# SETTINGS: space-separated "VAR=val,VAR=val" ("-" = defaults); ROUNDS: bench rounds; TESTK: optional parity tests first
set -o pipefail
O=gpurun_out/${TAG:-ab_env}; mkdir -p $O
if [ -n "${TESTK:-}" ]; then
  env ${TESTENV:-} timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_ragged.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "$TESTK" > $O/tests.log 2>&1
  rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -30; exit $rc; }
fi
for cfg in ${SETTINGS:--}; do
  envs=""; [ "$cfg" != "-" ] && envs=$(echo "$cfg" | tr ',' ' ')
  env $envs timeout -k 10 180 python3 tools/sampler_probe.py '{}' > $O/p.txt 2>&1 || { cat $O/p.txt; exit 1; }
  echo "probe $cfg: $(grep wall $O/p.txt) $(grep -h 'dilated\|outproj' $O/p.txt | awk '{printf "%s %s us; ", $1, $7}')"
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in ${SETTINGS:--}; do
    envs=""; [ "$cfg" != "-" ] && envs=$(echo "$cfg" | tr ',' ' ')
    env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', sys.argv[2], d['value'], d['ms_per_step'])" $O/b.json "$cfg"
  done
done
