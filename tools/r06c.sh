# Round 6: gate_ws period-3 counters, then a same-box A/B of the PLMS update in diff_head's epilogue (SVC_DIFF_HEAD 2)
# against its own launch (1), alternating (run from the repo root via gpurun).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06c}; mkdir -p $O
TAG=${TAG:-r06c} bash tools/pmc_gate_period.sh > $O/gate_period.txt 2>&1 || { tail -20 $O/gate_period.txt; exit 1; }
cat $O/gate_period.txt
for r in 1 2; do
  for v in 1 2; do
    SVC_DIFF_HEAD=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-calib --steps 3 --warmup 1 > $O/ab_dh$v.json 2> $O/ab_dh$v.err || exit $?
    python3 -c "import json,sys;d=json.loads(open('$O/ab_dh$v.json').read().strip().splitlines()[-1]);k=d['kernels'];print('diff_head=$v',d['value'],d['ms_per_step'],d['clocks'].get('sclk_mhz',{}).get('median'),[(n,v['ms_per_step']) for n,v in k.items() if 'diff_head' in n or 'mel_proj' in n])"
  done
done
