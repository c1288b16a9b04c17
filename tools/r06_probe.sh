# Round 6 probe (run from the repo root via gpurun): the sampler tests touched this round, a quick bench, the PMC counter
# list, the long-context throughput record (BASELINE configs[3]: one 180 s song on one GPU) and the gate_ws step stamps
# at M = 29 984 / 14 992.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_headline.py -x -q --timeout 300 --timeout-method thread -k "head or res_proj or plms or gate_ws" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['calib_us'],d['clocks'].get('sclk_mhz'));k=d['kernels'];[print(n,v['ms_per_step'],v['launches_per_step']) for n,v in k.items() if 'diff_head' in n or 'mel_proj' in n or 'plms' in n]"
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || echo "counter list failed"
timeout -k 10 400 python3 bench.py --batch 1 --seconds 180 --steps 3 --warmup 1 --no-cpu-baseline > $O/long180.json 2> $O/long180.err || { tail -5 $O/long180.err; exit 1; }
tail -c 300 $O/long180.json
timeout -k 10 300 python3 tools/gws_stamps.py 29984 14992 > $O/stamps.txt 2>&1 || { tail -5 $O/stamps.txt; exit 1; }
cat $O/stamps.txt
