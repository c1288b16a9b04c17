# Experiment A/B on one box (run from the repo root via gpurun): parity tests with the experiment on ($XON, env
# assignments), the gate GEMM microbenchmark and the sampler probe off / on, then alternating quick benches.
set -o pipefail
O=gpurun_out/${TAG:-r03x}; mkdir -p $O
XON=${XON:-SVC_X_A3=1}
env $XON timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_ragged.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "${TESTK:-gate or denoiser or eps or plms or sampler or ragged or bf16}" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -30; exit $rc; }
for x in off on; do
  E=""; [ $x = on ] && E="$XON"
  echo "== $x" > $O/m_$x.txt
  env $E GEMM_BENCH_TORCH=0 GEMM_BENCH_SHAPES="dilated(gate)" GEMM_BENCH_CUSTOM="29984,768,384,3,1;14992,768,384,3,1" \
    timeout -k 10 120 python3 tools/gemm_bench.py 24 >> $O/m_$x.txt 2>&1 || { cat $O/m_$x.txt; exit 1; }
  env $E timeout -k 10 180 python3 tools/sampler_probe.py '{}' '{"sampler_streams": 1}' >> $O/m_$x.txt 2>&1 || { cat $O/m_$x.txt; exit 1; }
  grep -v amdgpu $O/m_$x.txt | grep -v "^    " ; grep "dilated" $O/m_$x.txt
done
for r in 1 2; do
  for x in off on; do
    E=""; [ $x = on ] && E="$XON"
    env $E timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/b_$x.json 2> $O/b_$x.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/b_$x.json $x
  done
done
