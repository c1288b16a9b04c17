# res_proj.hip check on one box (run from the repo root via gpurun): its parity tests, the residual-projection
# microbenchmark (conv_gemm3 v15 against res_proj v30, warm and after a cache flush), then alternating quick benches
# with the stream (SVC_RES_PROJ=1) and the tiled GEMM (0).
set -o pipefail
O=gpurun_out/${TAG:-r03i}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stages.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "res_proj or denoiser or bf16_eps or eps_gemm or plms_and_ddpm or sampler_sub" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -30; exit $rc; }
: > $O/gemm.txt
for dep in ${RP_DEPTHS:-3}; do
  echo "ring depth $dep" >> $O/gemm.txt
  SVC_RP_DEPTH=$dep GEMM_BENCH_TORCH=0 GEMM_BENCH_SHAPES="outproj(split" timeout -k 10 120 python3 tools/gemm_bench.py 15 30 >> $O/gemm.txt 2>&1 || { cat $O/gemm.txt; exit 1; }
  SVC_RP_DEPTH=$dep GEMM_BENCH_COLD=1 GEMM_BENCH_TORCH=0 GEMM_BENCH_SHAPES="outproj(split" timeout -k 10 120 python3 tools/gemm_bench.py 15 30 >> $O/gemm.txt 2>&1 || { cat $O/gemm.txt; exit 1; }
done
grep -v amdgpu $O/gemm.txt
for r in 1 2; do
  for v in ${RP_SETTINGS:-1 0}; do for dep in $([ $v = 0 ] && echo 3 || echo ${RP_DEPTHS:-3}); do
    SVC_RP_DEPTH=$dep SVC_RES_PROJ=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/b_$v.json 2> $O/b_$v.err || exit $?
    python3 - $O/b_$v.json $v $dep <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
pick = lambda s: round(sum(v["ms_per_step"] for kk, v in k.items() if kk.endswith("@" + s)), 3)
print("res_proj", sys.argv[2], "depth", sys.argv[3], d["value"], d["ms_per_step"], "dil", pick("diffsvc.dilated"), "outproj", pick("diffsvc.outproj"), flush=True)
PY
  done
  done
done
