# head-epilogue fusions A/B: off (separate PLMS update + input projection), PLMS only, PLMS + next input projection
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  SVC_PLMS_FUSED=0 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/q_off_$i.json 2>gpurun_out/q_off_$i.err || exit 1
  SVC_MELPRE_FUSED=0 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/q_plms_$i.json 2>gpurun_out/q_plms_$i.err || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/q_both_$i.json 2>gpurun_out/q_both_$i.err || exit 1
done
