# A/B of the BigVGAN up-sampling GEMM kernels (site bigvgan.ups): default, forced conv_gemm3 tiles
set -o pipefail
mkdir -p gpurun_out
for v in default 13 15; do
  if [ "$v" = default ]; then
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_ups_$v.json 2> gpurun_out/ab_ups_$v.err || exit $?
  else
    SVC_SITE_VARIANT="bigvgan.ups=$v" timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_ups_$v.json 2> gpurun_out/ab_ups_$v.err || exit $?
  fi
  python3 - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_ups_{sys.argv[1]}.json").read().strip().splitlines()[-1])
ups = {k: v["ms_per_step"] for k, v in d["kernels"].items() if k.endswith("@bigvgan.ups")}
print(sys.argv[1], d["value"], round(sum(ups.values()), 3), ups, flush=True)
PY
done
