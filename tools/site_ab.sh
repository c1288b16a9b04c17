set -o pipefail
mkdir -p gpurun_out
i=0
for sv in "-" "bigvgan.amp_c1=20" "bigvgan.amp_c2=20" "whisper.fc1=20" "bigvgan.ups=20"; do
  i=$((i+1))
  if [ "$sv" = "-" ]; then unset SVC_SITE_VARIANT; else export SVC_SITE_VARIANT="$sv"; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/sab_$i.log 2>&1 || exit $?
  python3 - gpurun_out/sab_$i.log "$sv" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
site = sys.argv[2].split("=")[0]
ks = {k: v["ms_per_step"] for k, v in d["kernels"].items() if site != "-" and k.endswith("@" + site)}
print(sys.argv[2], d["value"], d["ms_per_step"], ks)
PY
done
