# A/B of two builds of libsvc_hip.so on one box: ab/libsvc_hip_base.so (reference build) against the in-tree library,
# alternating, N rounds (default 2). Prints audio-s/s and the per-site kernel times named in SITES.
set -o pipefail
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
SITES=${SITES:-diffsvc.outproj,bigvgan.amp_c2,bigvgan.amp_c1,whisper.out,whisper.fc2}
for r in $(seq 1 $ROUNDS); do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/ab/libsvc_hip_base.so; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    SVC_HIP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_$lib.json 2> gpurun_out/ab_$lib.err || exit $?
    python3 - $lib "$SITES" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
sites = sys.argv[2].split(",")
ks = {s: round(sum(v["ms_per_step"] for k, v in d["kernels"].items() if k.endswith("@" + s)), 3) for s in sites}
print(sys.argv[1], d["value"], d["ms_per_step"], ks, flush=True)
PY
  done
done
