# Round 6: the full GPU suite on the current tree, the gate_ws step stamps, then a same-box A/B of the tree's library
# against ab/libsvc_hip_base.so (the tree with round 5's gate_ws.hip and amp_conv.hip), alternating.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06e}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 tools/gws_stamps.py 29984 14992 > $O/stamps.txt 2>&1 || { tail -5 $O/stamps.txt; exit 1; }
grep -E "M=|per step|k % 3" $O/stamps.txt
summ() {
python3 - $1 "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
fam = {}
for n, v in k.items():
    f = n.split("@")[0].split("<")[0]
    fam[f] = fam.get(f, 0) + v["ms_per_step"]
g = {n.split("@")[0] + "@" + n.split("@")[1].split(".")[1]: round(v["ms_per_step"], 2) for n, v in k.items() if "amp_conv" in n or "diff_head" in n}
print(sys.argv[2], d["value"], d["ms_per_step"], d["clocks"].get("sclk_mhz", {}).get("median"), d["roofline"]["avg_launch_us"],
      {f: round(v, 2) for f, v in sorted(fam.items(), key=lambda x: -x[1])[:9]}, g, flush=True)
PY
}
for r in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then L=$PWD/ab/libsvc_hip_base.so; else L=$PWD/svc_inference_pipeline_amd/libsvc_hip.so; fi
    SVC_HIP_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-calib --steps 3 --warmup 1 > $O/b_$lib.json 2> $O/b_$lib.err || exit $?
    summ $O/b_$lib.json $lib
  done
done
