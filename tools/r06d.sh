# Round 6: parity of this round's kernel changes (gate_ws preamble stores, diff_head epilogue waits, fused PLMS,
# persistent conv_gemm3), then a same-box A/B of the persistent GEMM (SVC_GEMM3_DIRECT 19 vs 3) and of the PLMS
# epilogue (SVC_DIFF_HEAD 2 vs 1), alternating (run from the repo root via gpurun).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06d}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_ops.py tests/test_gpu_headline.py -x -q --timeout 600 --timeout-method thread -k "gate_ws or head or plms or conv1d_persistent or persistent_gemm or headline_batch or test_conv1d or bigvgan or whisper_medium" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for cfg in "3 1" "19 1" "19 2"; do
    set -- $cfg
    SVC_GEMM3_DIRECT=$1 SVC_DIFF_HEAD=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-calib --steps 3 --warmup 1 > $O/ab_$1_$2.json 2> $O/ab_$1_$2.err || exit $?
    python3 - $O/ab_$1_$2.json "g3d=$1 dh=$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
fam = {}
for n, v in k.items():
    f = n.split("@")[0].split("<")[0]
    fam[f] = fam.get(f, 0) + v["ms_per_step"]
site = {}
for n, v in k.items():
    s = n.split("@")[1].split(".")[0] if "@" in n else n
    site[s] = site.get(s, 0) + v["ms_per_step"]
g = {n: round(v["ms_per_step"], 2) for n, v in k.items() if "whisper.fc1" in n or "whisper.qkv" in n or "amp_c2" in n and "gemm" in n}
print(sys.argv[2], d["value"], d["ms_per_step"], d["clocks"].get("sclk_mhz", {}).get("median"), d["roofline"]["avg_launch_us"],
      {f: round(v, 1) for f, v in sorted(fam.items(), key=lambda x: -x[1])[:9]}, {s: round(v, 1) for s, v in site.items()}, g)
PY
  done
done
