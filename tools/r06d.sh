# Round 6: parity of this round's kernel changes (gate_ws preamble stores, diff_head epilogue waits, fused PLMS,
# persistent conv_gemm3, amp_conv epilogue loads), then same-box A/Bs, alternating (run from the repo root via gpurun):
# the persistent GEMM (SVC_GEMM3_DIRECT 19 vs 3), the PLMS epilogue (SVC_DIFF_HEAD 2 vs 1) and, when
# ab/libsvc_hip_base.so exists, that library (the previous commit) against the tree's.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06d}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_ops.py tests/test_gpu_headline.py -x -q -rA --timeout 600 --timeout-method thread -k "${TESTK:-gate_ws or head or plms or conv1d_persistent or persistent_gemm or headline_batch or test_conv1d or bigvgan or whisper_medium or amp_conv or activation1d}" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log; grep -h "persistent launches" $O/tests.log | head -3
summ() {
python3 - $1 "$2" <<'PY'
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
g = {n: round(v["ms_per_step"], 2) for n, v in k.items() if "whisper.fc1" in n or "whisper.qkv" in n or "amp_c2" in n}
print(sys.argv[2], d["value"], d["ms_per_step"], d["clocks"].get("sclk_mhz", {}).get("median"), d["roofline"]["avg_launch_us"],
      {f: round(v, 1) for f, v in sorted(fam.items(), key=lambda x: -x[1])[:10]}, {s: round(v, 1) for s, v in site.items()}, g, flush=True)
PY
}
for r in 1 2; do
  for cfg in ${ARMS:-"3 1" "19 1" "19 2"}; do
    set -- $(echo $cfg | tr ',' ' ')
    SVC_GEMM3_DIRECT=$1 SVC_DIFF_HEAD=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-calib --steps 3 --warmup 1 > $O/ab_$1_$2.json 2> $O/ab_$1_$2.err || exit $?
    summ $O/ab_$1_$2.json "g3d=$1 dh=$2"
  done
  if [ -f ab/libsvc_hip_base.so ]; then
    SVC_HIP_LIB=$PWD/ab/libsvc_hip_base.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-calib --steps 3 --warmup 1 > $O/ab_base.json 2> $O/ab_base.err || exit $?
    summ $O/ab_base.json "base lib"
  fi
done
