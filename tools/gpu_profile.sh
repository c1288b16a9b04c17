#!/bin/bash
# Round profiling on the GPU box (run from the repo root via gpurun):
#   1. bench.py (N=1, with the CPU baseline)              -> gpurun_out/$TAG/bench.json
#   2. rocprofv3 --kernel-trace --stats of the same bench -> gpurun_out/$TAG/trace/*kernel_stats.csv
#   3. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) on the dominant kernel family
# Every GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
TAG=${1:-prof}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# a profiled pass writes nothing until it ends: tick a file under gpurun_out/ so the run is not taken for hung
( while sleep 30; do date +%s >> $R/gpurun_out/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
STEPS=${STEPS:-3}
if [ -z "${PMC_ONLY:-}" ]; then
timeout -k 10 900 python3 bench.py --steps $STEPS --warmup 1 > $OUT/bench.json 2> $OUT/bench.err
echo "bench done"; tail -c 600 $OUT/bench.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace_bench.err
echo "trace done"
fi
# rocprofv3 matches the kernel symbol as recorded (templates with bool parameters stay mangled): derive the
# regex of bench.py's dominant kernel tag, e.g. conv_gemm3<128,128,pair> -> conv_gemm3_kernelILi128ELi128ELb.ELb1E
if [ -z "${KRE:-}" ]; then
  KRE=$(python3 - "$OUT/bench.json" <<'PY'
import json, re, sys
tag = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["roofline"]["kernel"]
m = re.match(r"conv_gemm3<(\d+),(\d+)(,pair)?>", tag)
m4 = re.match(r"conv_gemm4<128,128(,pair|,gate)?>", tag)
if m:
    print(f"conv_gemm3_kernelILi{m[1]}ELi{m[2]}ELb.ELb{1 if m[3] else 0}E")
elif m4:
    print(f"conv_gemm4_kernelILb.ELb{1 if m4[1] else 0}ELb{1 if m4[1] == ',gate' else 0}E")
else:
    print(tag.split("<")[0])
PY
)
fi
echo "PMC kernel regex: $KRE"
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $OUT/pmc_fetch.err
echo "pmc fetch done"
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $OUT/pmc_write.err
echo "pmc write done"
find $OUT -name "*.csv" | head -20
