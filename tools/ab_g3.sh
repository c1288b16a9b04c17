set -o pipefail
O=gpurun_out/r03ab; mkdir -p $O
TAG=r03ab TESTS=tests/test_gpu_ops.py MICRO="g3" ROUNDS=2 bash tools/ab_lib.sh > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
for g in ${GROUPS_MICRO:-}; do
  SVC_G3_GROUP=$g GEMM_BENCH_SHAPES="outproj(split,whisper.fc,skipsum,bigvgan.s2" timeout -k 10 180 python3 tools/gemm_bench.py 15 > $O/m.txt 2>&1 || { cat $O/m.txt; exit 1; }
  grep -v amdgpu $O/m.txt | sed "s/^/group $g: /" >> $O/ab.log
done
for g in ${GROUPS_BENCH:-}; do
  SVC_G3_GROUP=$g timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench group', sys.argv[2], d['value'], d['ms_per_step'])" $O/b.json $g >> $O/ab.log
done
cat $O/ab.log
