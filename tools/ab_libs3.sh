# A/B/C of library builds on one box, alternating: every ab/libsvc_hip_<name>.so listed in LIBS, ROUNDS rounds
set -o pipefail
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${LIBS}; do
    SVC_HIP_LIB=$PWD/ab/libsvc_hip_$lib.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab3_$lib.json 2> gpurun_out/ab3_$lib.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=sum(v['ms_per_step'] for n,v in d['kernels'].items() if n.endswith('@diffsvc.dilated')); print(sys.argv[2], d['value'], d['ms_per_step'], round(k,1), flush=True)" gpurun_out/ab3_$lib.json $lib
  done
done
