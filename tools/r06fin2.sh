set -o pipefail
T=r06fin; mkdir -p gpurun_out/$T
timeout -k 10 400 python3 bench.py --batch 1 --seconds 180 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$T/long180.json 2> gpurun_out/$T/long180.err || { tail -5 gpurun_out/$T/long180.err; exit 1; }
tail -c 300 gpurun_out/$T/long180.json; echo
TAG=${T}_pmc PASSES="3 4" NOSUM=1 PASS_TIMEOUT=400 bash tools/pmc_kernels.sh || exit 1
SET="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU GRBM_GUI_ACTIVE"
O=gpurun_out/${T}_issue; mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "gate_ws_kernel" -f csv -d $O/p5 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/p5.log 2>&1 && echo "issue pass done"
