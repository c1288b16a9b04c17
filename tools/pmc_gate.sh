set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  for v in 40 41; do
    GEMM_BENCH_TORCH=0 GEMM_BENCH_CUSTOM=29984,768,384,3,1 timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "gate_ws_kernel|dlayer_kernel" -f csv -d $O/p$i/v$v -o run -- python3 tools/gemm_bench.py $v 4 > $O/p${i}_$v.log 2>&1 || { echo "pass $i v$v failed"; tail -3 $O/p${i}_$v.log; exit 1; }
  done
  echo "pass $i done"
done
python3 tools/pmc_kernels.py $O $O/summary.json > $O/summary.txt; cat $O/summary.txt
