set -uo pipefail
R=$(pwd); O=$R/gpurun_out/gemmprof; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/gemm_bench.py -1 0 1 > $O/bench.txt 2>&1 || exit 1
cat $O/bench.txt
export GEMM_BENCH_SHAPES="dilated(store)"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "conv_gemm2_kernel<256, 128, 4, 2, 3, false>" -f csv -d $O/p$i -o run -- python3 $R/tools/gemm_bench.py 1 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; }
done
echo done
