#!/bin/bash
# Per-kernel hardware counters of one bench.py step (run from the repo root via gpurun): MFMA busy, LDS, HBM bytes
# for the GEMM / attention / activation kernels. rocprofv3 serialises dispatches while counting, so each dispatch's
# counters are its own. One pass per counter group (gfx950 limits: 8 SQ, 4 TCC, 2 GRBM per pass).
#   TAG: output dir under gpurun_out; KRE: kernel regex; PASSES: which counter passes (default 1 2 3 4; 3 / 4 = HBM
#   bytes, which tools/gpu_profile.sh also collects)
set -uo pipefail
R=$(pwd); TAG=${TAG:-pmc}; O=$R/gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
# a profiled pass writes nothing until it ends: tick a file under gpurun_out/ so the run is not taken for hung
( while sleep 30; do date +%s >> $R/gpurun_out/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
KRE=${KRE:-gate_ws_kernel|conv_gemm4_kernel|conv_gemm3_kernel|res_proj_kernel|mel_proj_kernel|diff_head_kernel|attention_kernel|amp_conv_kernel|activation1d}
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  case " ${PASSES:-1 2 3 4} " in *" $i "*) ;; *) continue ;; esac
  timeout -k 10 ${PASS_TIMEOUT:-300} rocprofv3 --pmc $set --kernel-include-regex "$KRE" -f csv -d $O/p$i -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/p$i.log 2>&1 || { rc=$?; echo "pass $i failed (exit $rc)"; tail -5 $O/p$i.log; exit 1; }
  echo "pass $i done"
done
[ -n "${NOSUM:-}" ] && exit 0  # passes split over calls: summarised where all of them are
python3 $R/tools/pmc_kernels.py $O $O/summary.json > $O/summary.txt && cat $O/summary.txt && rm -rf $O/p1 $O/p2 $O/p3 $O/p4
