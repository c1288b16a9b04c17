# Profile of record at HEAD (run from the repo root via gpurun): bench line with the CPU baseline, rocprofv3
# kernel-trace stats, FETCH_SIZE / WRITE_SIZE passes on the roofline kernel (tools/gpu_profile.sh), then the per-kernel
# PMC passes (MFMA busy, VALU / MFMA, LDS conflicts, HBM bytes: tools/pmc_kernels.sh).
set -o pipefail
TAG=${TAG:-r03prof}
bash tools/gpu_profile.sh $TAG > gpurun_out/${TAG}_profile.log 2>&1 || { tail -20 gpurun_out/${TAG}_profile.log; exit 1; }
tail -5 gpurun_out/${TAG}_profile.log
TAG=${TAG}_pmc bash tools/pmc_kernels.sh > gpurun_out/${TAG}_pmc.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc.log; exit 1; }
head -40 gpurun_out/${TAG}_pmc.log
