# DiffSVC input-projection (melpre) tile per call site (SVC_SITE_VARIANT), 3-stream PLMS-100 sampler wall time
set -o pipefail
mkdir -p gpurun_out
for v in "" 10 11 12 13 14 20 24 ""; do
  if [ -n "$v" ]; then export SVC_SITE_VARIANT="diffsvc.melpre=$v"; else unset SVC_SITE_VARIANT; fi
  timeout -k 10 120 python3 -u tools/sampler_probe.py "{}" > gpurun_out/mps_$v.log 2>&1 || exit $?
  echo "variant ${v:-default}: $(grep -m1 wall gpurun_out/mps_$v.log) $(grep -m1 melpre gpurun_out/mps_$v.log)"
done
