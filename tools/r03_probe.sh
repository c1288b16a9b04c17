# Sampler probe under kernel-site settings (run from the repo root via gpurun): PLMS-100, B = 32 x 937, wall time and
# the top kernel@site times per setting; each setting ("VAR=val,VAR=val" or "-") in its own process.
set -o pipefail
O=gpurun_out/${TAG:-r03probe}; mkdir -p $O
for cfg in ${PROBE_ENVS:--}; do
  envs=""; [ "$cfg" != "-" ] && envs=$(echo "$cfg" | tr ',' ' ')
  echo "== $cfg"
  env $envs timeout -k 10 180 python3 tools/sampler_probe.py '{}' > $O/p.txt 2>&1 || { cat $O/p.txt; exit 1; }
  grep -v amdgpu $O/p.txt
done
