# GPU box: PMC traffic passes for the C3-scale configs (C3 frames, C3I, C3R) with the current kernels.
set -e
R=$GRAFT_REPO_ROOT
cd $R
for cfg in C3I C3R C3; do
  timeout -k 10 500 bash tools/gpu_pmc.sh r3_$cfg $cfg > gpurun_out/pmc_r3_$cfg.log 2>&1 || { tail -20 gpurun_out/pmc_r3_$cfg.log; exit 1; }
  python3 tools/pmc_traffic.py gpurun_out/pmc_r3_$cfg $cfg gpurun_out/pmc_traffic_r3.json > /dev/null
  echo "$cfg done"
done
cat gpurun_out/pmc_traffic_r3.json
