# GPU box, round 5: the ICP timeline with the level set-up stamped (timing build), and C2 A/B of
# two hop-2 polls in flight (IP_POLL2 = 4 and 16 sleeps apart).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5p
TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so timeout -k 10 120 python tools/icp_timeline.py > gpurun_out/r5p/icp_timeline.txt 2>&1 \
  || { tail -20 gpurun_out/r5p/icp_timeline.txt; exit 1; }
grep "level set-up" gpurun_out/r5p/icp_timeline.txt | cut -c1-330
bash tools/gpu_ab_lib.sh tree p2s4 p2s16 2>&1 | tee gpurun_out/r5p/ab.txt
