# GPU box, round 6: the lane-parallel SVD micro only (bits vs serial + oracle, latency, counts).
#   gpurun -- bash tools/gpu_r6_micro.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6m}
mkdir -p $O
timeout -k 10 200 ./tools/micro/svd_lanes tests/golden/icp_systems_C2_opencv4.f32 > $O/svd_lanes.txt 2>&1
timeout -k 10 200 ./tools/micro/svd_lanes_stats tests/golden/icp_systems_C2_opencv4.f32 > $O/svd_lanes_stats.txt 2>&1
cat $O/svd_lanes.txt
head -3 $O/svd_lanes_stats.txt
timeout -k 10 200 ./tools/micro/svd_lanes_timing tests/golden/icp_systems_C2_opencv4.f32 > $O/svd_lanes_timing.txt 2>&1
tail -9 $O/svd_lanes_timing.txt
