# GPU box, round 6: the persistent ICP's timeline (timing build) under the default algebra and
# under the canonical one.
#   gpurun -- bash tools/gpu_r6_tl.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6tl}
mkdir -p $O
TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so timeout -k 10 120 python tools/icp_timeline.py > $O/icp_timeline_opencv4.txt 2>&1 || { tail -20 $O/icp_timeline_opencv4.txt; exit 1; }
TFUSION_ICP_SOLVE=canonical TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so timeout -k 10 120 python tools/icp_timeline.py > $O/icp_timeline_canonical.txt 2>&1 || { tail -20 $O/icp_timeline_canonical.txt; exit 1; }
cut -c1-200 $O/icp_timeline_opencv4.txt | head -21
