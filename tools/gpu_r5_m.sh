# GPU box, round 5: the ICP tail in row layout (IP_TAIL_ROWS): ICP parity (bit-exact against the
# oracle's scalar algebra), the debug timeline, C2 A/B against norows and HEAD.
#   gpurun -- bash tools/gpu_r5_m.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r5m}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 120 tools/micro/icp_tail > $O/icp_tail.txt 2>&1 || { tail -5 $O/icp_tail.txt; exit 1; }
head -3 $O/icp_tail.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pose_algebra.py tests/test_gpu_failures.py \
  -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so timeout -k 10 120 python tools/icp_timeline.py > $O/icp_timeline.txt 2>&1 \
  || { tail -20 $O/icp_timeline.txt; exit 1; }
tail -4 $O/icp_timeline.txt | cut -c1-200
bash tools/gpu_ab_lib.sh tree norows head 2>&1 | tee $O/ab.txt
