# GPU box, round 5: ICP parity on the tree (8 hop-2 copies, reciprocal branch), the debug
# timeline, and C2 A/B against okshort (short-circuit flags), pc1 (one hop-2 copy) and HEAD.
#   gpurun -- bash tools/gpu_r5_h.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r5h}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pose_algebra.py \
  -m gpu -x -q -rs -k "icp or sequence or bench_timed_window or algebra" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so timeout -k 10 120 python tools/icp_timeline.py > $O/icp_timeline.txt 2>&1 \
  || { tail -20 $O/icp_timeline.txt; exit 1; }
tail -3 $O/icp_timeline.txt | cut -c1-250
bash tools/gpu_ab_lib.sh tree okshort pc1 head 2>&1 | tee $O/ab.txt
