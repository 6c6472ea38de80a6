# GPU box, round 5: the ICP tail's 27 sums broadcast through LDS (tree, IP_SM_LDS=1) instead of
# readlanes (smlds0): ICP parity on the tree library, C2 A/B.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5x
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pose_algebra.py -m gpu -x -q -rs -k "icp or sequence or timed_window or pose" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
bash tools/gpu_ab_lib.sh tree smlds0 2>&1 | tee $O/ab.txt
TFUSION_HIP_LIB=$PWD/tools/_build/libtfusion_hip_timing.so timeout -k 10 200 python tools/icp_timeline.py > $O/icp_timeline.txt 2>&1 || { tail -20 $O/icp_timeline.txt; exit 1; }
grep -E "^it (1|9|15):|median" $O/icp_timeline.txt
