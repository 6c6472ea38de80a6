# GPU box, round 5: long ray tiles (previous frame > RAY_PF_US) prefetch their rays' segments
# (grid cells + voxel lines) before the march: raycast parity on pf30, C2 A/B against the tree.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5z
mkdir -p $O
TFUSION_HIP_LIB=$PWD/tools/_build/pf30/libtfusion_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rs -k "raycast or sequence or render or timed_window" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
bash tools/gpu_ab_lib.sh tree pf30 pf30b4 pf30g pf20 2>&1 | tee $O/ab.txt
