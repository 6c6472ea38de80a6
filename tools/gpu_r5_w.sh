# GPU box, round 5: issue priority for the ray tiles that were long in the previous frame
# (TF_PAIR_PRIO_US 15 / 25 / 35): raycast parity on one, C2 A/B against the tree.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5w
mkdir -p $O
TFUSION_HIP_LIB=$PWD/tools/_build/prio25/libtfusion_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rs -k "raycast or sequence or render or timed_window" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
bash tools/gpu_ab_lib.sh tree prio15 prio25 prio35 2>&1 | tee $O/ab.txt
