# GPU box, round 5: ROUND(x) as x + copysign(0.5, x) (tree, TF_ROUND_BFI=1) against compare + select
# (rnd0): raycast / sequence parity on the tree, C2 A/B.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5aa
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rs -k "raycast or sequence or render or timed_window or c3" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
bash tools/gpu_ab_lib.sh tree rnd0 2>&1 | tee $O/ab.txt
bash tools/gpu_ab_lib.sh tree rnd0 2>&1 | tee -a $O/ab.txt
