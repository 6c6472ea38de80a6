# GPU box, round 5: the ICP rows split across SIMDs (IP_SPLIT) and without the division select
# wave-uniform branch, bitwise correspondence flags): parity (ICP / sequence / bench window, the
# OpenCV algebras), then C2 and C3I A/B against HEAD (tools/_build/head).
#   gpurun -- bash tools/gpu_r5_e.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r5e}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pose_algebra.py \
  -m gpu -x -q -rs --timeout 600 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
bash tools/gpu_ab_lib.sh tree nosplit head 2>&1 | tee $O/ab.txt
bash tools/gpu_ab_c3i.sh tree head 2>&1 | tee $O/ab_c3i.txt
