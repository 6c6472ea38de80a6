# GPU box, round 5: the stand-alone integration pass with a lane's four voxels along y (tools/_build/
# ycol, TF_INTEG_PASS_YCOL): the C3 parity tests on it, then C3I A/B against the tree.
#   gpurun -- bash tools/gpu_r5_n.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r5n}
O=gpurun_out/$TAG
mkdir -p $O
TFUSION_HIP_LIB=$PWD/tools/_build/ycol/libtfusion_hip.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -rs -k "c3 or stage or integrate or engine" \
  --timeout 300 --timeout-method thread > $O/tests_ycol.log 2>&1 || { tail -30 $O/tests_ycol.log; exit 1; }
tail -n 1 $O/tests_ycol.log
bash tools/gpu_ab_c3i.sh ycol tree 2>&1 | tee $O/ab_c3i.txt
