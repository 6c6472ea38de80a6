# GPU box, round 5: the whole GPU suite on the tree (16-bit dist codes sampled by the integration),
# then C3I and C2 A/B against f32d (the float dists) and HEAD.
#   gpurun -- bash tools/gpu_r5_i.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r5i}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
bash tools/gpu_ab_c3i.sh tree f32d head 2>&1 | tee $O/ab_c3i.txt
bash tools/gpu_ab_lib.sh tree f32d head 2>&1 | tee $O/ab.txt
