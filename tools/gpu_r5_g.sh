# GPU box, round 5: C2 A/B of ICP variants by register footprint (tools/_build: allold, oldrcpbr,
# pc8old, pc8w0, pc8tree) against HEAD.   gpurun -- bash tools/gpu_r5_g.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r5g}
O=gpurun_out/$TAG
mkdir -p $O
bash tools/gpu_ab_lib.sh allold oldrcpbr pc8old pc8w0 pc8tree head 2>&1 | tee $O/ab.txt
