# GPU box: the GPU suite on a library variant (TFUSION_HIP_LIB=tools/_build/V/libtfusion_hip.so),
# then the C2 A/B of that variant against the tree's library.  Outputs: gpurun_out/TAG/.
#   gpurun -- bash tools/gpu_variant_suite_ab.sh TAG V
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=$1; V=$2
O=gpurun_out/$TAG
mkdir -p $O
TFUSION_HIP_LIB=$PWD/tools/_build/$V/libtfusion_hip.so timeout -k 10 800 python -u -m pytest tests -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/tests_$V.log 2>&1 || { tail -40 $O/tests_$V.log; exit 1; }
tail -1 $O/tests_$V.log
bash tools/gpu_ab_lib.sh tree $V 2>&1 | tee $O/ab.txt
