# GPU box: parity of a library variant (GPU parity tests through TFUSION_HIP_LIB), then an A/B of
# it against the tree's library on C2.   gpurun -- bash tools/gpu_ab_check.sh VARIANT [pytest files...]
set -e
cd $GRAFT_REPO_ROOT
V=$1; shift
SEL=${@:-tests/test_gpu_parity.py}
mkdir -p gpurun_out/ab
TFUSION_HIP_LIB=$PWD/tools/_build/$V/libtfusion_hip.so timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/ab/tests_$V.log 2>&1 || { tail -30 gpurun_out/ab/tests_$V.log; exit 1; }
tail -1 gpurun_out/ab/tests_$V.log
bash tools/gpu_ab_lib.sh tree $V
