# GPU box, round 5: (1) the memory-model ICP hand-off (-DIP_XCD_STORE=0, tools/_build/xcd0) through
# the ICP / sequence / bench-window parity tests; (2) C2 A/B of the tree against the ICP-tail
# variants (ldl: LDL^T solve, pdiv: IEEE division for RN(1/z), both) and xcd0.
#   gpurun -- bash tools/gpu_r5_d.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r5d}
O=gpurun_out/$TAG
mkdir -p $O
TFUSION_HIP_LIB=$PWD/tools/_build/xcd0/libtfusion_hip.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -x -q -rs -k "icp_stage or sequence or bench_timed_window" --timeout 600 --timeout-method thread > $O/tests_xcd0.log 2>&1 \
  || { tail -30 $O/tests_xcd0.log; exit 1; }
tail -n 1 $O/tests_xcd0.log
bash tools/gpu_ab_lib.sh tree ldl pdiv both idiv xcd0 2>&1 | tee $O/ab.txt
bash tools/gpu_ab_c3i.sh tree idiv 2>&1 | tee $O/ab_c3i.txt
