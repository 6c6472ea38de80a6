# GPU box, round 5: the ICP rows' SIMD placement (tools/micro/wave_simd), then ICP parity on the
# tree (virtual-wave roles, split CTAs, wave-0 hop-2 gather, pair-merged reciprocal branch) and
# on pcopy8, then C2 A/B of the tree against one-switch-off variants and HEAD.
#   gpurun -- bash tools/gpu_r5_f.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r5f}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 60 tools/micro/wave_simd | tee $O/wave_simd.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pose_algebra.py tests/test_gpu_failures.py \
  -m gpu -x -q -rs --timeout 500 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
TFUSION_HIP_LIB=$PWD/tools/_build/pcopy8/libtfusion_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -x -q -rs -k "icp_stage or sequence or bench_timed_window" --timeout 300 --timeout-method thread > $O/tests_pcopy8.log 2>&1 \
  || { tail -30 $O/tests_pcopy8.log; exit 1; }
tail -n 1 $O/tests_pcopy8.log
bash tools/gpu_ab_lib.sh tree novw nosplit now0 rcpsel pcopy8 head 2>&1 | tee $O/ab.txt
