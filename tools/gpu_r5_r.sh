# GPU box, round 5: ray march with the corner fetch on near-surface steps (TF_RAY_SPEC) -- parity and
# C2 A/B; the ICP kernel capped at 168 VGPRs (waves_per_eu 3) in the same A/B.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5r
mkdir -p $O
TFUSION_HIP_LIB=$PWD/tools/_build/spec8/libtfusion_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rs \
  -k "raycast or sequence or render or c3 or batched or bench_shape or timed_window or excess" --timeout 300 --timeout-method thread > $O/tests_spec8.log 2>&1 || { tail -30 $O/tests_spec8.log; exit 1; }
tail -n 1 $O/tests_spec8.log
TFUSION_HIP_LIB=$PWD/tools/_build/wpe3/libtfusion_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rs \
  -k "icp_stage or timed_window" --timeout 300 --timeout-method thread > $O/tests_wpe3.log 2>&1 || { tail -30 $O/tests_wpe3.log; exit 1; }
tail -n 1 $O/tests_wpe3.log
bash tools/gpu_ab_lib.sh tree spec8 spec8L spec8t1 spec8t02 wpe3 2>&1 | tee $O/ab.txt
