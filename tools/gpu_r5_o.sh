# GPU box, round 5: the finer levels' maps prefetched into L2 during the coarsest level
# (IP_PREFETCH): ICP parity, the debug timeline, C2 A/B against nopf.   gpurun -- bash tools/gpu_r5_o.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r5o}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rs -k "icp or sequence or bench_timed_window" \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so timeout -k 10 120 python tools/icp_timeline.py > $O/icp_timeline.txt 2>&1 \
  || { tail -20 $O/icp_timeline.txt; exit 1; }
bash tools/gpu_ab_lib.sh tree nopf 2>&1 | tee $O/ab.txt
