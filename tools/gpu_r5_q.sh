# GPU box, round 5: staged per-iteration prefetch of the finer ICP levels' maps by wave 4
# (IP_PREFETCH2): ICP parity, the level set-up timeline, C2 A/B against nopf2.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_failures.py -m gpu -x -q -rs -k "icp or sequence or bench_timed_window or peer" \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so timeout -k 10 120 python tools/icp_timeline.py > $O/icp_timeline.txt 2>&1 \
  || { tail -20 $O/icp_timeline.txt; exit 1; }
grep "level set-up" $O/icp_timeline.txt | cut -c1-330
bash tools/gpu_ab_lib.sh tree nopf2 2>&1 | tee $O/ab.txt
