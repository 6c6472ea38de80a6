# GPU box, round 4: failure / fallback tests, the whole GPU suite (incl. the 800-frame timed window),
# the default bench line and a rocprofv3 kernel trace of it.  Outputs under gpurun_out/TAG/.
#   gpurun -- bash tools/gpu_r4c.sh TAG
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-r4c}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_failures.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_fail.log 2>&1 || { tail -40 $O/tests_fail.log; exit 1; }
tail -3 $O/tests_fail.log
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_failures.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-300
