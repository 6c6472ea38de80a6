# GPU box: parity tests, then the default bench line and the C3 scale lines.  Outputs under
# gpurun_out/check_TAG/.   gpurun -- bash tools/gpu_check.sh TAG [pytest -k expression]
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-chk}
K=${2:-}
O=$R/gpurun_out/check_$TAG
mkdir -p $O
cd $R
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
fi
tail -3 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.log 2>&1 || { tail -30 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log
timeout -k 10 300 python bench.py --config C3I > $O/bench_c3i.log 2>&1 || { tail -30 $O/bench_c3i.log; exit 1; }
tail -1 $O/bench_c3i.log
timeout -k 10 300 python bench.py --config C3R > $O/bench_c3r.log 2>&1 || { tail -30 $O/bench_c3r.log; exit 1; }
tail -1 $O/bench_c3r.log
