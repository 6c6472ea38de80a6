# GPU box, round 5 final (part 1): smoke(), the whole GPU suite (verbose log), the default bench
# line (with the CPU baseline and the roofline).  Outputs: gpurun_out/TAG/.
#   gpurun -- bash tools/gpu_r5_final.sh TAG
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-fin}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 500 python bench.py > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-300
