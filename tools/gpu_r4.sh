# GPU box, round 4: the hash-stress tests first, then the whole GPU suite, then the C5E lines
# (swapping off / on) and the default C2 line.  Outputs under gpurun_out/TAG/.
#   gpurun -- bash tools/gpu_r4.sh TAG
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-r4}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_hash_stress.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_hash.log 2>&1 || { tail -40 $O/tests_hash.log; exit 1; }
tail -3 $O/tests_hash.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_hash_stress.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --config C5E > $O/bench_C5E.log 2>&1 || { tail -20 $O/bench_C5E.log; exit 1; }
tail -1 $O/bench_C5E.log | cut -c1-400
timeout -k 10 300 python bench.py --config C5E --swapping > $O/bench_C5E_swapping.log 2>&1 || { tail -20 $O/bench_C5E_swapping.log; exit 1; }
tail -1 $O/bench_C5E_swapping.log | cut -c1-400
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-200
