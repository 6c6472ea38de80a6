# GPU box recipe: parity tests, bench, kernel trace.  Usage: gpurun -- bash tools/gpu_all.sh TAG
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-run}
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-profile > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -30 $R/gpurun_out/prof_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/prof_$TAG.log
