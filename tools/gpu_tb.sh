set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log
