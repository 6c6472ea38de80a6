# GPU box: rocprofv3 kernel trace of a short bench run (no HIP-event profiling), for per-kernel
# times of the current default schedule.  Usage: gpurun -- bash tools/gpu_trace.sh TAG [C2|C3]
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-trace}
CFG=${2:-C2}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_$TAG -o run -- \
  python $R/bench.py --config $CFG --steps 100 --warmup 10 --no-cpu-baseline --no-profile > $R/gpurun_out/trace_$TAG.log 2>&1 \
  || { tail -20 $R/gpurun_out/trace_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/trace_$TAG.log | cut -c1-200
cd $R && python tools/trace_summary.py gpurun_out/trace_$TAG/run_kernel_trace.csv
