# GPU box recipe: rocprofv3 kernel trace + stats of the default bench command (the line the
# driver records), for the per-kernel durations the bench's roofline objects must agree with.
# Usage: gpurun -- bash tools/gpu_prof.sh TAG [bench args...]
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-prof}
shift || true
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/bench.py "$@" > $O/bench.log 2>&1 \
  || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
python3 $R/tools/trace_summary.py "$(find $O -name '*kernel_trace.csv' | head -1)" > $O/summary.txt 2>&1 || true
head -40 $O/summary.txt
