# GPU box, round 6: the rocprofv3 kernel trace + stats of the default bench command only.
#   gpurun -- bash tools/gpu_r6_prof.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r6p}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || { tail -30 $O/prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py $f > $O/kernel_trace_summary.txt
head -12 $O/kernel_trace_summary.txt
