# GPU box: the round's bench lines (C2 with the CPU baseline, C3, C3I, C3R, C5, C5 swapping) and
# a rocprofv3 kernel trace + stats of the default bench command.  Outputs under gpurun_out/r3_TAG/.
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-final}
O=$R/gpurun_out/r3_$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-200
for cfg in C3 C3I C3R; do
  timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline > $O/bench_$cfg.log 2>&1 || { tail -20 $O/bench_$cfg.log; exit 1; }
  tail -1 $O/bench_$cfg.log | cut -c1-160
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv > $O/kernel_trace_summary.txt 2>&1 || true
head -12 $O/kernel_trace_summary.txt
