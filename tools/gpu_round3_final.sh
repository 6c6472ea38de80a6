# GPU box: the round-3 evidence at HEAD -- bench lines (C2 with the CPU baseline, C3, C3I, C3R,
# C5, C5 with swapping), a rocprofv3 kernel trace + stats of the default bench command, and the
# C2 PMC traffic per frame type.  Outputs under gpurun_out/r3f_TAG/ (and gpurun_out/pmcf_TAG/).
#   gpurun -- bash tools/gpu_round3_final.sh TAG
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-final}
O=$R/gpurun_out/r3f_$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log | cut -c1-160
for cfg in C3 C3I C3R C5; do
  timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline > $O/bench_$cfg.log 2>&1 || { tail -20 $O/bench_$cfg.log; exit 1; }
  tail -1 $O/bench_$cfg.log | cut -c1-160
done
timeout -k 10 400 python bench.py --config C5 --swapping --no-cpu-baseline > $O/bench_C5_swapping.log 2>&1 || { tail -20 $O/bench_C5_swapping.log; exit 1; }
tail -1 $O/bench_C5_swapping.log | cut -c1-160
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv > $O/kernel_trace_summary.txt 2>&1 || true
head -10 $O/kernel_trace_summary.txt | cut -c1-160
timeout -k 10 700 bash tools/gpu_pmc_frames.sh $TAG > $O/pmc_frames.log 2>&1 || { tail -20 $O/pmc_frames.log; exit 1; }
tail -5 $O/pmc_frames.log
