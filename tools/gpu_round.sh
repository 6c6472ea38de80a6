# GPU box recipe for a round's committed evidence: parity tests, the default bench line (with
# the CPU baseline), a rocprofv3 kernel-trace/stats run of the same bench, and the PMC passes.
#   gpurun -- bash tools/gpu_round.sh TAG      (outputs under gpurun_out/round_TAG/)
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
O=$R/gpurun_out/round_$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
tail -1 $O/prof.log
cd $R
bash tools/gpu_pmc.sh $TAG
for cfg in C3 C3I C3R; do
  timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline > $O/bench_$cfg.log 2>&1 || { tail -30 $O/bench_$cfg.log; exit 1; }
  tail -1 $O/bench_$cfg.log | cut -c1-160
done
