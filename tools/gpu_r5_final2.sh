# GPU box, round 5 final (part 2): a rocprofv3 kernel trace + stats of the default bench command,
# its per-kernel summary, the PMC traffic passes of C2 and C3I, and the secondary bench lines.
#   gpurun -- bash tools/gpu_r5_final2.sh TAG
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-fin2}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R
TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so timeout -k 10 120 python tools/icp_timeline.py > $O/icp_timeline.txt 2>&1 \
  || { tail -20 $O/icp_timeline.txt; exit 1; }
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv > $O/kernel_trace_summary.txt 2>&1 || true
head -8 $O/kernel_trace_summary.txt | cut -c1-160
timeout -k 10 300 bash tools/gpu_pmc.sh ${TAG}_c2 C2 > $O/pmc_c2.log 2>&1 || { tail -20 $O/pmc_c2.log; exit 1; }
timeout -k 10 300 bash tools/gpu_pmc.sh ${TAG}_c3i C3I > $O/pmc_c3i.log 2>&1 || { tail -20 $O/pmc_c3i.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc_${TAG}_c2 C2 $O/pmc_traffic.json > /dev/null
python3 tools/pmc_traffic.py gpurun_out/pmc_${TAG}_c3i C3I $O/pmc_traffic.json > /dev/null
for cfg in "--config C3I" "--config C5E" "--colour"; do
  name=$(echo "$cfg" | tr -d ' -')
  timeout -k 10 400 python bench.py $cfg --no-cpu-baseline > $O/bench_$name.log 2>&1 || { tail -20 $O/bench_$name.log; exit 1; }
  tail -1 $O/bench_$name.log | cut -c1-200
done
