# GPU box: kernel traces of the default bench with the tree's library and with a diagnostic build that
# puts an empty launch between the ICP and the allocation (tools/_build/nop, -DTF_DIAG_NOP_AFTER_ICP),
# each summarised by tools/trace_gaps.py.  Outputs: gpurun_out/TAG/.
#   gpurun -- bash tools/gpu_gap_diag.sh TAG
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-gap}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in tree nop; do
  if [ $v = tree ]; then L=$R/topfusion_amd/libtfusion_hip.so; else L=$R/tools/_build/$v/libtfusion_hip.so; fi
  TFUSION_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$v -o run -- \
    python3 $R/bench.py --no-cpu-baseline --per-call-frames 0 > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  echo "== $v"
  python3 $R/tools/trace_gaps.py $O/prof_$v/run_kernel_trace.csv | tee $O/gaps_$v.txt
done
