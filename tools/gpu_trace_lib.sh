# GPU box: rocprofv3 kernel trace of a short C2 bench run with a variant library
# (tools/_build/<v>/libtfusion_hip.so, or "tree"), summarised with the inter-kernel gaps.
#   gpurun -- bash tools/gpu_trace_lib.sh v
set -e
R=$GRAFT_REPO_ROOT
v=$1
if [ $v = tree ]; then L=$R/topfusion_amd/libtfusion_hip.so; else L=$R/tools/_build/$v/libtfusion_hip.so; fi
cd /tmp && export TMPDIR=/tmp
TFUSION_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tracelib_$v -o run -- \
  python3 $R/bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-profile --per-call-frames 0 > $R/gpurun_out/tracelib_$v.log 2>&1 \
  || { tail -20 $R/gpurun_out/tracelib_$v.log; exit 1; }
cd $R && python tools/trace_summary.py gpurun_out/tracelib_$v/run_kernel_trace.csv | grep -E "^k_|^void k_|->" | head -24
