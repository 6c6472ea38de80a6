# GPU box: round-3 diagnostics -- ray-march step statistics (TF_RAY_STATS build) and a kernel +
# memory-copy trace of the per-call path (tools/percall.py) on the C2 timed frames.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/diag
TFUSION_HIP_LIB=$R/tools/_build/raystats/libtfusion_hip.so timeout -k 10 300 python tools/ray_stats.py 24 > gpurun_out/diag/ray_stats.log 2>&1
tail -2 gpurun_out/diag/ray_stats.log
cd /tmp && export TMPDIR=/tmp
PERCALL_SKIP=160 PERCALL_FRAMES=128 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/diag/pc -o run -- python3 $R/tools/percall.py > $R/gpurun_out/diag/percall.log 2>&1
tail -1 $R/gpurun_out/diag/percall.log
