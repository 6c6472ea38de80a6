# GPU box: kernel trace of the per-call path (tools/percall.py) on the C2 timed frames, summarised.
#   gpurun -- bash tools/gpu_percall_trace.sh TAG
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-pc}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
PERCALL_SKIP=160 PERCALL_FRAMES=128 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$TAG/tr -o run -- python3 $R/tools/percall.py > $R/gpurun_out/$TAG/percall.log 2>&1
tail -1 $R/gpurun_out/$TAG/percall.log
f=$(find $R/gpurun_out/$TAG/tr -name '*kernel_trace.csv' | head -1)
python3 $R/tools/trace_summary.py $f > $R/gpurun_out/$TAG/summary.txt
grep -E "k_dists|k_pyr|k_icp_frame|raycast_pair|alloc|k_vis|integrate|icp_maps" $R/gpurun_out/$TAG/summary.txt | cut -c1-150
rm -rf $R/gpurun_out/$TAG/tr
