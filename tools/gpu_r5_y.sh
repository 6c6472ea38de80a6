# GPU box, round 5: ICP tail micro-benchmark (tools/micro/icp_tail) with the S' solve candidate
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5y
timeout -k 10 120 tools/micro/icp_tail > gpurun_out/r5y/icp_tail_micro.txt 2>&1 || { tail gpurun_out/r5y/icp_tail_micro.txt; exit 1; }
cat gpurun_out/r5y/icp_tail_micro.txt
