# GPU box, round 6: full GPU suite, then smoke + the default bench line + rocprofv3 kernel trace.
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-r6fin}
bash tools/gpu_r6_tests.sh ${TAG}_t
bash tools/gpu_r6_bench.sh ${TAG}_b
