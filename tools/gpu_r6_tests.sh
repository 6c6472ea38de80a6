# GPU box, round 6: the whole GPU suite (verbose log under gpurun_out/TAG/).
#   gpurun -- bash tools/gpu_r6_tests.sh TAG [pytest selection...]
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r6t}; shift || true
SEL=${@:-tests}
mkdir -p gpurun_out/$TAG
timeout -k 10 1080 python -u -m pytest $SEL -m gpu -x -v -rs --timeout 400 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { tail -60 gpurun_out/$TAG/tests.log; exit 1; }
tail -3 gpurun_out/$TAG/tests.log
