# GPU box: round-3 step b -- full GPU suite, then the lite ray march A/B (tree vs lite0) on C2,
# then the per-call path with and without the published-mirror completion.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r3b
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r3b/tests.log 2>&1 || { tail -30 gpurun_out/r3b/tests.log; exit 1; }
tail -1 gpurun_out/r3b/tests.log
timeout -k 10 400 bash tools/gpu_ab_lib.sh tree lite0 > gpurun_out/r3b/ab.log 2>&1 || { tail -20 gpurun_out/r3b/ab.log; exit 1; }
cat gpurun_out/r3b/ab.log
for pubv in 1 0; do
  TFUSION_PUBLISH=$pubv PERCALL_SKIP=160 PERCALL_FRAMES=256 timeout -k 10 200 python tools/percall.py > gpurun_out/r3b/percall_$pubv.log 2>&1 || { tail -20 gpurun_out/r3b/percall_$pubv.log; exit 1; }
  echo "publish=$pubv $(tail -1 gpurun_out/r3b/percall_$pubv.log)"
done
