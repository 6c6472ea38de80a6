# GPU box, round 5 closing check on the final tree: smoke() and the parity tests of the frame path
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5af
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5af/smoke.log 2>&1 || { tail -20 gpurun_out/r5af/smoke.log; exit 1; }
tail -1 gpurun_out/r5af/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/r5af/tests.log 2>&1 || { tail -30 gpurun_out/r5af/tests.log; exit 1; }
tail -1 gpurun_out/r5af/tests.log
