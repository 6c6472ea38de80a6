# GPU box, round 5: the persistent-ICP ordering event without a system-scope fence (tree) against
# the old event (sysfence): the multi-context parity tests, then the batched C2 rate of a context
# alone and beside a second context (tools/two_ctx_rate.py).
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rs -k "contexts" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for v in tree sysfence; do
  if [ $v = tree ]; then L=$PWD/topfusion_amd/libtfusion_hip.so; else L=$PWD/tools/_build/$v/libtfusion_hip.so; fi
  TFUSION_HIP_LIB=$L timeout -k 10 300 python tools/two_ctx_rate.py > $O/rate_$v.txt 2>&1 || { tail -20 $O/rate_$v.txt; exit 1; }
  echo "$v $(tail -1 $O/rate_$v.txt)"
done
