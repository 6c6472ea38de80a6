# GPU box, round 5: the integration's wave lane map (four y rows x eight z layers per wave):
# parity (ICP/scene sequence, colour, the C5E stress), then C3I and C2 A/B against HEAD.
#   gpurun -- bash tools/gpu_r5_l.sh TAG
set -e
cd $GRAFT_REPO_ROOT
TAG=${1:-r5l}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_colour.py tests/test_gpu_hash_stress.py tests/test_gpu_engines.py \
  -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
bash tools/gpu_ab_c3i.sh tree head 2>&1 | tee $O/ab_c3i.txt
