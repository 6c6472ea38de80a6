# GPU box: the GPU suite, then an A/B of environment switches on C2 (tools/gpu_ab_env.sh) and the
# pair kernel's workgroup timeline (tools/pair_timeline.py, TF_PAIR_TIMELINE build in tools/_build/ptl).
#   gpurun -- bash tools/gpu_suite_env_ab.sh TAG base NAME=VALUE ...
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-sab}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab_env.sh "$@" 2>&1 | tee $O/ab.txt
if [ -f tools/_build/ptl/libtfusion_hip.so ]; then
  TFUSION_HIP_LIB=tools/_build/ptl/libtfusion_hip.so timeout -k 10 200 python tools/pair_timeline.py > $O/pair_timeline.txt 2>&1 \
    || { tail -20 $O/pair_timeline.txt; exit 1; }
  grep -v resident $O/pair_timeline.txt | head -14
fi
