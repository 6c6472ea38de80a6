# GPU box: the GPU suite, the ICP timeline (debug build) and an A/B of library variants on C2
# (tools/_build/<v>/libtfusion_hip.so vs the tree's, alternated twice).  Outputs: gpurun_out/TAG/.
#   gpurun -- bash tools/gpu_r4d.sh TAG v1 v2 ...
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-r4d}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so timeout -k 10 120 python tools/icp_timeline.py > $O/icp_timeline.txt 2>&1 \
  || { tail -20 $O/icp_timeline.txt; exit 1; }
tail -3 $O/icp_timeline.txt | cut -c1-250
for round in 1 2; do
  for v in tree "$@"; do
    if [ $v = tree ]; then L=$PWD/topfusion_amd/libtfusion_hip.so; else L=$PWD/tools/_build/$v/libtfusion_hip.so; fi
    TFUSION_HIP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --per-call-frames 0 > $O/ab_${v}_$round.log 2>&1 \
      || { tail -20 $O/ab_${v}_$round.log; exit 1; }
    python -c "
import json
e=json.loads(open('$O/ab_${v}_$round.log').read().strip().splitlines()[-1])
print('$v', 'C2 fps', e['value'], {k: v for k, v in e['stage_ms_per_frame'].items() if v})"
  done
done
