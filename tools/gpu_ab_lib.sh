# GPU box A/B of library variants on C2 (driver shape, every 16th frame's stages timed by their
# dispatches): tools/_build/<v>/libtfusion_hip.so or the tree's own ("tree"), alternated twice.
#   gpurun -- bash tools/gpu_ab_lib.sh tree v1 ...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for round in 1 2; do
  for v in "$@"; do
    if [ $v = tree ]; then L=$PWD/topfusion_amd/libtfusion_hip.so; else L=$PWD/tools/_build/$v/libtfusion_hip.so; fi
    TFUSION_HIP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --per-call-frames 0 > gpurun_out/ab/lib_$v.log 2>&1 \
      || { tail -20 gpurun_out/ab/lib_$v.log; exit 1; }
    python -c "
import json
e=json.loads(open('gpurun_out/ab/lib_$v.log').read().strip().splitlines()[-1])
print('$v', 'C2 fps', e['value'], {k: v for k, v in e['stage_ms_per_frame'].items() if v})"
  done
done
