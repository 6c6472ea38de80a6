# GPU box A/B of library variants on C3R (and the driver-shape C2 line): tools/_build/<v>/libtfusion_hip.so
# or the tree's own library, alternated, through TFUSION_HIP_LIB.   gpurun -- bash tools/gpu_ab_c3r.sh v1 v2 ...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for round in 1 2; do
  for v in "$@"; do
    if [ $v = tree ]; then L=$PWD/topfusion_amd/libtfusion_hip.so; else L=$PWD/tools/_build/$v/libtfusion_hip.so; fi
    TFUSION_HIP_LIB=$L timeout -k 10 200 python bench.py --config C3R > gpurun_out/ab/c3r_$v.log 2>&1
    TFUSION_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --per-call-frames 0 > gpurun_out/ab/c2_$v.log 2>&1
    python -c "
import json
d=json.loads(open('gpurun_out/ab/c3r_$v.log').read().strip().splitlines()[-1]); e=json.loads(open('gpurun_out/ab/c2_$v.log').read().strip().splitlines()[-1])
print('$v', 'C3R ms', d['ms_per_step'], 'C2 fps', e['value'], 'stages', {k: v for k, v in e.get('stage_ms_per_frame', {}).items() if v})"
  done
done
