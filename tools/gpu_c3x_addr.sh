# GPU box, round 5: what in C3I's depth samples costs time -- addresses or cache lines.  C3I pass
# time per diagnostic build (tools/_build: c3x1 all samples one pixel, c3x4 samples rounded to
# 16 B, c3x8 to 128 B lines) against the tree, alternated twice.   gpurun -- bash tools/gpu_c3x_addr.sh
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c3xa
for round in 1 2; do
  for v in tree c3x1 c3x4 c3x8; do
    if [ $v = tree ]; then L=$PWD/topfusion_amd/libtfusion_hip.so; else L=$PWD/tools/_build/$v/libtfusion_hip.so; fi
    TFUSION_HIP_LIB=$L timeout -k 10 200 python bench.py --config C3I > gpurun_out/c3xa/c3i_$v.log 2>&1 || { tail -20 gpurun_out/c3xa/c3i_$v.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/c3xa/c3i_$v.log').read().strip().splitlines()[-1]); print('$v C3I ms', d['ms_per_step'])"
  done
done
