set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c3i
for v in old head tree old head tree; do
  if [ $v = tree ]; then L=$PWD/topfusion_amd/libtfusion_hip.so; else L=$PWD/tools/_build/$v/libtfusion_hip.so; fi
  TFUSION_HIP_LIB=$L timeout -k 10 200 python bench.py --config C3I --no-cpu-baseline > gpurun_out/c3i/$v.log 2>&1
  python -c "import json; d=json.loads(open('gpurun_out/c3i/$v.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])"
done
