# A/B of env-selected schedules on one box: bench (no CPU baseline) once per setting.
#   gpurun -- bash tools/gpu_ab.sh "VAR=a" "VAR=b" ...
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/ab
i=0
for setting in "$@"; do
  i=$((i+1))
  env $setting timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/ab/$i.log 2>&1 || { tail -20 gpurun_out/ab/$i.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$i.log').read().strip().splitlines()[-1]); print('$setting', d['value'], d['stage_ms_per_frame'])"
done
