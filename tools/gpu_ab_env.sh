# GPU box A/B of environment switches on C2 (driver shape): each "NAME=VALUE" (or "base") alternated twice.
#   gpurun -- bash tools/gpu_ab_env.sh base TFUSION_INTEG_WG_FRAME=1024 ...
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --per-call-frames 0 > gpurun_out/ab/env.log 2>&1 \
      || { tail -20 gpurun_out/ab/env.log; exit 1; }
    python -c "
import json
e=json.loads(open('gpurun_out/ab/env.log').read().strip().splitlines()[-1])
print('$v', 'C2 fps', e['value'], {k: v for k, v in e['stage_ms_per_frame'].items() if v})"
  done
done
