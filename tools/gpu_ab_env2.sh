# GPU box: selected GPU tests, then the default bench line under each value of one env switch.
#   gpurun -- bash tools/gpu_ab_env2.sh TAG VAR "v1 v2 ..." [pytest -k expression]
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=$1; VAR=$2; VALS=$3; K=${4:-}
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  python -c "
import json
e=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1])
print('$VAR=$v: C2 fps', e['value'], 'per-call', e['per_call_frames_per_sec'], {k: v for k, v in e['stage_ms_per_frame'].items() if v})"
done
