# GPU box: the GPU suite, then the default bench line (no CPU baseline) -- the check after a change.
#   gpurun -- bash tools/gpu_tests_bench.sh TAG [pytest selection...]
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-t}; shift || true
SEL=${@:-tests}
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest $SEL -m gpu -x -q -rs --timeout 400 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1 || { tail -40 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/bench.log 2>&1 || { tail -20 gpurun_out/$TAG/bench.log; exit 1; }
python -c "
import json
e=json.loads(open('gpurun_out/$TAG/bench.log').read().strip().splitlines()[-1])
print('C2 fps', e['value'], 'per-call', e['per_call_frames_per_sec'], {k: v for k, v in e['stage_ms_per_frame'].items() if v})"
