# GPU box: the GPU suite, then the default bench line under the per-call variants
# (TFUSION_PERCALL_EARLY / TFUSION_PERCALL_OVERLAP).   gpurun -- bash tools/gpu_percall_ab.sh TAG [pytest selection]
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-pc}; shift || true
SEL=${@:-tests}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 700 python -u -m pytest $SEL -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in "1 1" "1 0" "0 0"; do
  set -- $v
  TFUSION_PERCALL_EARLY=$1 TFUSION_PERCALL_DEFER=$2 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$1$2.log 2>&1 || { tail -20 $O/bench_$1$2.log; exit 1; }
  python -c "
import json
e=json.loads(open('$O/bench_$1$2.log').read().strip().splitlines()[-1])
print('early $1 defer $2: C2 fps', e['value'], 'per-call', e['per_call_frames_per_sec'], 'batched same', e.get('per_call_batched_same_frames'))"
done
