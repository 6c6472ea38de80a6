# GPU box, round 5: micro-benchmarks, the whole GPU suite (no -x: every failure listed), the
# default C2 line, the C5E four/seven-launch A/B.  Outputs: gpurun_out/TAG/.
#   gpurun -- bash tools/gpu_r5_c.sh TAG
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-r5c}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 60 ./tools/micro/icp_tail > $O/icp_tail.txt 2>&1 || { cat $O/icp_tail.txt; exit 1; }
cat $O/icp_tail.txt
st=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || st=$?
tail -12 $O/tests.log
[ $st -eq 0 ] || [ $st -eq 1 ] || exit $st
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json
e=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('C2 fps', e['value'], 'resets', e['resets'], 'per-call', e['per_call_frames_per_sec'], {k: v for k, v in e['stage_ms_per_frame'].items() if v})"
for v in 1 0; do
  TFUSION_FUSE_TAIL=$v timeout -k 10 300 python bench.py --config C5E --steps 20 > $O/c5e_$v.json 2> $O/c5e_$v.err || { tail -20 $O/c5e_$v.err; exit 1; }
  python -c "import json; e=json.loads(open('$O/c5e_$v.json').read().strip().splitlines()[-1]); print('C5E fuse_tail=$v', e['value'], 'sat', e['saturated_frames_per_sec'], 'first_fail', e['first_failure_frame'])"
done
