# GPU box, round 6: the secondary bench lines at the current code (no CPU baseline): C2 colour,
# C3, C3I, C3R, C5 (50 k frames), C5E, C5E swapping.  Outputs: gpurun_out/TAG/bench_*.json.
#   gpurun -- bash tools/gpu_r6_lines.sh TAG
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6l}
mkdir -p $O
for cfg in "--colour" "--config C3" "--config C3I" "--config C3R" "--config C5" "--config C5E" "--config C5E --swapping"; do
  name=$(echo "$cfg" | tr -d ' -')
  timeout -k 10 300 python bench.py $cfg --no-cpu-baseline > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  python3 -c "
import json,sys
e=json.loads(open('$O/bench_$name.json').read().strip().splitlines()[-1])
print('$name', e['value'], e['unit'], e.get('pose_algebra'), (e.get('roofline') or {}).get('kernel'), (e.get('roofline') or {}).get('frac'))"
done
