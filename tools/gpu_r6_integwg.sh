# GPU box, round 6: frame-path integration grid A/B (TFUSION_INTEG_WG_FRAME), C2 default line, alternated.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${1:-r6iwg}
mkdir -p $O
ARGS="--no-cpu-baseline --no-other-algebra"
for k in 1 2; do
  for w in 768 512 640 1024; do
    TFUSION_INTEG_WG_FRAME=$w timeout -k 10 300 python bench.py $ARGS > $O/bench_${w}_$k.json 2> $O/bench_${w}_$k.err || { tail -20 $O/bench_${w}_$k.err; exit 1; }
    python3 -c "
import json; e=json.loads(open('$O/bench_${w}_$k.json').read().strip().splitlines()[-1]); print('$w', $k, e['value'], e['stage_ms_per_frame']['integrate'], e['frames_ok'], e['resets'])"
  done
done
