# GPU box, round 6: ICP hand-off poll interval A/B (IP_SLEEP 1 = product, 0, 2), C2 default line, alternated.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${1:-r6sleep}
mkdir -p $O
ARGS="--no-cpu-baseline --no-other-algebra"
for k in 1 2; do
  for v in prod sleep0 sleep2; do
    L=""; [ $v != prod ] && L=tools/_build/$v/libtfusion_hip.so
    TFUSION_HIP_LIB=$L timeout -k 10 300 python bench.py $ARGS > $O/bench_${v}_$k.json 2> $O/bench_${v}_$k.err || { tail -20 $O/bench_${v}_$k.err; exit 1; }
    python3 -c "
import json; e=json.loads(open('$O/bench_${v}_$k.json').read().strip().splitlines()[-1]); print('$v', $k, e['value'], e['roofline']['avg_launch_ms'], e['frames_ok'], e['resets'])"
  done
done
