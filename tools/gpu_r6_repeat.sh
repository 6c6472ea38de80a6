# GPU box, round 6: the default C2 line three times (run-to-run spread), no CPU baseline.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${1:-r6rep}
mkdir -p $O
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$k.json 2> $O/bench_$k.err || { tail -20 $O/bench_$k.err; exit 1; }
done
python3 - <<PY
import json
v = []
for k in (1, 2, 3):
    e = json.loads(open("$O/bench_%d.json" % k).read().strip().splitlines()[-1])
    v.append(e["value"])
    print(k, e["value"], e["pose_algebra"], e["frames_ok"], e["resets"], e["roofline"]["avg_launch_ms"], e["other_algebra"]["frames_per_sec"])
print("min/max spread", round((max(v) - min(v)) / min(v) * 100, 2), "%")
PY
