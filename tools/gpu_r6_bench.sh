# GPU box, round 6: smoke, the driver's default bench line (CPU baseline included), and the
# rocprofv3 kernel trace + stats of the default bench command (no CPU baseline: same GPU work).
#   gpurun -- bash tools/gpu_r6_bench.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r6b}
mkdir -p $O
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python - <<PY
import json
e = json.loads(open("$O/bench.json").read().strip().splitlines()[-1])
print("value", e["value"], e["pose_algebra"], "ok", e["frames_ok"], "resets", e["resets"], "roof", e["roofline"]["kernel"], e["roofline"]["frac"])
print("other", e["other_algebra"])
print({k: v for k, v in e["stage_ms_per_frame"].items() if v})
print("cpu", e["cpu_baseline"]["value"], e["cpu_baseline"]["cores"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || { tail -30 $O/prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py $f > $O/kernel_trace_summary.txt
head -12 $O/kernel_trace_summary.txt
