# GPU box, round 6: XCD-banded integration (TFUSION_INTEG_BANDS) -- parity subset, then the C2
# line A/B (bands off / on, twice each), kernel-trace integrate times and FETCH_SIZE per variant.
#   gpurun -- bash tools/gpu_r6_bands.sh TAG [pytest selection...]
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-r6bands}; shift || true
SEL=${@:-tests/test_gpu_parity.py}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v -rs --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ARGS="--no-cpu-baseline --no-other-algebra"
for k in 1 2; do
  for b in 0 1; do
    TFUSION_INTEG_BANDS=$b timeout -k 10 300 python bench.py $ARGS > $O/bench_b${b}_$k.json 2> $O/bench_b${b}_$k.err || { tail -20 $O/bench_b${b}_$k.err; exit 1; }
  done
done
python3 - <<PY
import json
for k in (1, 2):
    for b in (0, 1):
        e = json.loads(open("$O/bench_b%d_%d.json" % (b, k)).read().strip().splitlines()[-1])
        print("bands", b, "run", k, "fps", e["value"], "ok", e["frames_ok"], "resets", e["resets"], "integ", e["stage_ms_per_frame"]["integrate"], "alloc", e["stage_ms_per_frame"]["alloc"])
PY
cd /tmp && export TMPDIR=/tmp
for b in 0 1; do
  TFUSION_INTEG_BANDS=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b$b -o run -- python3 $R/bench.py $ARGS --steps 5 > $O/prof_b$b.log 2>&1 || { tail -20 $O/prof_b$b.log; exit 1; }
  f=$(find $O/prof_b$b -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_summary.py $f > $O/kernel_trace_summary_b$b.txt
  grep -E "k_integrate|k_vis_build|k_icp_frame<4>|k_raycast_pair" $O/kernel_trace_summary_b$b.txt | head -5
  TFUSION_INTEG_BANDS=$b timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_b$b -o run -- python3 $R/bench.py $ARGS --steps 2 --warmup 1 --no-profile > $O/fetch_b$b.log 2>&1 || { tail -20 $O/fetch_b$b.log; exit 1; }
  f=$(find $O/fetch_b$b -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
s = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r.get("Kernel_Name", "")
    if "k_integrate" in n or "k_vis_build" in n:
        s[n[:34]].append(float(r["Counter_Value"]))
for n, v in s.items():
    v = sorted(v)
    print("FETCH_SIZE KiB", n, "n", len(v), "median", v[len(v) // 2], "mean", round(sum(v) / len(v), 1))
PY
done
