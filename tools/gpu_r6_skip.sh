# GPU box, round 6: integration skipping blockless pairs (TF_INTEG_SKIP_EMPTY) -- parity subset,
# C2 A/B against the previous build (tools/_build/noskip), kernel traces.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${1:-r6skip}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_colour.py tests/test_gpu_engines.py -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ARGS="--no-cpu-baseline --no-other-algebra"
for k in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > $O/bench_new_$k.json 2> $O/bench_new_$k.err || { tail -20 $O/bench_new_$k.err; exit 1; }
  TFUSION_HIP_LIB=tools/_build/noskip/libtfusion_hip.so timeout -k 10 300 python bench.py $ARGS > $O/bench_old_$k.json 2> $O/bench_old_$k.err || { tail -20 $O/bench_old_$k.err; exit 1; }
done
python3 - <<PY
import json
for k in (1, 2):
    for b in ("old", "new"):
        e = json.loads(open("$O/bench_%s_%d.json" % (b, k)).read().strip().splitlines()[-1])
        print(b, "run", k, "fps", e["value"], "ok", e["frames_ok"], "resets", e["resets"], "integ", e["stage_ms_per_frame"]["integrate"])
PY
cd /tmp && export TMPDIR=/tmp
for b in new old; do
  L=""; [ $b = old ] && L=$R/tools/_build/noskip/libtfusion_hip.so
  TFUSION_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$b -o run -- python3 $R/bench.py $ARGS --steps 5 > $O/prof_$b.json 2> $O/prof_$b.err || { tail -20 $O/prof_$b.err; exit 1; }
  f=$(find $O/prof_$b -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_summary.py $f > $O/kernel_trace_summary_$b.txt
  echo "== $b"; grep -E "k_integrate" $O/kernel_trace_summary_$b.txt | head -1 | cut -c1-170
done
