# GPU box, round 6: merged longest-first tile order -- tile-order + parity tests, pair timelines,
# C2 A/B against the previous order (tools/_build/oldorder), kernel traces.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${1:-r6ord}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tile_order.py tests/test_gpu_parity.py -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
TFUSION_HIP_LIB=tools/_build/ptl/libtfusion_hip.so timeout -k 10 200 python tools/pair_timeline.py > $O/pair_timeline.txt 2>&1 || { tail -20 $O/pair_timeline.txt; exit 1; }
PTL_BATCH=1 TFUSION_HIP_LIB=tools/_build/ptl_la/libtfusion_hip.so timeout -k 10 200 python tools/pair_timeline.py > $O/pair_timeline_batch.txt 2>&1 || { tail -20 $O/pair_timeline_batch.txt; exit 1; }
head -12 $O/pair_timeline.txt | cut -c1-200; echo ==; head -12 $O/pair_timeline_batch.txt | cut -c1-200
ARGS="--no-cpu-baseline --no-other-algebra"
for k in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > $O/bench_new_$k.json 2> $O/bench_new_$k.err || { tail -20 $O/bench_new_$k.err; exit 1; }
  TFUSION_HIP_LIB=tools/_build/oldorder/libtfusion_hip.so timeout -k 10 300 python bench.py $ARGS > $O/bench_old_$k.json 2> $O/bench_old_$k.err || { tail -20 $O/bench_old_$k.err; exit 1; }
done
python3 - <<PY
import json
for k in (1, 2):
    for b in ("old", "new"):
        e = json.loads(open("$O/bench_%s_%d.json" % (b, k)).read().strip().splitlines()[-1])
        print(b, "run", k, "fps", e["value"], "ok", e["frames_ok"], "resets", e["resets"], "raycast_icp", e["stage_ms_per_frame"]["raycast_icp"])
PY
cd /tmp && export TMPDIR=/tmp
for b in new old; do
  L=""; [ $b = old ] && L=$R/tools/_build/oldorder/libtfusion_hip.so
  TFUSION_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$b -o run -- python3 $R/bench.py $ARGS --steps 5 > $O/prof_$b.json 2> $O/prof_$b.err || { tail -20 $O/prof_$b.err; exit 1; }
  f=$(find $O/prof_$b -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_summary.py $f > $O/kernel_trace_summary_$b.txt
  echo "== $b"; grep -E "k_raycast_pair|k_icp_maps_end" $O/kernel_trace_summary_$b.txt | head -3 | cut -c1-170
done
