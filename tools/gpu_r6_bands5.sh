# GPU box, round 6: XCD bands -- band check, integrate timeline by XCD, parity subset, C2 A/B.
#   gpurun -- bash tools/gpu_r6_bands5.sh TAG [pytest selection...]
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-r6bands5}; shift || true
SEL=${@:-tests/test_gpu_parity.py}
O=$R/gpurun_out/$TAG
mkdir -p $O
TFUSION_INTEG_BANDS=1 TFUSION_HIP_LIB=tools/_build/itl/libtfusion_hip.so timeout -k 10 200 python tools/band_check.py > $O/band_check.txt 2>&1 || { tail -20 $O/band_check.txt; exit 1; }
cat $O/band_check.txt
for b in 0 1; do
  TFUSION_INTEG_BANDS=$b TFUSION_HIP_LIB=tools/_build/itl/libtfusion_hip.so timeout -k 10 200 python tools/integ_timeline.py > $O/itl_b$b.txt 2>&1 || { tail -20 $O/itl_b$b.txt; exit 1; }
  echo "== bands $b"; grep -E "integrate |XCD|band_on|span" $O/itl_b$b.txt
done
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
