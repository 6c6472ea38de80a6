# GPU box, round 5: the OpenCV pose-algebra parity tests, then the default C2 line and the same
# line under the reference's OpenCV algebra (ICP cost of the SVD solve).  Outputs: gpurun_out/TAG/.
#   gpurun -- bash tools/gpu_r5_pose.sh TAG [pytest selection...]
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-pose}; shift || true
SEL=${@:-tests/test_gpu_pose_algebra.py}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 700 python -u -m pytest $SEL -m gpu -x -v -rs --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_canonical.json 2> $O/bench_canonical.err || { tail -20 $O/bench_canonical.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --pose-algebra opencv4 > $O/bench_opencv4.json 2> $O/bench_opencv4.err || { tail -20 $O/bench_opencv4.err; exit 1; }
python - <<PY
import json
for n in ("canonical", "opencv4"):
    e = json.loads(open("$O/bench_" + n + ".json").read().strip().splitlines()[-1])
    print(n, e["pose_algebra"], "fps", e["value"], "ok", e["frames_ok"], "resets", e["resets"], {k: v for k, v in e["stage_ms_per_frame"].items() if v})
PY
