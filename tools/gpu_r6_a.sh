# GPU box, round 6: the lane-parallel cv::solve(DECOMP_SVD) -- micro (bits vs serial + oracle,
# latency), the OpenCV pose-algebra parity tests, the C2 line under canonical and opencv4.
#   gpurun -- bash tools/gpu_r6_a.sh TAG [pytest selection...]
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-r6a}; shift || true
SEL=${@:-tests/test_gpu_pose_algebra.py}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 200 ./tools/micro/svd_lanes tests/golden/icp_systems_C2_opencv4.f32 > $O/svd_lanes.txt 2>&1
timeout -k 10 200 ./tools/micro/svd_lanes_stats tests/golden/icp_systems_C2_opencv4.f32 > $O/svd_lanes_stats.txt 2>&1
cat $O/svd_lanes.txt
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
