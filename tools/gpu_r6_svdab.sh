# GPU box, round 6: A/B of lane-SVD variants (each binary: bits vs serial + oracle, latency).
#   gpurun -- bash tools/gpu_r6_svdab.sh TAG bin1 bin2 ...
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6ab}; shift
mkdir -p $O
for b in "$@"; do
  timeout -k 10 200 ./tools/micro/$b tests/golden/icp_systems_C2_opencv4.f32 > $O/$b.txt 2>&1
  echo "== $b"; grep -E "differ|lanes  " $O/$b.txt
done
