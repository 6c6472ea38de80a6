# GPU box, round 5: the SDF mirror in bricks of 8^3 blocks (variant sdfm8) against the tree library
# (no mirror) and against itself with the mirror off (TFUSION_SDF_MIRROR=0): raycast parity, C2 A/B.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5u
mkdir -p $O
L=$PWD/tools/_build/sdfm8a/libtfusion_hip.so
TFUSION_HIP_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rs -k "raycast or sequence or render" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
bash tools/gpu_ab_lib.sh tree sdfm8a 2>&1 | tee $O/ab_lib.txt
