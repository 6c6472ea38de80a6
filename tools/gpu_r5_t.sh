# GPU box, round 5: the SDF mirror (raycast steps in one round trip) -- the whole GPU suite on the
# tree library (mirror on), then C2 A/B: mirror on / off (TFUSION_SDF_MIRROR=0) / mirror + gradient.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5t
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
bash tools/gpu_ab_env.sh base TFUSION_SDF_MIRROR=0 2>&1 | tee $O/ab_env.txt
bash tools/gpu_ab_lib.sh nrm 2>&1 | tee $O/ab_nrm.txt
