# GPU box, round 5: CreateICPMaps in the pair launch's tail (tree default) -- the whole GPU suite,
# then C2 A/B against TFUSION_MAPS_IN_PAIR=0 (the maps in k_icp_maps_end).
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ad
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
bash tools/gpu_ab_env.sh base TFUSION_MAPS_IN_PAIR=0 2>&1 | tee $O/ab.txt
bash tools/gpu_ab_env.sh base TFUSION_MAPS_IN_PAIR=0 2>&1 | tee -a $O/ab.txt
