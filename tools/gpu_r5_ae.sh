# GPU box, round 5: CreateICPMaps in the pair launch's tail, maps blocks polling every 2 / 16 / 63
# x 64 cycles (tree / ms16 / ms63), against the maps in k_icp_maps_end (tree, TFUSION_MAPS_IN_PAIR=0)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5ae
TFUSION_MAPS_IN_PAIR=0 bash tools/gpu_ab_lib.sh tree 2>&1 | sed 's/^tree/tree(maps_end)/' | tee gpurun_out/r5ae/ab.txt
bash tools/gpu_ab_lib.sh tree ms16 ms63 2>&1 | tee -a gpurun_out/r5ae/ab.txt
