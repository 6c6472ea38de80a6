# GPU box, round 5: the batch end's wait spins on hipStreamQuery (tree default) against
# hipStreamSynchronize (TFUSION_SYNC_SPIN=0): C2 A/B, alternated twice each.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5ac
bash tools/gpu_ab_env.sh base TFUSION_SYNC_SPIN=0 2>&1 | tee gpurun_out/r5ac/ab.txt
bash tools/gpu_ab_env.sh base TFUSION_SYNC_SPIN=0 2>&1 | tee -a gpurun_out/r5ac/ab.txt
