# GPU box, round 6: XCD bands -- k_vis_build / k_integrate timelines (TF_VIS_TIMELINE build), bands on / off.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${1:-r6bands9}
mkdir -p $O
for b in 1 0; do
TFUSION_INTEG_BANDS=$b TFUSION_HIP_LIB=tools/_build/vtl/libtfusion_hip.so timeout -k 10 200 python tools/band_check.py > $O/band_check_b$b.txt 2>&1 || { tail -20 $O/band_check_b$b.txt; exit 1; }
echo "== bands $b"; tail -9 $O/band_check_b$b.txt
done
