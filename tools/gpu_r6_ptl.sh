# GPU box, round 6: k_raycast_pair workgroup timelines (single tracked frame; last launch of a 32-frame batch).
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${1:-r6ptl}
mkdir -p $O
TFUSION_HIP_LIB=tools/_build/ptl/libtfusion_hip.so timeout -k 10 200 python tools/pair_timeline.py > $O/pair_timeline.txt 2>&1 || { tail -20 $O/pair_timeline.txt; exit 1; }
PTL_BATCH=1 TFUSION_HIP_LIB=tools/_build/ptl_la/libtfusion_hip.so timeout -k 10 200 python tools/pair_timeline.py > $O/pair_timeline_batch.txt 2>&1 || { tail -20 $O/pair_timeline_batch.txt; exit 1; }
head -16 $O/pair_timeline.txt | cut -c1-250
echo ==; head -16 $O/pair_timeline_batch.txt | cut -c1-250
