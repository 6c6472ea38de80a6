# GPU box, round 5: the pair kernel's workgroup timeline, single-frame path and the batch path
# (the bench's shape: each launch carries later frames' pyramid / bilateral workgroups).
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5s
mkdir -p $O
TFUSION_HIP_LIB=$PWD/tools/_build/ptl/libtfusion_hip.so timeout -k 10 200 python tools/pair_timeline.py > $O/ptl_single.txt 2>&1 || { tail -20 $O/ptl_single.txt; exit 1; }
grep -v resident $O/ptl_single.txt | head -12
PTL_BATCH=1 TFUSION_HIP_LIB=$PWD/tools/_build/ptl_la/libtfusion_hip.so timeout -k 10 200 python tools/pair_timeline.py > $O/ptl_batch.txt 2>&1 || { tail -20 $O/ptl_batch.txt; exit 1; }
cat $O/ptl_batch.txt
