set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${1:-r6dv}
mkdir -p $O
timeout -k 10 300 python tools/seq_diverge.py 16 > $O/new.txt 2>&1 || { tail -20 $O/new.txt; exit 1; }
cat $O/new.txt
TFUSION_HIP_LIB=tools/_build/nocompact/libtfusion_hip.so timeout -k 10 300 python tools/seq_diverge.py 16 > $O/old.txt 2>&1 || { tail -20 $O/old.txt; exit 1; }
echo "== old"; cat $O/old.txt
