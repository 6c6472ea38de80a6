# GPU box, round 6: the parity sequence tests, repeated, for the current build and the
# TF_INTEG_COMPACT=0 build (a non-reproducible range-image difference seen once).
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${1:-r6fl}
mkdir -p $O
SEL="tests/test_gpu_parity.py -k sequence"
for k in 1 2 3; do
  for b in new old; do
    L=""; [ $b = old ] && L=tools/_build/nocompact/libtfusion_hip.so
    TFUSION_HIP_LIB=$L timeout -k 10 400 python -u -m pytest $SEL -m gpu -q -rs --timeout 300 --timeout-method thread > $O/t_${b}_$k.log 2>&1 || true
    echo "$b $k: $(tail -1 $O/t_${b}_$k.log)"; grep -E "^E +AssertionError" $O/t_${b}_$k.log | head -2 || true
  done
done
