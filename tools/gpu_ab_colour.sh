# GPU box: the colour-TSDF parity tests on each library variant, then an A/B of the C2 colour line
# (bench.py --colour) over the variants, alternated twice.  Variants: tools/_build/<v>/ or "tree".
#   gpurun -- bash tools/gpu_ab_colour.sh TAG v1 v2 ...
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
lib() { if [ $1 = tree ]; then echo $PWD/topfusion_amd/libtfusion_hip.so; else echo $PWD/tools/_build/$1/libtfusion_hip.so; fi; }
for v in "$@"; do
  TFUSION_HIP_LIB=$(lib $v) timeout -k 10 400 python -u -m pytest tests/test_gpu_colour.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -40 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
for round in 1 2; do
  for v in "$@"; do
    TFUSION_HIP_LIB=$(lib $v) timeout -k 10 300 python bench.py --colour --no-cpu-baseline --per-call-frames 0 > $O/bench_$v.log 2>&1 \
      || { tail -20 $O/bench_$v.log; exit 1; }
    python -c "
import json
e=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1])
print('$v', 'colour fps', e['value'], {k: v for k, v in e['stage_ms_per_frame'].items() if v})"
  done
done
