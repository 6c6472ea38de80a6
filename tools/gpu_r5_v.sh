# GPU box, round 5: address-translation PMC (UTCL1 hits / misses) of k_raycast_pair, tree library
# (VBA reads) against the SDF-mirror variant (tools/_build/sdfm8a).
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/r5v
mkdir -p $O
ARGS="--steps 2 --warmup 1 --per-call-frames 0 --no-cpu-baseline --no-profile"
for v in tree sdfm8a; do
  if [ $v = tree ]; then L=$R/topfusion_amd/libtfusion_hip.so; else L=$R/tools/_build/$v/libtfusion_hip.so; fi
  TFUSION_HIP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum \
    --output-format csv -d $O/$v -o run -- python3 $R/bench.py $ARGS > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  python3 - $O/$v <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
acc = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name']
    if 'raycast_pair' in k or 'integrate' in k or 'icp_frame' in k:
        acc[k[:30]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in acc.items():
    print(sys.argv[1].split('/')[-1], k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
done
