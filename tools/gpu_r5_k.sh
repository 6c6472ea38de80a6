# GPU box, round 5: is the ICP tail's in-kernel slowness instruction fetch?  The timing build's
# timeline with each tail half run twice back to back (shader-clock cycles), and a PMC pass of
# the instruction-cache counters over a short C2 run.   gpurun -- bash tools/gpu_r5_k.sh TAG
set -e
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-r5k}
O=$R/gpurun_out/$TAG
mkdir -p $O
TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so timeout -k 10 120 python tools/icp_timeline.py > $O/icp_timeline.txt 2>&1 \
  || { tail -20 $O/icp_timeline.txt; exit 1; }
tail -26 $O/icp_timeline.txt | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --output-format csv \
  -d $O/pmc_icache -o run -- python3 $R/bench.py --steps 2 --warmup 1 --per-call-frames 0 --no-cpu-baseline --no-profile \
  > $O/pmc_icache.log 2>&1 || { tail -20 $O/pmc_icache.log; exit 1; }
python3 - <<PY
import csv, glob, collections
v = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob("$O/pmc_icache/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0][:40]
        v[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(v.items()):
    print(k, {c: int(sorted(x)[len(x) // 2]) for c, x in cs.items()}, "launches", len(next(iter(cs.values()))))
PY
