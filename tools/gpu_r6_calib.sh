# GPU box, round 6: FETCH_SIZE calibration of scattered 4-byte gathers (tools/micro/fetch_calib.hip).
#   gpurun -- bash tools/gpu_r6_calib.sh TAG
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r6cal}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- $R/tools/micro/fetch_calib > $O/calib.log 2>&1 || { tail -20 $O/calib.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/req -o run -- $R/tools/micro/fetch_calib > $O/calib2.log 2>&1 || tail -5 $O/calib2.log
cat $O/calib.log
for f in $(find $O -name "*counter_collection.csv"); do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print(r.get("Dispatch_Id"), r.get("Kernel_Name", "")[:40], r.get("Counter_Name"), r.get("Counter_Value"))
PY
done
