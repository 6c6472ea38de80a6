"""Per-kernel averages of the rocprofv3 PMC passes written by tools/gpu_pmc.sh."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
for path in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
names = sorted({c for k in agg for c in agg[k]})
for k in sorted(agg):
    d = {c: sum(v) / len(v) for c, v in agg[k].items()}
    print(k)
    for c in names:
        if c in d:
            print(f"   {c:22s} {d[c]:16.1f}")
