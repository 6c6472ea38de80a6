"""Mean end -> start gap (us) per consecutive kernel pair of a rocprofv3 kernel-trace CSV."""
import csv, sys
from collections import defaultdict
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
g = defaultdict(list)
for a, b in zip(rows, rows[1:]):
    g[(a["Kernel_Name"].split("(")[0], b["Kernel_Name"].split("(")[0])].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
for k, v in sorted(g.items(), key=lambda kv: -len(kv[1])):
    v = sorted(v)
    print(f"{k[0]:>12} -> {k[1]:<12} n={len(v):4d} median={v[len(v)//2]:6.2f} mean={sum(v)/len(v):6.2f}")
