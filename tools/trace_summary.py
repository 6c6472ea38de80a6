import csv, sys
from collections import defaultdict
path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = defaultdict(list)
for r in rows:
    key = (r["Kernel_Name"].split("(")[0], r["Grid_Size_X"])
    by[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
tot = sum(sum(v) for v in by.values())
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0]:24s} grid={k[1]:>8} n={len(v):5d} avg={sum(v)/len(v):8.2f}us min={min(v):8.2f} tot%={100*sum(v)/tot:5.1f}")
gaps = defaultdict(list)
for a, b in zip(rows, rows[1:]):
    gaps[a["Kernel_Name"].split("(")[0] + "->" + b["Kernel_Name"].split("(")[0]].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000)
print("--- gaps (us)")
for k, v in sorted(gaps.items(), key=lambda kv: -len(kv[1]))[:12]:
    print(f"{k:50s} n={len(v):5d} avg={sum(v)/len(v):7.2f} min={min(v):7.2f}")
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1000
print("span us", span, "busy us", tot)
