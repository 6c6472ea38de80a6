"""Per-kernel summary of a rocprofv3 --kernel-trace CSV (the committed profiles/rNN_kernel_trace_summary.txt).

The device-driven frame loop enqueues every stage of every frame; on frames where the device
decided a stage does not run (frame-0 path after a reset, ICP failure) the launch exits at
once (~1.5 us).  `avg_exec` averages only the launches that did work (> EARLY_US), which is
what bench.py's HIP events report ("averages per executed launch").  `avg_full` averages the
launches of at least half the 90th-percentile duration: for k_icp_frame these are the frames whose
ICP ran all its iterations (bench.py times only those: stage_ran), the others ending early at a
failed det check; `med_full` is their median, and launches past 20x the median are reported as
`stalled` and left out (queue stalls under the profiler, not kernel time)."""
import csv, sys
from collections import defaultdict
EARLY_US = 3.0
path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = defaultdict(list)
for r in rows:
    key = (r["Kernel_Name"].split("(")[0], r["Grid_Size_X"])
    by[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
tot = sum(sum(v) for v in by.values())
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    ex = [x for x in v if x > EARLY_US]
    avg_ex = sum(ex) / len(ex) if ex else 0.0
    p90 = sorted(v)[int(0.9 * (len(v) - 1))]
    full = [x for x in v if x >= 0.5 * p90]
    # launches stretched past 20x the median by something outside the kernel (a stall of the
    # queue under the profiler: two pair launches of 17-19 ms in round 5's trace) are counted
    # apart, not averaged in
    med = sorted(v)[len(v) // 2]
    stalled = [x for x in full if x > 20 * med]
    full = [x for x in full if x <= 20 * med]
    fs = sorted(full)
    print(f"{k[0]:24s} grid={k[1]:>8} n={len(v):5d} avg={sum(v)/len(v):8.2f}us n_exec={len(ex):5d} "
          f"avg_exec={avg_ex:8.2f}us n_full={len(full):5d} avg_full={sum(full)/len(full):8.2f}us "
          f"med_full={fs[len(fs) // 2]:8.2f}us stalled={len(stalled)} min={min(v):8.2f} tot%={100*sum(v)/tot:5.1f}")
gaps = defaultdict(list)
for a, b in zip(rows, rows[1:]):
    gaps[a["Kernel_Name"].split("(")[0] + "->" + b["Kernel_Name"].split("(")[0]].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000)
print("--- gaps (us)")
for k, v in sorted(gaps.items(), key=lambda kv: -len(kv[1]))[:12]:
    print(f"{k:50s} n={len(v):5d} avg={sum(v)/len(v):7.2f} min={min(v):7.2f}")
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1000
print("span us", span, "busy us", tot)
