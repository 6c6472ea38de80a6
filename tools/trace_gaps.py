"""Dispatch gaps between consecutive kernels of a rocprofv3 kernel trace: for each (kernel, next
kernel) pair seen more than --min times, the p10 / p50 / p90 of next.start - kernel.end in us.

    python tools/trace_gaps.py gpurun_out/TAG/prof/run_kernel_trace.csv
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--min", type=int, default=500)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gaps = collections.defaultdict(list)
    for a, b in zip(rows, rows[1:]):
        key = (a["Kernel_Name"].split("(")[0], b["Kernel_Name"].split("(")[0])
        gaps[key].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000.0)
    for (ka, kb), v in gaps.items():
        if len(v) < args.min:
            continue
        v.sort()
        n = len(v)
        print(f"{ka:32s} -> {kb:32s} n={n:5d} p10 {v[n // 10]:6.2f} p50 {v[n // 2]:6.2f} p90 {v[9 * n // 10]:6.2f}")


if __name__ == "__main__":
    main()
