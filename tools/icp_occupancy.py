"""Occupancy, wait and LDS figures of the ICP kernel (k_icp_frame) from a rocprofv3 PMC pass
(tools/gpu_pmc.sh pass "occ": SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT
SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE), derived with rocprofiler-sdk's
gfx950 definitions (counter_defs.yaml): SQ_WAVE_CYCLES counts in units of 4 cycles and rocprofv3
reports GRBM_GUI_ACTIVE summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back), so with
T = GRBM_GUI_ACTIVE / 8 the dispatch's active cycles: mean resident waves per CU =
4 * SQ_WAVE_CYCLES / T / CU_NUM (OccupancyPercent = that / 32 waves per CU); wait fraction =
SQ_WAIT_ANY / SQ_WAVE_CYCLES; LDS bank-conflict cycles per conflict-free cycle =
SQ_LDS_BANK_CONFLICT / (SQ_LDS_IDX_ACTIVE - SQ_LDS_BANK_CONFLICT); LDS utilisation =
SQ_LDS_IDX_ACTIVE / (T * CU_NUM).  Only full launches count (GRBM_GUI_ACTIVE at least half its
90th percentile: the frames whose ICP ran every iteration, as bench.py times).  Writes
profiles/icp_occupancy.json, which bench.py attaches to the ICP roofline entry.

    python tools/icp_occupancy.py gpurun_out/pmc_TAG/occ [CONFIG=C2] [profiles/icp_occupancy.json]
"""
import csv, glob, json, os, sys
from collections import defaultdict

CU_NUM = 256
XCD_NUM = 8
KERNEL = "k_icp_frame"


def main():
    root = sys.argv[1]
    config = sys.argv[2] if len(sys.argv) > 2 else "C2"
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                            "profiles", "icp_occupancy.json")
    per = defaultdict(lambda: defaultdict(float))       # dispatch -> counter -> value
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if KERNEL not in r["Kernel_Name"]:
                continue
            per[r.get("Dispatch_Id", r.get("Correlation_Id"))][r["Counter_Name"]] += float(r["Counter_Value"])
    # dispatches that ran the tracking path (frame-0 / post-reset launches exit at once)
    ds = [d for d in per.values() if d.get("SQ_WAVE_CYCLES", 0) > 0 and d.get("GRBM_GUI_ACTIVE", 0) > 0]
    ds.sort(key=lambda d: d["GRBM_GUI_ACTIVE"])
    p90 = ds[int(0.9 * (len(ds) - 1))]["GRBM_GUI_ACTIVE"] if ds else 0
    ds = [d for d in ds if d["GRBM_GUI_ACTIVE"] >= 0.5 * p90]   # full launches only
    if not ds:
        print("no k_icp_frame dispatches found")
        return 1
    avg = {k: sum(d.get(k, 0.0) for d in ds) / len(ds) for k in ds[0]}
    T = avg["GRBM_GUI_ACTIVE"] / XCD_NUM
    waves_cu = 4.0 * avg["SQ_WAVE_CYCLES"] / T / CU_NUM
    res = {
        "kernel": KERNEL, "dispatches": len(ds),
        "designed": "256 workgroups x 8 waves, one workgroup per CU (56 KiB LDS pad): 8 waves/CU = 2 per SIMD",
        "mean_waves_per_cu": round(waves_cu, 3),
        "mean_waves_per_simd": round(waves_cu / 4, 3),
        "occupancy_pct_of_32_waves_per_cu": round(100 * waves_cu / 32, 2),
        "wait_any_frac_of_wave_cycles": round(avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"], 4),
        "lds_bank_conflict_ratio": round(avg["SQ_LDS_BANK_CONFLICT"] / max(1.0, avg["SQ_LDS_IDX_ACTIVE"] - avg["SQ_LDS_BANK_CONFLICT"]), 5),
        "lds_util_frac": round(avg["SQ_LDS_IDX_ACTIVE"] / (T * CU_NUM), 5),
        "active_cycles_per_launch": round(T, 1),
        "lds_insts_per_wave": round(avg.get("SQ_INSTS_LDS", 0.0) / max(1.0, avg["SQ_WAVES"]), 1),
        "raw_avg": {k: round(v, 1) for k, v in avg.items()},
        "source": os.path.relpath(root),
    }
    allcfg = json.load(open(out)) if os.path.exists(out) else {}
    allcfg[config] = res
    json.dump(allcfg, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
