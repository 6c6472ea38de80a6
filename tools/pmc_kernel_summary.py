"""Per-kernel averages of the rocprofv3 PMC passes tools/gpu_pmc_kernel.sh writes (one
directory per pass), for the dispatches of one kernel: counters, and the derived occupancy
(4 * SQ_WAVE_CYCLES / GRBM_GUI_ACTIVE / CUs; SQ_WAVE_CYCLES counts in units of 4 cycles on
gfx950), wait fraction, VALU instructions per wave, and traffic (FETCH_SIZE x2 for wide
reads, see pmc_traffic.py).

    python tools/pmc_kernel_summary.py gpurun_out/pmck_TAG KERNEL_SUBSTRING [--top-quartile]
"""
import csv, glob, json, os, sys
from collections import defaultdict

CU_NUM = 256


def main():
    root, kern = sys.argv[1], sys.argv[2]
    top = "--top-quartile" in sys.argv
    avg = {}
    for pdir in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(pdir):
            continue
        per = defaultdict(lambda: defaultdict(float))
        for path in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                if kern not in r["Kernel_Name"]:
                    continue
                per[r.get("Dispatch_Id", r.get("Correlation_Id"))][r["Counter_Name"]] += float(r["Counter_Value"])
        ds = list(per.values())
        if not ds:
            continue
        if top and "GRBM_GUI_ACTIVE" in ds[0]:
            ds.sort(key=lambda d: d["GRBM_GUI_ACTIVE"])
            ds = ds[len(ds) // 4:]
        for k in ds[0]:
            avg[k] = sum(d.get(k, 0.0) for d in ds) / len(ds)
        avg["dispatches_" + os.path.basename(pdir)] = len(ds)
    out = {"kernel": kern, "raw": {k: round(v, 1) for k, v in sorted(avg.items())}}
    g = avg.get("GRBM_GUI_ACTIVE")
    if g and "SQ_WAVE_CYCLES" in avg:
        out["waves_per_cu"] = round(4.0 * avg["SQ_WAVE_CYCLES"] / g / CU_NUM, 2)
        out["wait_any_frac"] = round(avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"], 3)
        out["busy_ms_at_2.4GHz"] = round(g / 2.4e6, 4)
    if "SQ_INSTS_VALU" in avg:
        out["valu_per_wave"] = round(avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"], 1)
        out["vmem_rd_per_wave"] = round(avg["SQ_INSTS_VMEM_RD"] / avg["SQ_WAVES"], 1)
        out["vmem_wr_per_wave"] = round(avg["SQ_INSTS_VMEM_WR"] / avg["SQ_WAVES"], 1)
        out["salu_per_wave"] = round(avg["SQ_INSTS_SALU"] / avg["SQ_WAVES"], 1)
    if "FETCH_SIZE" in avg:
        out["fetch_bytes_x2"] = int(avg["FETCH_SIZE"] * 1024 * 2)
    if "WRITE_SIZE" in avg:
        out["write_bytes"] = int(avg["WRITE_SIZE"] * 1024)
    if "TCC_HIT_sum" in avg:
        out["l2_hit_rate"] = round(avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]), 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
