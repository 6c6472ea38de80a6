"""Per-kernel averages of the rocprofv3 PMC passes tools/gpu_pmc_kernel.sh writes (one
directory per pass), for the dispatches of one kernel, and the figures derived from them.

Unit conventions (MI355X_MICROARCH.md; rocprofiler-sdk's gfx950 counter definitions):
  * GRBM_GUI_ACTIVE is reported summed over the 8 XCDs: a dispatch's active cycles are
    T = GRBM_GUI_ACTIVE / 8 (the guide's "DVFS give-back" note; it reads high on dispatches
    shorter than ~0.3 ms).
  * SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_* count quad-cycles (guide, "s_memtime tick vs SQ
    PMC units"): wave cycles = 4 x SQ_WAVE_CYCLES.
  * A wave64 VALU instruction takes 2 cycles of its SIMD's issue when waves share the SIMD (4 for
    one wave alone; guide, "Wave scheduling" and the per-instruction table).
Derived:
  waves_per_cu       = 4 SQ_WAVE_CYCLES / T / 256        mean resident waves per CU
  wave_lifetime_us   = 4 SQ_WAVE_CYCLES / SQ_WAVES / 2.4 GHz
  wait_any_frac      = SQ_WAIT_ANY / SQ_WAVE_CYCLES       (waiting on anything: memory, barriers, ...)
  issue_stall_frac   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES  (ready but not issued)
  valu_issue_frac    = 2 SQ_INSTS_VALU / (T x 1024 SIMDs) (share of the chip's VALU issue slots)
  busy_ms_at_2.4GHz  = T / 2.4e6
  lds_*              = from SQ_INSTS_LDS / SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE when collected
  traffic            = FETCH_SIZE x 1024 x 2 (wide reads, pmc_traffic.py) + WRITE_SIZE x 1024

    python tools/pmc_kernel_summary.py gpurun_out/pmck_TAG KERNEL_SUBSTRING [--top-quartile] [--full] [-o OUT.json]
        [--source TEXT]   (the recipe that produced the passes, recorded in "source")
    python tools/pmc_kernel_summary.py --from-json profiles/rNN/pmc_kernel_X.json [-o OUT.json]
        (re-derive from the "raw" averages a summary already holds)
"""
import csv, glob, json, os, sys
from collections import defaultdict

CU_NUM = 256
XCD_NUM = 8
SIMD_NUM = 4 * CU_NUM
CLOCK_HZ = 2.4e9


def derive(kern, avg, note=None):
    out = {"kernel": kern, "raw": {k: round(v, 1) for k, v in sorted(avg.items())},
           "units": "T = GRBM_GUI_ACTIVE / 8 XCDs; SQ_* cycle counters x 4 (quad-cycles); 2 cycles of SIMD issue "
                    "per wave64 VALU instruction (tools/pmc_kernel_summary.py)"}
    if note:
        out["note"] = note
    g = avg.get("GRBM_GUI_ACTIVE")
    T = g / XCD_NUM if g else None
    if T and "SQ_WAVE_CYCLES" in avg:
        out["waves_per_cu"] = round(4.0 * avg["SQ_WAVE_CYCLES"] / T / CU_NUM, 2)
        out["wait_any_frac"] = round(avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"], 3)
        if "SQ_WAIT_INST_ANY" in avg:
            out["issue_stall_frac"] = round(avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"], 3)
        if "SQ_WAVES" in avg:
            out["wave_lifetime_us"] = round(4.0 * avg["SQ_WAVE_CYCLES"] / avg["SQ_WAVES"] / CLOCK_HZ * 1e6, 2)
    if T:
        out["busy_ms_at_2.4GHz"] = round(T / CLOCK_HZ * 1e3, 4)
    if "SQ_INSTS_VALU" in avg and avg.get("SQ_WAVES"):
        out["valu_per_wave"] = round(avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"], 1)
        out["vmem_rd_per_wave"] = round(avg["SQ_INSTS_VMEM_RD"] / avg["SQ_WAVES"], 1)
        out["vmem_wr_per_wave"] = round(avg["SQ_INSTS_VMEM_WR"] / avg["SQ_WAVES"], 1)
        out["salu_per_wave"] = round(avg["SQ_INSTS_SALU"] / avg["SQ_WAVES"], 1)
        if T:
            out["valu_issue_frac"] = round(2.0 * avg["SQ_INSTS_VALU"] / (T * SIMD_NUM), 3)
    if "SQ_INSTS_LDS" in avg and avg.get("SQ_WAVES"):
        out["lds_insts_per_wave"] = round(avg["SQ_INSTS_LDS"] / avg["SQ_WAVES"], 1)
    if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg:
        out["lds_bank_conflict_ratio"] = round(avg["SQ_LDS_BANK_CONFLICT"] / max(1.0, avg["SQ_LDS_IDX_ACTIVE"] - avg["SQ_LDS_BANK_CONFLICT"]), 5)
        if T:
            out["lds_util_frac"] = round(avg["SQ_LDS_IDX_ACTIVE"] / (T * CU_NUM), 5)
    if "FETCH_SIZE" in avg:
        out["fetch_bytes_x2"] = int(avg["FETCH_SIZE"] * 1024 * 2)
    if "WRITE_SIZE" in avg:
        out["write_bytes"] = int(avg["WRITE_SIZE"] * 1024)
    if "TCC_HIT_sum" in avg:
        out["l2_hit_rate"] = round(avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]), 4)
    return out


def collect(root, kern, top=False, full=False):
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
        if (top or full) and "GRBM_GUI_ACTIVE" in ds[0]:
            ds.sort(key=lambda d: d["GRBM_GUI_ACTIVE"])
            if top:
                ds = ds[len(ds) // 4:]
            else:       # full launches (e.g. ICP frames that ran every iteration): >= half the p90
                p90 = ds[int(0.9 * (len(ds) - 1))]["GRBM_GUI_ACTIVE"]
                ds = [d for d in ds if d["GRBM_GUI_ACTIVE"] >= 0.5 * p90]
        for k in ds[0]:
            avg[k] = sum(d.get(k, 0.0) for d in ds) / len(ds)
        avg["dispatches_" + os.path.basename(pdir)] = len(ds)
    return avg


def main():
    args = sys.argv[1:]
    out_path = None
    source = None
    if "--source" in args:
        i = args.index("--source")
        source = args[i + 1]
        del args[i:i + 2]
    if "-o" in args:
        i = args.index("-o")
        out_path = args[i + 1]
        del args[i:i + 2]
    if args and args[0] == "--from-json":
        src = json.load(open(args[1]))
        res = derive(src["kernel"], src["raw"], src.get("note"))
        for k in ("source", "config"):
            if k in src:
                res[k] = src[k]
    else:
        root, kern = args[0], args[1]
        avg = collect(root, kern, "--top-quartile" in args, "--full" in args)
        res = derive(kern, avg)
        res["source"] = source or os.path.relpath(root)
    text = json.dumps(res, indent=1)
    if out_path:
        open(out_path, "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
