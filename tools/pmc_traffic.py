"""HBM-side traffic per launch of the bench's single-kernel stages, from the rocprofv3 PMC
passes of tools/gpu_pmc.sh, corrected as MI355X_MICROARCH.md §HBM prescribes (gfx950
FETCH_SIZE reports half the bytes of wide reads: x2; WRITE_SIZE as is; both in KiB).
Only full launches count (per counter: at least half its 90th percentile), as bench.py times
only frames whose stage ran.  Writes profiles/pmc_traffic.json, which bench.py reads for
roofline.traffic.

    python tools/pmc_traffic.py gpurun_out/pmc_TAG [CONFIG=C2] [profiles/pmc_traffic.json]

The output holds one entry per bench config (C2, C3); an existing file is updated in place."""
import csv, glob, json, os, sys
from collections import defaultdict

STAGE_OF = [("k_icp_frame", "icp"), ("k_raycast_pair", "raycast_icp"), ("k_integrate", "integrate")]


def per_kernel(root, counter):
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def full(vals):
    """The launches that did the stage's whole work: at least half the 90th percentile (frame-0
    and failed-ICP frames launch the kernels too, and they exit early)."""
    if not vals:
        return vals
    p90 = sorted(vals)[int(0.9 * (len(vals) - 1))]
    return [v for v in vals if v >= 0.5 * p90]


def main():
    root = sys.argv[1]
    config = sys.argv[2] if len(sys.argv) > 2 else "C2"
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                            "profiles", "pmc_traffic.json")
    fetch, write = per_kernel(root, "FETCH_SIZE"), per_kernel(root, "WRITE_SIZE")
    res = {}
    for key, stage in STAGE_OF:
        f = full([v for k, vs in fetch.items() if key in k for v in vs])
        w = full([v for k, vs in write.items() if key in k for v in vs])
        if not f or not w:
            continue
        fb = sum(f) / len(f) * 1024 * 2
        wb = sum(w) / len(w) * 1024
        res[stage] = {"kernel": key, "fetch_bytes_per_launch": round(fb), "write_bytes_per_launch": round(wb),
                      "bytes_per_launch": round(fb + wb), "launches_sampled": len(f),
                      "source": os.path.basename(os.path.normpath(root)),
                      "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads), WRITE_SIZE x1, KiB->B"}
    allcfg = {}
    if os.path.exists(out):
        allcfg = json.load(open(out))
    allcfg[config] = res
    json.dump(allcfg, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
