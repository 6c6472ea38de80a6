"""Per-frame-type HBM-side traffic of the frame kernels on the bench's TIMED frames, from rocprofv3
PMC passes over tools/pmc_frames.py (one pass for FETCH_SIZE, one for WRITE_SIZE), corrected as
MI355X_MICROARCH.md §HBM prescribes (gfx950 FETCH_SIZE counts half the bytes of wide reads: x2;
WRITE_SIZE as is; KiB -> B).  Dispatch i of a frame kernel is frame i (one launch per frame, in
order); frames are split by what they were (tracked / reset / frame0).  Beside each, the
algorithmic bytes per launch of the same frames (bench.stage_bytes with the timed region's
visible-block and voxel-lane means), and the ratio.  Updates profiles/pmc_traffic.json["C2"].

    python tools/pmc_frames_summary.py FETCH_DIR WRITE_DIR FRAMES.json [profiles/pmc_traffic.json]"""
import csv, glob, json, os, sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KERNELS = [("k_icp_frame", "icp"), ("k_raycast_pair", "raycast_icp"), ("k_integrate<true, false>", "integrate"),
           ("k_alloc_requests", "alloc_requests"), ("k_alloc_apply", "alloc_apply"), ("k_vis_count", "vis_count"),
           ("k_vis_apply", "vis_apply"), ("k_icp_maps_end", "icp_maps_end")]


def dispatches(root, counter):
    """{kernel name: [counter value per dispatch, in dispatch order]}"""
    rows = []
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    by = defaultdict(list)
    for _, k, v in rows:
        by[k].append(v)
    return by


def main():
    fdir, wdir, fjson = sys.argv[1], sys.argv[2], sys.argv[3]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "profiles", "pmc_traffic.json")
    fr = json.load(open(fjson))
    kind, first = fr["kind"], fr["timed_first"]
    fetch, write = dispatches(fdir, "FETCH_SIZE"), dispatches(wdir, "WRITE_SIZE")
    import bench
    from topfusion_amd import default_params, synth
    W, H = 640, 480
    fx, fy, cx, cy = synth.intrinsics(W, H)
    p = default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy)
    nvis = fr["nvis_mean_integrated"]
    lanes = fr["lanes_per_integrated_frame"]
    res = {}
    for key, stage in KERNELS:
        fk = [k for k in fetch if key in k.split("(")[0] or k.startswith(key)]
        wk = [k for k in write if key in k.split("(")[0] or k.startswith(key)]
        if not fk or not wk:
            continue
        fv, wv = fetch[fk[0]], write[wk[0]]
        if len(fv) != len(kind) or len(wv) != len(kind):
            res[stage] = {"error": f"{len(fv)} / {len(wv)} dispatches for {len(kind)} frames"}
            continue
        ent = {"kernel": fk[0].split("(")[0]}
        for t in ("tracked", "reset", "frame0"):
            idx = [i for i in range(first, len(kind)) if kind[i] == t]
            if not idx:
                continue
            fb = sum(fv[i] for i in idx) / len(idx) * 1024 * 2
            wb = sum(wv[i] for i in idx) / len(idx) * 1024
            ent[t] = {"frames": len(idx), "fetch_bytes": round(fb), "write_bytes": round(wb), "bytes": round(fb + wb)}
        alg = bench.stage_bytes(stage, p, nvis, W, H, lanes if stage == "integrate" else None)
        if alg and "tracked" in ent:
            ent["algorithmic_bytes_tracked"] = int(alg)
            ent["ratio_traffic_to_algorithmic"] = round(ent["tracked"]["bytes"] / alg, 3)
        res[stage] = ent
    res["_frames"] = {"timed": len(kind) - first, "first": first,
                      "by_kind": {t: sum(1 for k in kind[first:] if k == t) for t in ("tracked", "reset", "frame0")},
                      "nvis_mean_integrated": round(nvis, 1), "lanes_per_integrated_frame": [round(v) for v in lanes],
                      "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads), WRITE_SIZE x1, KiB->B",
                      "source": [os.path.basename(os.path.normpath(fdir)), os.path.basename(os.path.normpath(wdir))]}
    allcfg = json.load(open(out)) if os.path.exists(out) else {}
    allcfg["C2"] = res
    json.dump(allcfg, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
