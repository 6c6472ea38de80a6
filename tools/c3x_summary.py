"""C3I's reads split by source, from tools/gpu_c3x.sh's output: per library
(tree; TF_C3X=1 no depth-image traffic, =2 no voxel loads, =3 neither) the pass time, PMC
FETCH_SIZE (x2, tools/pmc_traffic.py) and the L2's memory-side read requests TCC_EA0_RDREQ.

    python tools/c3x_summary.py gpurun_out/c3x > profiles/r05/c3i_read_attribution.json"""
import csv, glob, json, os, sys
from collections import defaultdict


def req_counts(root):
    vals = defaultdict(list)
    for p in glob.glob(os.path.join(root, "req", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if "k_integrate" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sorted(v)[len(v) // 2] for k, v in vals.items()}


def main():
    d = sys.argv[1]
    out = {"is": "C3I (2^21 - 1 blocks, 1280x960 dists of a wall at 1.5 m): one integrate pass, per diagnostic build",
           "builds": {"tree": "product", "c3x1": "TF_C3X=1: every depth sample reads pixel 0",
                      "c3x2": "TF_C3X=2: no voxel loads", "c3x3": "TF_C3X=3: both"}, "runs": {}}
    for v in ("tree", "c3x1", "c3x2", "c3x3"):
        line = json.loads(open(os.path.join(d, f"c3i_{v}.log")).read().strip().splitlines()[-1])
        t = json.load(open(os.path.join(d, f"traffic_{v}.json")))["C3I"]["integrate"]
        rq = req_counts(os.path.join(d, f"pmc_{v}"))
        out["runs"][v] = {"ms_per_pass": line["ms_per_step"], "fetch_bytes_x2": t["fetch_bytes_per_launch"],
                          "write_bytes": t["write_bytes_per_launch"], "TCC_EA0_RDREQ_sum": rq.get("TCC_EA0_RDREQ_sum"),
                          "TCC_EA0_RDREQ_32B_sum": rq.get("TCC_EA0_RDREQ_32B_sum")}
    r = out["runs"]
    out["attribution"] = {
        "depth_samples": {"fetch_bytes_x2": r["tree"]["fetch_bytes_x2"] - r["c3x1"]["fetch_bytes_x2"],
                          "read_requests": r["tree"]["TCC_EA0_RDREQ_sum"] - r["c3x1"]["TCC_EA0_RDREQ_sum"],
                          "ms": round(r["tree"]["ms_per_pass"] - r["c3x1"]["ms_per_pass"], 4)},
        "voxel_lanes": {"fetch_bytes_x2": r["tree"]["fetch_bytes_x2"] - r["c3x2"]["fetch_bytes_x2"],
                        "read_requests": r["tree"]["TCC_EA0_RDREQ_sum"] - r["c3x2"]["TCC_EA0_RDREQ_sum"],
                        "ms": round(r["tree"]["ms_per_pass"] - r["c3x2"]["ms_per_pass"], 4)},
        "rest_ids_entries": {"fetch_bytes_x2": r["c3x3"]["fetch_bytes_x2"], "read_requests": r["c3x3"]["TCC_EA0_RDREQ_sum"]},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
