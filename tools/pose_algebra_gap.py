"""How far the canonical pose algebra (LDL^T solve + sinc Rodrigues: the GPU's default, shared
with the oracle) is from the reference's own -- OpenCV's cv::determinant / cv::solve(DECOMP_SVD)
/ cv::Affine3f(rvec, t) (projective_icp.cpp:197-209), restated in oracle/tf_oracle.c as a
test-only mode ("What's missing" 2).

The oracle runs the same frames in lockstep in several contexts, one per pose algebra, and per
frame records, against the first ("canonical"):
  * the largest relative pose difference  max|P_b - P_a| / max|P_a|  (3x4 camera->world pose),
  * ICP reset flips (the frame's bool differs) and ICP iteration-count differences,
  * the allocated-block set (hash entries with ptr >= 0, by block position) and the visible
    set (visible list, by block position): sizes of the symmetric differences,
  * every `--tsdf-every` frames, over the blocks both allocated: voxels whose weight differs and
    the largest |sdf| difference in LSB.

    python tools/pose_algebra_gap.py --config C2 --frames 800 --out profiles/r05/pose_algebra_gap_C2.json
    python tools/pose_algebra_gap.py --config C5 --frames 2000 --out profiles/r05/pose_algebra_gap_C5.json

Test infrastructure: CPU only, the oracle's OpenMP build; frames are the bench's own
(synth.render_room: the bits synth/tf_synth.hip renders on the GPU)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O            # noqa: E402
from topfusion_amd import synth           # noqa: E402

MODES = {"canonical": ("canonical", False), "opencv4_portable": ("opencv4", False),
         "opencv4_libm": ("opencv4", True), "opencv2_libm": ("opencv2", True)}


def frame_at(cfg, k, W, H, poses):
    R, t = poses
    return synth.render_room(R[k], t[k], W, H, seed=cfg["seed"], frame=k)


def block_keys(h, ids=None):
    """int64 keys of block positions: every allocated entry, or the entries `ids`."""
    e = h if ids is None else h[ids]
    if ids is None:
        e = e[e["ptr"] >= 0]
    return np.sort((e["x"].astype(np.int64) + 32768) << 32 | (e["y"].astype(np.int64) + 32768) << 16 |
                   (e["z"].astype(np.int64) + 32768))


def tsdf_diff(oa, ob):
    """Over the blocks allocated in both: voxels whose weight differs, largest |sdf| diff (LSB)."""
    ha, hb = oa.hash(), ob.hash()
    va, vb = oa.vba(), ob.vba()
    ka, kb = block_keys(ha), block_keys(hb)
    common = np.intersect1d(ka, kb)

    def ptrs(h, keys):
        e = h[h["ptr"] >= 0]
        k = (e["x"].astype(np.int64) + 32768) << 32 | (e["y"].astype(np.int64) + 32768) << 16 | (e["z"].astype(np.int64) + 32768)
        order = np.argsort(k)
        return e["ptr"][order][np.searchsorted(k[order], keys)]
    pa, pb = ptrs(ha, common), ptrs(hb, common)
    sa = va.reshape(-1, 512)[pa]
    sb = vb.reshape(-1, 512)[pb]
    dw = int((sa["w"] != sb["w"]).sum())
    ds = np.abs(sa["sdf"].astype(np.int32) - sb["sdf"].astype(np.int32))
    return {"common_blocks": int(len(common)), "voxels_weight_differs": dw,
            "voxels_sdf_differs": int((ds > 0).sum()), "max_sdf_diff_lsb": int(ds.max()) if ds.size else 0,
            "voxels_compared": int(sa.size)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=["C2", "C5"], default="C2")
    ap.add_argument("--frames", type=int, default=800)
    ap.add_argument("--modes", default="canonical,opencv4_portable,opencv4_libm,opencv2_libm")
    ap.add_argument("--tsdf-every", type=int, default=100)
    ap.add_argument("--out", default=None)
    ap.add_argument("--one-step", action="store_true",
                    help="instead of independent runs: before every frame, each compared mode's context takes a copy "
                         "of the baseline context's state, runs that one frame, and is compared with the baseline "
                         "after it -- the per-frame (local) disagreement, without the divergence of the trajectories")
    args = ap.parse_args()
    if args.one_step:
        return one_step(args)
    W, H = 640, 480
    if args.config == "C2":
        cfg = dict(seed=7, voxel=0.005)
        R = np.empty((args.frames, 3, 3)); t = np.empty((args.frames, 3))
        for k in range(args.frames):
            R[k], t[k] = synth.orbit_pose(k)
    else:
        cfg = dict(seed=13, voxel=0.01)
        R, t = synth.random_walk_poses(args.frames, seed=13)
    fx, fy, cx, cy = synth.intrinsics(W, H)
    kw = dict(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy, voxelSize=cfg["voxel"])
    names = args.modes.split(",")
    ctx = {m: O.Oracle(O.default_params(**kw), omp=True) for m in names}
    base = names[0]
    rec = {m: {"ok": [], "iters": [], "pose_rel": [], "alloc_xor": [], "visible_xor": [], "tsdf": {}} for m in names[1:]}
    base_ok, base_blocks = [], []
    t0 = time.time()
    for k in range(args.frames):
        f = frame_at(cfg, k, W, H, (R, t))
        res = {}
        for m in names:
            mode, libm = MODES[m]
            O.set_pose_algebra(mode, libm)
            ok = ctx[m](f)
            c = ctx[m].counters()
            h = ctx[m].hash()
            res[m] = (ok, c["icp_iterations"], ctx[m].pose().astype(np.float64), block_keys(h),
                      block_keys(h, ctx[m].visible_ids()))
        ok_a, it_a, P_a, al_a, vi_a = res[base]
        base_ok.append(bool(ok_a)); base_blocks.append(int(len(al_a)))
        for m in names[1:]:
            ok_b, it_b, P_b, al_b, vi_b = res[m]
            r = rec[m]
            r["ok"].append(bool(ok_b)); r["iters"].append(int(it_b) - int(it_a))
            r["pose_rel"].append(float(np.abs(P_b - P_a).max() / max(np.abs(P_a).max(), 1e-30)))
            r["alloc_xor"].append(int(len(np.setxor1d(al_a, al_b, assume_unique=True))))
            r["visible_xor"].append(int(len(np.setxor1d(vi_a, vi_b, assume_unique=True))))
            if args.tsdf_every and (k + 1) % args.tsdf_every == 0:
                r["tsdf"][str(k)] = tsdf_diff(ctx[base], ctx[m])
        if (k + 1) % 50 == 0:
            print(f"frame {k + 1}/{args.frames} {time.time() - t0:.0f}s " +
                  " ".join(f"{m}: pose {max(rec[m]['pose_rel']):.2e} flips {sum(a != b for a, b in zip(base_ok, rec[m]['ok']))} "
                           f"alloc_xor {rec[m]['alloc_xor'][-1]}" for m in names[1:]), flush=True)
    out = {"config": args.config, "frames": args.frames, "W": W, "H": H, "voxel_m": cfg["voxel"],
           "frames_are": "synth.render_room at the bench's poses (orbit seed 7 / walk seed 13), bit-identical to "
                         "the GPU-rendered bench stream",
           "baseline_mode": base, "baseline_resets": int(sum(not x for x in base_ok[1:])),
           "baseline_allocated_blocks_last": base_blocks[-1], "modes": {}}
    for m in names[1:]:
        r = rec[m]
        flips = [k for k in range(args.frames) if base_ok[k] != r["ok"][k]]
        pr = np.array(r["pose_rel"])
        ax, vx = np.array(r["alloc_xor"]), np.array(r["visible_xor"])
        first = lambda a: (int(np.argmax(a > 0)) if (a > 0).any() else None)   # noqa: E731
        out["modes"][m] = {
            "pose_algebra": MODES[m][0], "transcendentals": "glibc" if MODES[m][1] else "portable (tfo_sincos, tfo_cv_hypot)",
            "max_pose_rel_diff": float(pr.max()), "frames_pose_bits_differ": int((pr > 0).sum()),
            "first_frame_pose_differs": first(pr), "pose_rel_diff_p50_p99": [float(np.percentile(pr, 50)), float(np.percentile(pr, 99))],
            "frames_pose_rel_diff_over_1e-4": int((pr > 1e-4).sum()),
            "reset_flips": len(flips), "reset_flip_frames": flips[:50],
            "resets": int(sum(not x for x in r["ok"][1:])),
            "frames_iteration_count_differs": int(sum(x != 0 for x in r["iters"])),
            "first_frame_alloc_differs": first(ax), "frames_alloc_differs": int((ax > 0).sum()),
            "alloc_xor_max": int(ax.max()), "alloc_xor_mean": float(ax.mean()),
            "first_frame_visible_differs": first(vx), "frames_visible_differs": int((vx > 0).sum()),
            "visible_xor_max": int(vx.max()), "visible_xor_mean": float(vx.mean()),
            "tsdf_checkpoints": r["tsdf"],
            "per_frame": {"pose_rel": [float(f"{x:.3g}") for x in pr], "alloc_xor": ax.tolist(),
                          "visible_xor": vx.tolist(), "ok": [int(x) for x in r["ok"]]},
        }
    out["baseline_ok"] = [int(x) for x in base_ok]
    out["seconds"] = round(time.time() - t0, 1)
    s = json.dumps(out)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            f.write(s + "\n")
    summary = {m: {k: v for k, v in out["modes"][m].items() if k not in ("per_frame", "tsdf_checkpoints")}
               for m in names[1:]}
    print(json.dumps(summary, indent=1))


def one_step(args):
    W, H = 640, 480
    if args.config == "C2":
        cfg = dict(seed=7, voxel=0.005)
        R = np.empty((args.frames, 3, 3)); t = np.empty((args.frames, 3))
        for k in range(args.frames):
            R[k], t[k] = synth.orbit_pose(k)
    else:
        cfg = dict(seed=13, voxel=0.01)
        R, t = synth.random_walk_poses(args.frames, seed=13)
    fx, fy, cx, cy = synth.intrinsics(W, H)
    kw = dict(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy, voxelSize=cfg["voxel"])
    names = args.modes.split(",")
    base = names[0]
    prim = O.Oracle(O.default_params(**kw), omp=True)
    scratch = {m: O.Oracle(O.default_params(**kw), omp=True) for m in names[1:]}
    rec = {m: {"pose_rel": [], "flip": [], "iters": [], "alloc_xor": [], "visible_xor": [], "vox_w": [], "vox_sdf": [],
               "max_sdf": []} for m in names[1:]}
    ok_base = []
    t0 = time.time()
    for k in range(args.frames):
        f = frame_at(cfg, k, W, H, (R, t))
        for m in names[1:]:
            scratch[m].copy_state_from(prim)
        O.set_pose_algebra(*MODES[base])
        ok_a = prim(f)
        ok_base.append(bool(ok_a))
        ha = prim.hash()
        al_a, vi_a = block_keys(ha), block_keys(ha, prim.visible_ids())
        P_a = prim.pose().astype(np.float64)
        it_a = prim.counters()["icp_iterations"]
        for m in names[1:]:
            O.set_pose_algebra(*MODES[m])
            ok_b = scratch[m](f)
            hb = scratch[m].hash()
            r = rec[m]
            P_b = scratch[m].pose().astype(np.float64)
            r["pose_rel"].append(float(np.abs(P_b - P_a).max() / max(np.abs(P_a).max(), 1e-30)))
            r["flip"].append(int(ok_a != ok_b))
            r["iters"].append(int(scratch[m].counters()["icp_iterations"]) - int(it_a))
            r["alloc_xor"].append(int(len(np.setxor1d(al_a, block_keys(hb), assume_unique=True))))
            r["visible_xor"].append(int(len(np.setxor1d(vi_a, block_keys(hb, scratch[m].visible_ids()), assume_unique=True))))
            d = tsdf_diff(prim, scratch[m]) if (args.tsdf_every and k % args.tsdf_every == 0) else None
            r["vox_w"].append(None if d is None else d["voxels_weight_differs"])
            r["vox_sdf"].append(None if d is None else d["voxels_sdf_differs"])
            r["max_sdf"].append(None if d is None else d["max_sdf_diff_lsb"])
        if (k + 1) % 50 == 0:
            print(f"frame {k + 1}/{args.frames} {time.time() - t0:.0f}s " + " ".join(
                f"{m}: pose {max(rec[m]['pose_rel']):.2e} flips {sum(rec[m]['flip'])} alloc_xor_max {max(rec[m]['alloc_xor'])}"
                for m in names[1:]), flush=True)
    out = {"config": args.config, "frames": args.frames, "W": W, "H": H, "voxel_m": cfg["voxel"], "kind": "one-step",
           "is": "before every frame each compared mode's context copies the baseline context's state (scene, render "
                 "state, pose history, ICP maps) and runs that single frame; differences are after that frame",
           "baseline_mode": base, "baseline_resets": int(sum(not x for x in ok_base[1:])), "modes": {}}
    for m in names[1:]:
        r = rec[m]
        pr, ax, vx = np.array(r["pose_rel"]), np.array(r["alloc_xor"]), np.array(r["visible_xor"])
        tracked = np.array([ok_base[k] and k > 0 for k in range(args.frames)])
        vw = [x for x in r["vox_w"] if x is not None]
        vs = [x for x in r["vox_sdf"] if x is not None]
        ms = [x for x in r["max_sdf"] if x is not None]
        out["modes"][m] = {
            "pose_algebra": MODES[m][0], "transcendentals": "glibc" if MODES[m][1] else "portable",
            "max_pose_rel_diff": float(pr.max()), "max_pose_rel_diff_tracked_frames": float(pr[tracked].max()) if tracked.any() else None,
            "pose_rel_diff_p50_p99_tracked": [float(np.percentile(pr[tracked], 50)), float(np.percentile(pr[tracked], 99))] if tracked.any() else None,
            "frames_pose_bits_differ": int((pr > 0).sum()), "frames_pose_rel_diff_over_1e-4": int((pr > 1e-4).sum()),
            "reset_flips": int(sum(r["flip"])), "reset_flip_frames": [k for k in range(args.frames) if r["flip"][k]][:50],
            "frames_iteration_count_differs": int(sum(x != 0 for x in r["iters"])),
            "frames_alloc_differs": int((ax > 0).sum()), "alloc_xor_max": int(ax.max()), "alloc_xor_mean": float(ax.mean()),
            "frames_visible_differs": int((vx > 0).sum()), "visible_xor_max": int(vx.max()), "visible_xor_mean": float(vx.mean()),
            "tsdf_frames_checked": len(vw), "voxels_weight_differs_mean": float(np.mean(vw)) if vw else None,
            "voxels_sdf_differs_mean": float(np.mean(vs)) if vs else None, "max_sdf_diff_lsb": int(max(ms)) if ms else None,
            "per_frame": {"pose_rel": [float(f"{x:.3g}") for x in pr], "alloc_xor": ax.tolist(), "visible_xor": vx.tolist(),
                          "flip": r["flip"]},
        }
    out["seconds"] = round(time.time() - t0, 1)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            f.write(json.dumps(out) + "\n")
    print(json.dumps({m: {k: v for k, v in out["modes"][m].items() if k != "per_frame"} for m in names[1:]}, indent=1))


if __name__ == "__main__":
    main()
