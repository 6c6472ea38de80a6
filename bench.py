#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: fused frames/sec @640x480, 5 mm voxel hash
(ICP + integrate ms/frame reported alongside), on the C2 workload of SURVEY.md §8d.

A "step" is one TopFu::operator() frame (tfusion/src/topfu.cpp:161-330): preprocessing,
3-level projective ICP (19 iterations), hash allocation, TSDF integration, the grey
renderImage raycast, CreateExpectedDepths and the CreateICPMaps raycast.  Frames come from
the synthetic 640x480 orbit sequence (topfusion_amd/synth.py, seed 7 + rank), uploaded
to HBM before the timed region.  One process per GPU; each rank tracks its own
independent stream (replicas, weak scaling) and the per-rank frame counts / times are
combined by RCCL all-reduces (topfusion_amd/replicas.py: librccl through ctypes on the
product's own HIP runtime; no torch in a GPU process).

    python bench.py [--gpus N] [--steps K] [--warmup W]       (N > 1: this process starts N ranks)
    torchrun --nproc-per-node N bench.py --gpus N ...          (each rank started by torchrun)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

# stages that are one kernel launch per frame (persistent ICP), and that kernel's name
KERNEL_OF_STAGE = {"icp": "k_icp_frame",
                   "raycast_icp": "k_raycast_pair (CreateICPMaps castRay<true> + renderImage castRay + grey)",
                   "integrate": "k_integrate"}
SINGLE_KERNEL_STAGES = tuple(KERNEL_OF_STAGE)

# SURVEY.md §8d configs.  C3 raises the capacities past the reference's (2^21 - 1 blocks = 4 GiB
# of voxels, the most the raycasts' 32-bit offsets address; 2^22 buckets, 2^20 excess) -- sized
# for 288 GB of HBM, not for the reference's GPU.  steps are in units of --frames-per-step.
C3_CAPACITY = dict(n_buckets=1 << 22, n_excess=1 << 20, n_blocks=(1 << 21) - 1, vis_capacity=1 << 21,
                   max_render_blocks=1 << 20)
CONFIGS = {
    # C2 / C3 default to the driver's own command (--steps 20 --warmup 5), so the committed line
    # and the driver's time the same 640 frames of the orbit
    "C2": dict(cols=640, rows=480, voxel=0.005, capacity={}, walk=False, steps=20),
    "C3": dict(cols=1280, rows=960, voxel=0.002, capacity=C3_CAPACITY, walk=False, steps=20),
    # C5 hash stress: 10 mm voxels, 50 k-frame random walk (seed 13 + rank, <= 1 cm / 0.5 deg per
    # frame), reference capacities; frames rendered on the GPU (synth.walk_device)
    "C5": dict(cols=640, rows=480, voxel=0.01, capacity={}, walk=True, steps=1563),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps of --frames-per-step frames each (default: C2/C3 20, C5 1563 = 50 k frames)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed warm-up steps (default 5)")
    ap.add_argument("--frames-per-step", type=int, default=None,
                    help="frames per step: one tf_process_frames batch (default 32 = one enqueue group); C5E: one "
                         "tf_scene_fuse_frames batch (default 1000)")
    ap.add_argument("--per-call-frames", type=int, default=256,
                    help="frames of the per-call (one tf_process_frame per frame) rate beside the batched one; 0 = skip")
    ap.add_argument("--config", choices=["C2", "C3", "C3I", "C3R", "C5", "C5E"], default="C2",
                    help="C2: 640x480 orbit, 5 mm (BASELINE configs[1], the headline); "
                         "C3: 1280x960, 2 mm, capacities beyond the reference's (configs[2]); "
                         "C5: 10 mm hash stress, 50 k-frame random walk (configs[4]) through TopFu; "
                         "C5E: the same hash stress at the engine level -- AllocateSceneFromDepth + IntegrateIntoScene at "
                         "the ground-truth poses of an unconfined 50 k-frame walk through a tiled hall, saturating the VBA; "
                         "C3I: IntegrateIntoScene alone over 2^21 - 1 active blocks at C3 geometry (HBM-bound); "
                         "C3R: both raycasts (CreateICPMaps castRay<true> + renderImage castRay + grey) over the same "
                         "2^21 - 1 block scene")
    ap.add_argument("--cols", type=int, default=None)
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--voxel", type=float, default=None)
    ap.add_argument("--swapping", action="store_true",
                    help="a swapping scene (Scene(params, true)): enlarged-frustum visibility, the GlobalCache in HBM, "
                         "blocks out of view evicted / brought back every frame (SURVEY §8f-2; C5 churn)")
    ap.add_argument("--swap-transfer-blocks", type=int, default=0x1000,
                    help="blocks moved per direction per frame (SDF_TRANSFER_BLOCK_NUM, VoxelBlockHash.hpp:27)")
    ap.add_argument("--colour", action="store_true",
                    help="C2 with the colour TSDF: Voxel_s_rgb voxels integrated from a synthetic colour stream "
                         "(depth+colour, TopFu::operator()(depth, image), topfu.hpp:80); GPU-rendered RGB frames")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline sample length")
    ap.add_argument("--no-profile", action="store_true", help="disable the per-stage HIP-event timing")
    ap.add_argument("--profile-every", type=int, default=16,
                    help="timed region: HIP events around the dominant kernel on every N-th frame only "
                         "(an event pair is a few us of dispatch gap; 1 = every frame)")
    ap.add_argument("--breakdown-frames", type=int, default=64, help="frames of the per-stage timing pass")
    ap.add_argument("--pose-algebra", choices=["canonical", "opencv4", "opencv2"], default=None,
                    help="the ICP iterations' det / solve / Rodrigues (tf_set_pose_algebra): the reference's OpenCV "
                         "algebra (cv::determinant, cv::solve DECOMP_SVD, Affine3f), 3.x-4.x or 2.4.9, or canonical (LU "
                         "+ 2 x 2 block Schur + sinc Rodrigues); default: the library's (opencv4; TFUSION_ICP_SOLVE)")
    ap.add_argument("--no-other-algebra", action="store_true",
                    help="skip the canonical-algebra pass reported beside an OpenCV-algebra headline")
    ap.add_argument("--collective", choices=["rccl", "file"], default="rccl",
                    help="N > 1: how the ranks combine their numbers -- RCCL all-reduces (default) or the host-side "
                         "file group (topfusion_amd/replicas.py)")
    ap.add_argument("--standin", action="store_true",
                    help="CPU stand-in workload (tests): each rank runs the oracle over a few 80x60 orbit frames; "
                         "same launcher and line, file collective, no GPU")
    return ap.parse_args()


def stage_bytes(stage, p, nvis, W, H, lanes=None):
    """Algorithmic HBM bytes of ONE launch of a stage's frame-path kernel (plus the
    work the frame path fuses into that kernel's grid), batched path (two-frame lookahead).
      icp:         sum over levels of iters x W_l x H_l x 64 B.
      raycast_icp: k_raycast_pair -- both raycasts (float4 point image + uchar4 grey image out,
                   every visible block read once per raycast, 2064 B each), the fused
                   CreateExpectedDepths fill (the /8 range region written, the binned boxes read
                   once: 2 x 16 B per box), and the lookahead it carries: frame j+1's computeDists
                   (raw 2 B in, 4 B out), pyramid (level 0 in, levels 1-2 out) and points + normals
                   of three levels (32 B per level pixel), frame j+2's bilateral pass (2 B in, 2 B out).
      integrate:   k_integrate<true> -- the visible entries (id + hash entry, 20 B), the depth image,
                   16 B per voxel lane read (those with an update) and per lane written (those that
                   changed), counted on the device (`lanes` = (read, written) per launch; without
                   counts every voxel read and written), plus CreateExpectedDepths' projection in
                   its leading workgroups (entries read again, 24 B record + tiles + offset out,
                   2 x 16 B binned per box)."""
    npx = W * H
    if stage == "raycast_icp":
        rc, rr = (W - 1) // 8 + 1, (H - 1) // 8 + 1
        pre = npx * (2 + 4) + npx * 2 + (npx // 4 + npx // 16) * 2 + (npx + npx // 4 + npx // 16) * 32 + npx * (2 + 2)
        return npx * (16 + 4) + 2 * nvis * (2048 + 16) + rc * rr * 8 + nvis * 32 + pre
    if stage == "integrate":
        ed = nvis * (20 + 24 + 32)
        if lanes is not None:
            return nvis * 20 + npx * 4 + 16 * (lanes[0] + lanes[1]) + ed
        return nvis * (4096 + 20) + npx * 4 + ed           # voxel R+W + entry/id + depth image
    if stage == "grey":
        return npx * (16 + 4) + nvis * (2048 + 16)
    if stage == "icp":
        tot = 0
        for l in range(3):
            tot += p.icp_iter_num[l] * (W >> l) * (H >> l) * 64
        return tot
    return None


def pmc_tracked_bytes(pmc, stage):
    """HBM-side bytes per launch of a stage's kernel on the timed frames' tracked frames
    (profiles/pmc_traffic.json, tools/pmc_frames_summary.py), else the older per-launch figure."""
    e = pmc.get(stage) or {}
    return (e.get("tracked") or {}).get("bytes", e.get("bytes_per_launch"))


def omp_threads():
    """Threads the OpenMP build uses: OMP_NUM_THREADS (16 on the GPU box), else the CPUs this
    process may run on."""
    v = os.environ.get("OMP_NUM_THREADS")
    if v and v.isdigit() and int(v) > 0:
        return int(v)
    return len(os.sched_getaffinity(0))


def cpu_model():
    """Host CPU model name and logical CPU count (report nproc and the model)."""
    name = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return name, os.cpu_count()


def hbm_stream_copy(gib=1.0, reps=10):
    """Measured device-to-device copy bandwidth (read + write bytes / time, HIP events;
    synth/libtfsynth.so) beside the 8 TB/s spec peak the roofline fractions use."""
    from topfusion_amd import synth
    return synth.synth_lib().tfs_copy_gbs(int(gib * (1 << 30)), reps)


def device_sync():
    """hipDeviceSynchronize through the runtime the product library uses."""
    from topfusion_amd import synth
    assert synth.synth_lib().tfs_sync() == 0, "hipDeviceSynchronize"


def cpu_run(frames, params_kw, first, n, omp, start=None):
    """One timed run of the oracle over frames first..first+n-1: from `start`'s state (an oracle
    context that already ran frames 0..first-1, copied in untimed) or from a fresh context;
    returns seconds."""
    from oracle import oracle as O
    o = O.Oracle(O.default_params(**params_kw), omp=omp)
    if start is not None:
        o.copy_state_from(start)
    t0 = time.perf_counter()
    for k in range(first, first + n):
        o(frames[k])
    return time.perf_counter() - t0


def pose_algebra_gap_summary():
    """What the canonical algebra changes against the reference's (OpenCV 4) on the C2 frames, one
    step at a time (both from the same state before every frame): the committed measurement
    tools/pose_algebra_gap.py --one-step made (profiles/r05/pose_algebra_onestep_C2.json)."""
    path = os.path.join(ROOT, "profiles", "r05", "pose_algebra_onestep_C2.json")
    try:
        d = json.load(open(path))["modes"]["opencv4_portable"]
    except Exception:
        return None
    return {"frames": 800, "frames_pose_rel_diff_over_1e-4": d.get("frames_pose_rel_diff_over_1e-4"),
            "pose_rel_diff_p50_p99_tracked": d.get("pose_rel_diff_p50_p99_tracked"),
            "frames_alloc_differs": d.get("frames_alloc_differs"), "alloc_xor_mean": d.get("alloc_xor_mean"),
            "reset_flips": d.get("reset_flips"), "frames_iteration_count_differs": d.get("frames_iteration_count_differs"),
            "source": os.path.relpath(path, ROOT)}


def cpu_baseline_protocol(frames, first, params_kw, seconds, nt, algebra=0):
    """BASELINE.md CPU protocol on the GPU box's host, on the frames the GPU times: the OpenMP
    build (nt threads) runs frames 0..first-1 untimed (the GPU's warm-up frames), and from a
    copy of that state each timed run processes frames first..first+n-1 -- the first n frames of
    the GPU's timed region, with the same scene, pose history and resets.  For the OpenMP build
    and the serial build (from the same state): one warm-up run, then the median of 5 timed runs
    (n sized so the 5 runs take about `seconds` / 2 per build).  Plus C1 (the frame-0
    integrate-only path on frame 0 of a fresh context, median of 5 after a warm-up) as ms/frame."""
    from oracle import oracle as O
    O.set_pose_algebra(algebra)             # the GPU's pose algebra (tf_get_pose_algebra)
    t_w0 = time.perf_counter()
    state = O.Oracle(O.default_params(**params_kw), omp=True)
    for k in range(first):
        state(frames[k])
    t_state = time.perf_counter() - t_w0
    avail = len(frames) - first
    res = {}
    for name, omp in (("omp", True), ("serial", False)):
        t_warm = cpu_run(frames, params_kw, first, 2, omp, state)         # warm-up (also sizes the sample)
        per = max(t_warm / 2, 1e-3)
        n = int(max(3, min(avail, seconds / 2 / 5 / per)))
        runs = sorted(cpu_run(frames, params_kw, first, n, omp, state) for _ in range(5))
        c1 = sorted(cpu_run(frames, params_kw, 0, 1, omp) for _ in range(6))[1:]   # first = warm-up
        res[name] = {"fps": n / runs[2], "n": n, "runs_s": [round(r, 3) for r in runs],
                     "c1_ms": 1000.0 * sorted(c1)[2]}
    o, s1 = res["omp"], res["serial"]
    model, nproc = cpu_model()
    return {"value": round(o["fps"], 4), "unit": "frames/s", "cores": nt, "kind": "port",
            "sample": f"oracle (C restatement, OpenMP build: per-pixel / per-CTA / per-block loops on {nt} threads, "
                      f"allocation serial) on frames {first}..{first + o['n'] - 1} -- the first {o['n']} frames of the "
                      f"GPU's timed region -- from the state after frames 0..{first - 1} (run untimed by the OpenMP "
                      f"build, {t_state:.1f} s); median of 5 runs after 1 warm-up ({o['runs_s']} s); host CPU of the "
                      "GPU box",
            "frames": [first, first + o["n"]],
            "c1_ms_per_frame": round(o["c1_ms"], 3),
            "single_thread": {"value": round(s1["fps"], 4), "cores": 1,
                              "sample": f"serial oracle, frames {first}..{first + s1['n'] - 1} from the same state, "
                                        f"median of 5 runs after 1 warm-up ({s1['runs_s']} s)",
                              "c1_ms_per_frame": round(s1["c1_ms"], 3)},
            "cpu_model": model, "nproc": nproc, "affinity_cpus": len(os.sched_getaffinity(0)),
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "cores_note": ("OMP_NUM_THREADS: the GPU pool gives a one-GPU job a share of the host's CPUs (16 of the "
                           "machine's, which the 8 GPUs' jobs share); nproc / affinity show the whole machine")}


def c3_scene():
    """The C3 HBM-scale scene (~2 M active blocks): 2^21 - 1 voxel blocks
    (4 GiB of voxels) fill the 1280x960 frustum in layers from 0.3 m on (to ~2.8 m), every one in
    the visible list, uploaded as a valid hash table (synth.build_hash) + visible list; dists of a
    wall at 1.5 m.  Returns (context, params, W, H, voxel size, block count, visible ids,
    lastFreeExcessListId)."""
    from topfusion_amd import TopFu, default_params, synth
    from topfusion_amd import _lib as L
    from topfusion_amd.topfu import HASH_DTYPE
    cfg = CONFIGS["C3"]
    W, H, vox = cfg["cols"], cfg["rows"], cfg["voxel"]
    fx, fy, cx, cy = synth.intrinsics(W, H)
    p = default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy, voxelSize=vox, **cfg["capacity"])
    nb = p.n_blocks
    bs = 8 * vox
    blocks, z = [], 0.3
    while sum(len(b) for b in blocks) < nb:                # frustum layers of blocks, near to far
        bz = int(np.floor(z / bs))
        zc = (bz + 0.5) * bs
        x0, x1 = int(np.floor((0 - cx) / fx * zc / bs)), int(np.ceil((W - cx) / fx * zc / bs))
        y0, y1 = int(np.floor((0 - cy) / fy * zc / bs)), int(np.ceil((H - cy) / fy * zc / bs))
        yy, xx = np.meshgrid(np.arange(y0, y1), np.arange(x0, x1), indexing="ij")
        blocks.append(np.stack([xx.ravel(), yy.ravel(), np.full(xx.size, bz)], 1))
        z = (bz + 1) * bs + 1e-6
    pos = np.concatenate(blocks)[:nb]
    tf = TopFu(p, device=0)
    # a valid hash (every block at its bucket or in its bucket's excess chain, as allocation lays
    # them out), so hash walks, the block grid and the oracle all find the same blocks
    h, entry, last_free_excess = synth.build_hash(pos, p.n_buckets, p.n_excess, HASH_DTYPE)
    assert len(h) == tf.nbytes(L.TF_BUF_HASH) // HASH_DTYPE.itemsize
    tf.upload(L.TF_BUF_HASH, h)
    ids = np.zeros(tf.nbytes(L.TF_BUF_VISIBLE_IDS) // 4, np.int32)
    ids[:nb] = entry                                       # visible list: the blocks, near to far
    tf.upload(L.TF_BUF_VISIBLE_IDS, ids)
    tf.set_counters(-1, last_free_excess, nb)
    tf.stage_preprocess(np.full((H, W), 1500, np.uint16))   # dists of a wall at 1.5 m
    return tf, p, W, H, vox, nb, entry, last_free_excess


def _pmc(config, stage):
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            return (json.load(open(pmc_path)).get(config, {}) or {}).get(stage, {}) or {}
        except Exception:
            return {}
    return {}


def c3_integrate(args):
    """C3I ("integrate over the active list is truly HBM-bound"): one
    IntegrateIntoScene pass per step over the c3_scene() blocks against the wall at 1.5 m, all
    passes back to back on the context stream, timed by HIP events.  Algorithmic bytes per
    pass: Nvis x 20 (entry/id) + W x H x 4 (dists) + 16 B per voxel lane read (those with an
    update: a depth and eta >= -mu) and per lane written (those that changed), counted on the
    device; the reference's pass reads and writes every voxel (Nvis x 4096 B), reported beside
    as the reference-equivalent rate."""
    tf, p, W, H, vox, nb = c3_scene()[:6]
    I = np.eye(4, dtype=np.float32)[:3]
    tf.time_stage("integrate", I, 2)                        # warm-up
    tf.reset_totals()
    ms = tf.time_stage("integrate", I, args.steps)
    tot = tf.totals()
    rd, wr = tot["integrate_lanes_read"] / args.steps, tot["integrate_lanes_written"] / args.steps
    b = stage_bytes("integrate", p, nb, W, H, (rd, wr))
    b_ref = nb * (4096 + 20) + W * H * 4
    ach = b / (ms * 1e-3) / 1e9
    pmc = _pmc("C3I", "integrate")
    out = {"metric": f"IntegrateIntoScene passes/sec over {nb} active voxel blocks @{W}x{H}, {vox * 1000:g} mm",
           "value": round(1000.0 / ms, 2), "unit": "passes/s", "n_gpus": 1, "steps": args.steps, "warmup": 2,
           "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f32", "data": "synthetic",
           "config": {"workload": "C3I: k_integrate over 2^21 - 1 blocks filling the frustum from 0.3 m, wall at 1.5 m",
                      "cols": W, "rows": H, "voxel_m": vox, "active_blocks": int(nb), "parallelism": "replicas1"},
           "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(ach / PEAK_HBM_GBS, 5), "traffic": pmc.get("bytes_per_launch"),
                        "kernel": "k_integrate", "algorithmic_bytes_per_launch": int(b), "avg_launch_ms": round(ms, 5),
                        "timing": "HIP events around back-to-back launches on the context stream",
                        "voxel_lanes_read": int(rd), "voxel_lanes_written": int(wr),
                        "voxel_lanes_total": int(nb) * 128,
                        "reference_equivalent_bytes": int(b_ref),
                        "reference_equivalent_GBs": round(b_ref / (ms * 1e-3) / 1e9, 2)}}
    print(json.dumps(out))
    tf.close()


def c3_raycast(args):
    """C3R ("integrate and raycast over the active list"): the c3_scene()
    blocks after 4 integrate passes against the wall at 1.5 m (free space in front of it, the
    surface band at it), the range image at RenderState's initial (0.2 m, 3.0 m); one step = one
    k_raycast_pair launch -- CreateICPMaps' castRay<true> + renderImage's castRay + grey over
    every pixel -- back to back, HIP events.  Algorithmic bytes per launch: W x H x (16 point
    image + 4 grey image) + 2 x B x 2064, B = the blocks the ICP-map raycast reads (its
    castRay<true> visibility marks, counted after the run)."""
    from topfusion_amd import _lib as L
    tf, p, W, H, vox, nb = c3_scene()[:6]
    I = np.eye(4, dtype=np.float32)[:3]
    tf.time_stage("integrate", I, 4)                        # the surface at 1.5 m
    rng = np.empty((H, W, 2), np.float32)
    rng[..., 0], rng[..., 1] = p.viewFrustum_min, p.viewFrustum_max
    tf.upload(L.TF_BUF_RANGE, rng)
    tf.upload(L.TF_BUF_VISIBLE_TYPE, np.zeros(tf.nbytes(L.TF_BUF_VISIBLE_TYPE), np.uint8))
    tf.time_stage("raycast_render", I, 2)                   # warm-up
    ms = tf.time_stage("raycast_render", I, args.steps)
    touched = int((tf.visible_type() > 0).sum())
    ray = tf.raycast_result()
    hit = float((ray[..., 3] > 0).mean())
    b = W * H * (16 + 4) + 2 * touched * (2048 + 16)
    ach = b / (ms * 1e-3) / 1e9
    pmc = _pmc("C3R", "raycast_icp")
    out = {"metric": f"raycast passes/sec (CreateICPMaps + renderImage castRay, grey) over {nb} allocated voxel blocks "
                     f"@{W}x{H}, {vox * 1000:g} mm",
           "value": round(1000.0 / ms, 2), "unit": "passes/s", "n_gpus": 1, "steps": args.steps, "warmup": 2,
           "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f32", "data": "synthetic",
           "config": {"workload": "C3R: k_raycast_pair over 2^21 - 1 blocks filling the frustum 0.3-2.8 m, "
                                  "surface of a wall at 1.5 m, range 0.2-3.0 m",
                      "cols": W, "rows": H, "voxel_m": vox, "allocated_blocks": int(nb),
                      "blocks_read_by_rays": touched, "rays_hit_fraction": round(hit, 4), "parallelism": "replicas1"},
           "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(ach / PEAK_HBM_GBS, 5), "traffic": pmc.get("bytes_per_launch"),
                        "kernel": "k_raycast_pair", "algorithmic_bytes_per_launch": b, "avg_launch_ms": round(ms, 5),
                        "timing": "HIP events around back-to-back launches on the context stream"}}
    print(json.dumps(out))
    tf.close()


def orbit_frames(n, W, H, seed):
    """C2/C3 input: n frames of the synthetic orbit (room + sphere, 0.25 deg per frame
    around a pivot 1.2 m ahead, swinging +-25 deg so the camera stays inside the room for any n;
    1 mm noise), rendered on the GPU straight into HBM (synth.orbit_device: synth/tf_synth.hip,
    bit-identical to synth.render_room) through the HIP runtime the product library uses.
    Returns a synth.DeviceStream."""
    from topfusion_amd import synth
    return synth.orbit_device(n, W, H, seed)


def walk_frames(n, W, H, seed):
    """C5 input: the seed-13 random walk in the room (<= 1 cm / 0.5 deg per frame), on the GPU."""
    from topfusion_amd import synth
    return synth.walk_device(n, W, H, seed)


def per_call_rate(tf, base, frame_bytes, n):
    """TopFu::operator() semantics (demo.cpp:102-105): one tf_process_frame call per frame (each
    returns on its frame's ICP verdict; its last two launches go out with the next call), wall
    clock over n frames including the last frame's whole work."""
    device_sync()
    t0 = time.perf_counter()
    for k in range(n):
        tf(base + k * frame_bytes)
    tf.stats()                 # (the last frame's deferred launches, enqueued and waited for)
    device_sync()
    return n / (time.perf_counter() - t0)


def batched_rate(tf, base, n, F):
    """The same frames through tf_process_frames in F-frame batches (wall clock)."""
    device_sync()
    t0 = time.perf_counter()
    for k0 in range(0, n, F):
        tf.process_frames(base + k0 * tf.W * tf.H * 2, min(F, n - k0))
    device_sync()
    return n / (time.perf_counter() - t0)


def icp_occupancy():
    """The ICP kernel's occupancy / wait / LDS figures from the newest committed PMC summary of it
    (profiles/rNN/pmc_kernel_c2_k_icp_frame.json: tools/gpu_r4_evidence.sh +
    tools/pmc_kernel_summary.py, units in that file's "units"), if present."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_kernel_c2_k_icp_frame.json")))
    if not paths:
        return None
    try:
        d = json.load(open(paths[-1]))
    except Exception:
        return None
    keys = ("waves_per_cu", "wave_lifetime_us", "wait_any_frac", "issue_stall_frac", "valu_issue_frac",
            "lds_insts_per_wave", "lds_bank_conflict_ratio", "lds_util_frac", "l2_hit_rate")
    out = {k: d[k] for k in keys if k in d}
    out["designed"] = "256 workgroups x 8 waves, one workgroup per CU: 8 waves/CU = 2 per SIMD"
    out["units"] = d.get("units")
    out["source"] = os.path.relpath(paths[-1], ROOT)
    return out


def c5e_bench(args):
    """C5E (BASELINE configs[4], SURVEY §8d C5: "capacity saturation and silent allocation failure"):
    the engine-level hash stress.  A 50 k-frame seed-13 walk (<= 1 cm / 0.5 deg per frame) through
    the unbounded tiled hall of synth.render_hall, rendered on the GPU into HBM first; per frame
    computeDists + AllocateSceneFromDepth + IntegrateIntoScene at the ground-truth pose (+ the
    swapping engine with --swapping) through tf_scene_fuse_frames -- no ICP, so no frame-mixing
    resets, and the reference capacities (65 536 blocks, 2^20 buckets, 2^17 excess), so the VBA fills
    and every later frame's new blocks fail silently (SceneReconstructionEngine_host.cu:358-413).
    A step is one tf_scene_fuse_frames batch of F frames; the per-frame records give the allocated
    blocks, the failed requests and (swapping) the evictions / merges of every frame."""
    rank, local_rank, world, rep = rank_setup(args)
    from topfusion_amd import TopFu, default_params, synth
    F = args.frames_per_step or 1000
    steps = args.steps if args.steps is not None else 50
    warm = args.warmup if args.warmup is not None else 1
    W, H = args.cols or 640, args.rows or 480
    vox = args.voxel or 0.01
    seed = 13 + rank
    n = (warm + steps) * F
    t0 = time.perf_counter()
    stream, R, t = synth.hall_device(n, W, H, seed)
    w2c = synth.world_to_camera_rt(R, t)
    t_render = time.perf_counter() - t0
    fx, fy, cx, cy = synth.intrinsics(W, H)
    pkw = dict(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy, voxelSize=vox)
    if args.swapping:
        pkw.update(use_swapping=1, swap_transfer_blocks=args.swap_transfer_blocks)
    tf = TopFu(default_params(**pkw), device=local_rank)
    recs = []
    for k in range(warm):
        recs.append(tf.fuse_frames(stream.frame_ptr(k * F), w2c[k * F:(k + 1) * F]))
    tf.reset_totals()
    device_sync()
    rep.barrier()
    step_s = []
    t0 = time.perf_counter()
    for k in range(warm, warm + steps):
        ts = time.perf_counter()
        recs.append(tf.fuse_frames(stream.frame_ptr(k * F), w2c[k * F:(k + 1) * F]))
        step_s.append(time.perf_counter() - ts)
    device_sync()
    rep.barrier()
    elapsed = time.perf_counter() - t0
    tot = tf.totals()
    rec = np.concatenate(recs)
    timed = rec[warm * F:]
    nb = tf.params().n_blocks
    fails = rec["alloc_failed_type1"].astype(np.int64) + rec["alloc_failed_type2"]
    first_fail = int(np.argmax(fails > 0)) if (fails > 0).any() else None
    # steps whose frames all come after the first failure: the saturated-VBA rate
    sat_steps = [i for i in range(steps) if first_fail is not None and (warm + i) * F >= first_fail]
    sat_s = sum(step_s[i] for i in sat_steps)
    elapsed_max, total_frames, multi = rep.summary(elapsed, steps * F, identity=rank_identity(args, local_rank, rank),
                                                   extra={"frames_failed_alloc": int((fails[warm * F:] > 0).sum())})
    if rank == 0:
        late = timed[-min(len(timed), 10 * F):]
        allocated = nb - 1 - rec["lastFreeBlockId"]
        out = {
            "metric": f"engine-level fused frames/sec (AllocateSceneFromDepth + IntegrateIntoScene) @{W}x{H}, "
                      f"{vox * 1000:g} mm voxel hash, saturating hash stress" + (" (swapping scene)" if args.swapping else ""),
            "value": round(total_frames / elapsed_max, 2), "unit": "frames/s", "n_gpus": world, "steps": steps,
            "warmup": warm, "ms_per_step": round(elapsed_max / steps * 1000.0, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"C5E: seed-{seed} walk through the tiled hall (synth.render_hall), <= 1 cm / 0.5 deg "
                                   f"per frame, unconfined; {W}x{H}, {vox * 1000:g} mm voxels, reference capacities",
                       "step": f"one tf_scene_fuse_frames batch of {F} frames resident in HBM", "frames_per_step": F,
                       "capacity": {"n_blocks": nb, "n_buckets": tf.params().n_buckets, "n_excess": tf.params().n_excess},
                       "swapping": (f"on: <= {args.swap_transfer_blocks} blocks per direction per frame")
                                   if args.swapping else "off", "parallelism": f"replicas{world}"},
            "ms_per_frame": round(elapsed_max / (steps * F) * 1000.0, 5),
            "first_failure_frame": first_fail,
            "saturated_frames_per_sec": round(len(sat_steps) * F / sat_s, 2) if sat_steps else None,
            "saturated_frames": len(sat_steps) * F,
            "allocated_blocks_last": int(allocated[-1]),
            "allocated_blocks_at": {str(k): int(allocated[k]) for k in range(0, n, max(1, n // 10))},
            "lastFreeExcessListId_last": int(rec["lastFreeExcessListId"][-1]),
            "frames_with_failures_timed": int((fails[warm * F:] > 0).sum()),
            "frames_with_failures_last_10_steps_frac": round(float((late["alloc_failed_type1"] + late["alloc_failed_type2"] > 0).mean()), 4),
            "failed_type1_per_frame_timed": round(float(timed["alloc_failed_type1"].mean()), 2),
            "failed_type2_per_frame_timed": round(float(timed["alloc_failed_type2"].mean()), 2),
            "failed_totals_timed": {"type1": int(tot["alloc_failed_type1"]), "type2": int(tot["alloc_failed_type2"])},
            "visible_blocks_mean_timed": round(float(timed["noVisibleEntries"].mean()), 1),
            "swapped_out_per_frame": round(float(timed["swapped_out"].mean()), 2) if args.swapping else None,
            "swapped_in_merged_per_frame": round(float(timed["swapped_in_merged"].mean()), 2) if args.swapping else None,
            "swap_realloc_per_frame": round(float(timed["swap_realloc"].mean()), 2) if args.swapping else None,
            "render_s": round(t_render, 2),
            "multi_gpu": multi if world > 1 else None,
        }
        print(json.dumps(out))
        check_distinct_devices(multi if world > 1 else None)
    tf.close()
    stream.free()
    rep.close()


def rank_setup(args):
    """This process's rank, local rank and world (torchrun's or replicas.launch's environment), the
    product library on device LOCAL_RANK, and the ranks' collective (topfusion_amd/replicas.py).
    Exits non-zero when the world differs from --gpus or the node has too few devices."""
    from topfusion_amd import replicas
    rank, local_rank, world = replicas.world_from_env()
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launch has WORLD_SIZE {world}")
    if not args.standin:
        from topfusion_amd import _lib as L
        lib = L.load()
        n_dev = L.device_count()
        if os.environ.get("TFUSION_RANK_DEVICE_MODULO") == "1" and n_dev > 0:
            local_rank %= n_dev          # tests only: several ranks on a one-GPU box
        if local_rank >= n_dev:
            sys.exit(f"bench.py: rank {rank} needs HIP device {local_rank}, the node has {n_dev}")
        L.check(lib.tf_set_device(local_rank), "tf_set_device")
    rep = replicas.Replicas(rank, local_rank, world, kind="file" if args.standin else args.collective)
    return rank, local_rank, world, rep


def rank_identity(args, local_rank, rank):
    """This rank's device (PCI bus id) for the multi-GPU fields; the stand-in's placeholder."""
    from topfusion_amd import replicas
    if args.standin:      # (TFUSION_STANDIN_SAME_DEVICE=1, tests: every rank claims one device)
        return replicas.device_identity(0 if os.environ.get("TFUSION_STANDIN_SAME_DEVICE") == "1" else rank, standin=True)
    return replicas.device_identity(local_rank)


def check_distinct_devices(multi):
    """An N-GPU line must come from N distinct devices: exit non-zero (after the line is printed)
    when two ranks report the same bus id, unless the tests' several-ranks-per-device mode
    (TFUSION_RANK_DEVICE_MODULO=1) asked for exactly that."""
    if multi and not multi.get("distinct_devices", True) and os.environ.get("TFUSION_RANK_DEVICE_MODULO") != "1":
        sys.stdout.flush()
        sys.exit(f"bench.py: two ranks ran on the same device: {multi.get('per_rank_device')}")


def standin(args):
    """CPU stand-in for the launcher tests: each rank runs the oracle (test infrastructure; never a
    measured GPU number) over a few frames of its own 80x60 orbit stream (seed 7 + rank), then
    the ranks combine their numbers exactly as the GPU path does, over the file collective."""
    rank, local_rank, world, rep = rank_setup(args)
    from oracle import oracle as O
    from topfusion_amd import synth
    W, H, n = 80, 60, max(1, args.steps or 2)
    fx, fy, cx, cy = synth.intrinsics(W, H)
    frames = synth.orbit_sequence(n, W, H, seed=7 + rank)
    o = O.Oracle(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy)
    rep.barrier()
    t0 = time.perf_counter()
    ok = sum(bool(o(f)) for f in frames)
    rep.barrier()
    elapsed = time.perf_counter() - t0
    emax, total, multi = rep.summary(elapsed, n, identity=rank_identity(args, local_rank, rank),
                                     extra={"frames_ok": ok})
    if rank == 0:
        print(json.dumps({"metric": "stand-in: oracle frames/sec @80x60 (launcher test, not a GPU number)",
                          "value": round(total / emax, 4), "unit": "frames/s", "n_gpus": world, "steps": n,
                          "warmup": 0, "ms_per_step": round(emax / n * 1000, 4), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
                          "config": {"workload": "standin", "parallelism": f"replicas{world}"},
                          "frames_ok_rank0": ok, "frame_sum_rank0": int(frames.astype(np.int64).sum()),
                          "multi_gpu": multi}))
        check_distinct_devices(multi)
    rep.close()


def main():
    args = parse()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and args.config in ("C3I", "C3R"):
        sys.exit(f"bench.py: --config {args.config} times one stage on one GPU; run it with --gpus 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one fresh process per GPU, started before anything here touches a GPU
        from topfusion_amd import replicas
        sys.exit(replicas.launch(os.path.abspath(__file__), sys.argv[1:], args.gpus))
    if args.standin:
        return standin(args)
    if args.pose_algebra is not None:            # every context this process creates (tf_create reads it)
        os.environ["TFUSION_ICP_SOLVE"] = args.pose_algebra
    if args.config == "C5E":
        return c5e_bench(args)
    if args.config == "C3I":
        if args.steps is None:
            args.steps = 20
        return c3_integrate(args)
    if args.config == "C3R":
        if args.steps is None:
            args.steps = 20
        return c3_raycast(args)
    rank, local_rank, world, rep = rank_setup(args)
    from topfusion_amd import TopFu, default_params, synth

    cfg = CONFIGS[args.config]
    if args.steps is None:
        args.steps = cfg["steps"]
    if args.warmup is None:
        args.warmup = 5
    W = args.cols or cfg["cols"]
    H = args.rows or cfg["rows"]
    if args.voxel is None:
        args.voxel = cfg["voxel"]
    F = args.frames_per_step or 32
    fx, fy, cx, cy = synth.intrinsics(W, H)
    pkw = dict(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy, voxelSize=args.voxel, **cfg["capacity"])
    if args.swapping:
        pkw.update(use_swapping=1, swap_transfer_blocks=args.swap_transfer_blocks)
    if args.colour:
        pkw.update(voxel_rgb=1)            # rgb_intr 0 / depth_to_rgb 0: the colour camera registered with the depth one
    n_breakdown = 0 if args.no_profile else min(args.breakdown_frames, args.steps * F)
    n_frames = (args.warmup + args.steps) * F
    seed = (13 if cfg["walk"] else 7) + rank
    dev = (walk_frames if cfg["walk"] else orbit_frames)(n_frames, W, H, seed)
    frame_bytes = W * H * 2
    base = dev.ptr
    rgb = synth.orbit_colour_device(n_frames, W, H) if args.colour else None
    rgb_bytes = W * H * 4

    def run(tfx, k0, n):
        """frames k0..k0+n-1 of the stream as one tf_process_frames(_rgb) batch"""
        if rgb is None:
            return tfx.process_frames(base + k0 * frame_bytes, n)
        return tfx.process_frames(base + k0 * frame_bytes, n, rgb_frames=rgb.ptr + k0 * rgb_bytes, rgb_stride=rgb_bytes)

    # per-stage breakdown first (outside the timed region, a context of its own): a fresh context
    # replays the warm-up and the first frames of the timed region with every stage timed; the
    # dominant single-kernel stage -- by measured time per full launch -- is the one the timed
    # region times and the roofline names
    prof = {}
    lanes_bd = nvis_bd = None
    tb = TopFu(default_params(**pkw), device=local_rank)
    single = [k for k in SINGLE_KERNEL_STAGES if k != "icp" or tb.icp_persistent()]
    dominant = "icp" if tb.icp_persistent() else "raycast_icp"
    if n_breakdown:
        run(tb, 0, args.warmup * F)
        tb.profile(True)
        tb.reset_totals()
        run(tb, args.warmup * F, n_breakdown)
        prof = tb.profile_read()
        tbt = tb.totals()
        n_int = max(1, tbt["frames"] - tbt["resets"])
        lanes_bd = (tbt["integrate_lanes_read"] / n_int, tbt["integrate_lanes_written"] / n_int)
        nvis_bd = tbt["visible_sum"] / n_int
        avg = {k: prof[k][0] / prof[k][1] for k in single if prof[k][1]}
        if avg:
            dominant = max(avg, key=avg.get)
    tb.close()
    device_sync()

    tf = TopFu(default_params(**pkw), device=local_rank)
    device_sync()
    for w in range(args.warmup):                      # warm-up: whole steps (full enqueue groups)
        run(tf, w * F, F)
    # timed region: HIP events only around the dominant kernel's stage, on every
    # --profile-every-th frame (an event pair costs a few us of dispatch gap)
    tf.profile(not args.no_profile, stages=[dominant], every=args.profile_every)
    tf.reset_totals()
    device_sync()
    rep.barrier()
    t0 = time.perf_counter()
    oks = []
    for k in range(args.steps):
        oks.append(run(tf, (args.warmup + k) * F, F))
    device_sync()
    rep.barrier()
    elapsed = time.perf_counter() - t0
    ok = np.concatenate(oks)
    prof_timed = tf.profile_read() if not args.no_profile else {}
    tot = tf.totals()
    st = tf.stats()
    # the timed context closes here: the measurements below each run a context of their own, and
    # with two contexts on a device every persistent ICP launch is ordered after the other
    # context's by a stream event (tf_capi.hip icp_order_*), a dispatch gap no single user sees
    tf_params, tf_alg, tf_persistent = tf.params(), tf.pose_algebra(), tf.icp_persistent()
    tf.close()

    # the other algebra beside the headline one: the same frames, warm-up and timed steps through
    # a fresh context under the canonical algebra (when the headline ran the reference's) -- wall
    # clock, and the ICP's full launches timed as in the timed region
    other = None
    if rgb is None and tf_alg != 0 and not args.no_other_algebra:
        tc = TopFu(default_params(**pkw), device=local_rank)
        tc.set_pose_algebra("canonical")
        device_sync()
        for w in range(args.warmup):
            run(tc, w * F, F)
        tc.profile(not args.no_profile, stages=["icp"], every=args.profile_every)
        tc.reset_totals()
        device_sync()
        tcs = time.perf_counter()
        okc = np.concatenate([run(tc, (args.warmup + k) * F, F) for k in range(args.steps)])
        device_sync()
        el_c = time.perf_counter() - tcs
        pc = tc.profile_read() if not args.no_profile else {}
        totc = tc.totals()
        tc.close()
        other = {"pose_algebra": "canonical", "frames_per_sec": round(args.steps * F / el_c, 2),
                 "icp_ms_full_launch": round(pc["icp"][0] / pc["icp"][1], 5) if pc and pc["icp"][1] else None,
                 "frames_ok": int(okc.sum()), "resets": int(totc["resets"]),
                 "is": "the same frames, warm-up and timed steps on one GPU through a fresh context under the "
                       "canonical algebra (LU + 2 x 2 block Schur solve + sinc Rodrigues; not the reference's "
                       "arithmetic: its trajectory and allocated blocks differ from the reference's)",
                 "one_step_gap": pose_algebra_gap_summary()}

    # TopFu::operator() per call (one call per frame, returning on the frame's verdict) over the first
    # frames of the timed region, from a fresh context, and the batched rate of a fresh context on
    # the same frames beside it (the orbit's cost per frame varies along it: compare like with like)
    per_call = per_call_batched = None
    nc = min(args.per_call_frames, args.steps * F) if rgb is None else 0   # (colour: RGB frames wait for the whole frame)
    if nc > 0:
        pc_base = base + args.warmup * F * frame_bytes
        tc = TopFu(default_params(**pkw), device=local_rank)
        per_call = per_call_rate(tc, pc_base, frame_bytes, nc)
        tc.close()
        tc = TopFu(default_params(**pkw), device=local_rank)
        per_call_batched = batched_rate(tc, pc_base, nc, F)
        tc.close()

    # C1 (BASELINE configs[0]): the frame-0 path -- computeDists + preprocessing,
    # AllocateSceneFromDepth and IntegrateIntoScene of the first frame, no ICP (topfu.cpp:200-207) --
    # on a fresh context each time: wall time of the call (host sync included), median of 5 after a
    # warm-up, beside the CPU baseline's c1_ms_per_frame on the same frame
    c1_gpu = None
    if rgb is None:
        c1 = []
        for _ in range(6):
            t1 = TopFu(default_params(**pkw), device=local_rank)
            device_sync()
            ts = time.perf_counter()
            run(t1, 0, 1)
            c1.append(time.perf_counter() - ts)
            t1.close()
        c1_gpu = 1000.0 * sorted(c1[1:])[2]
    total_steps_frames = args.steps * F
    elapsed_max, total_frames, multi = rep.summary(
        elapsed, total_steps_frames, identity=rank_identity(args, local_rank, rank),
        extra={"frames_ok": int(ok.sum()), "icp_fallbacks": int(tot["icp_fallbacks"]), "resets": int(tot["resets"])})

    if rank == 0:
        value = total_frames / elapsed_max
        ms_per_step = elapsed_max / args.steps * 1000.0
        per_stage = {k: (v[0] / v[1] if v[1] else None) for k, v in prof.items()}
        timed_ms = None
        if prof_timed and prof_timed[dominant][1]:
            timed_ms = prof_timed[dominant][0] / prof_timed[dominant][1]
        icp_integ = None
        if prof and prof["icp"][1]:
            icp_integ = per_stage["icp"] + per_stage["alloc"] + per_stage["integrate"]
        integrated = max(1, tot["frames"] - tot["resets"])
        nvis_mean = tot["visible_sum"] / integrated
        # roofline of the dominant single-kernel stage (by measured time); every single-kernel
        # stage is also reported under roofline_stages, with the mean visible-block count of the
        # timed frames
        roof, roof_all = None, {}
        if prof or prof_timed:
            pmc = {}
            pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc_path):
                try:
                    pmc = json.load(open(pmc_path)).get(args.config, {})
                except Exception:
                    pmc = {}
            for k in single:
                ms = timed_ms if (k == dominant and timed_ms) else per_stage.get(k)
                if not ms:
                    continue
                if k == "integrate" and lanes_bd is not None:    # lanes counted in the breakdown pass
                    b = stage_bytes(k, tf_params, nvis_bd, W, H, lanes_bd)
                else:
                    b = stage_bytes(k, tf_params, nvis_mean, W, H)
                ach = b / (ms * 1e-3) / 1e9
                roof_all[k] = {"bound": "hbm", "achieved": round(ach, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                               "frac": round(ach / PEAK_HBM_GBS, 5),
                               "traffic": pmc_tracked_bytes(pmc, k),
                               "kernel": KERNEL_OF_STAGE[k], "algorithmic_bytes_per_launch": int(b),
                               "avg_launch_ms": round(ms, 5),
                               "timing": (f"HIP events tied to the dispatch of every {args.profile_every}-th launch of the "
                                          f"timed region (hipExtLaunchKernelGGL; {prof_timed[k][1]} launches that ran the "
                                          "whole stage)") if (k == dominant and timed_ms)
                                         else "HIP events tied to each launch's dispatch in the breakdown pass"}
            if dominant in roof_all:
                roof = roof_all[dominant]
            occ = icp_occupancy()
            if occ and "icp" in roof_all:
                roof_all["icp"]["occupancy"] = occ
            if "icp" in roof_all:
                roof_all["icp"]["limit"] = ("latency, not HBM: 19 dependent iterations, each rows -> two cross-CU "
                                            "hand-offs -> the 6x6 solve on one wave (the reference's algebra: the "
                                            "lane-parallel Jacobi SVD, ~20 k cycles; DESIGN.md 5); the previous-frame "
                                            "gathers hit L2, so PMC traffic is a fraction of the algorithmic bytes")
        stream_gbs = round(hbm_stream_copy(), 1)
        cpu = None
        if not args.no_cpu_baseline and world == 1:        # (rank 0 at N = 1 only)
            # all cores: the OpenMP build of the oracle; 1 thread: the serial build (reported
            # beside); BASELINE.md protocol: one warm-up frame, then the median of 5 repeats of a
            # bounded sample of the same stream
            first = args.warmup * F
            frames = dev.download(0, min(n_frames, first + 128))
            nt = omp_threads()
            cpu = cpu_baseline_protocol(frames, first, pkw, args.cpu_seconds, nt, tf_alg)
        out = {
            "metric": f"fused frames/sec @{W}x{H}, {args.voxel * 1000:g} mm voxel hash; ICP+integrate ms/frame"
                      + (" (swapping scene)" if args.swapping else "")
                      + (" (depth+colour stream, Voxel_s_rgb)" if args.colour else ""),
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"{args.config} {'random walk' if cfg['walk'] else 'orbit'}, {W}x{H}, "
                                   f"{args.voxel * 1000:g} mm voxels, 8^3 blocks, "
                                   "3-level ICP (10/5/4) + alloc + integrate + renderImage + expected depths + "
                                   "ICP-map raycast; one independent stream per GPU",
                       "step": f"one tf_process_frames batch of {F} consecutive frames (one enqueue group), "
                               f"frames resident in HBM",
                       "frames_per_step": F,
                       "cols": W, "rows": H, "voxel_m": args.voxel, "parallelism": f"replicas{world}",
                       "capacity": cfg["capacity"] or "reference defaults",
                       "swapping": (f"on: GlobalCache in HBM, <= {args.swap_transfer_blocks} blocks per direction "
                                    "per frame") if args.swapping else "off (topfu.cpp:67)"},
            "ms_per_frame": round(elapsed_max / total_steps_frames * 1000.0, 5),
            "c1": None if c1_gpu is None else {
                "gpu_ms_per_frame": round(c1_gpu, 4),
                "cpu_ms_per_frame": cpu["c1_ms_per_frame"] if cpu else None,
                "cpu_single_thread_ms_per_frame": cpu["single_thread"]["c1_ms_per_frame"] if cpu else None,
                "is": "BASELINE configs[0]: the frame-0 path (preprocessing + AllocateSceneFromDepth + IntegrateIntoScene, "
                      "no ICP; topfu.cpp:200-207) of the stream's first frame on a fresh context; GPU: wall time of the "
                      "call with its host sync, median of 5 after a warm-up; CPU: the oracle on the same frame"},
            "colour": ("on: Voxel_s_rgb, the colour camera registered with the depth one, GPU-rendered colour stream "
                       "(synth/tf_synth.hip k_render_room_rgb); computeUpdatedVoxelColorInfo in every integration") if args.colour else None,
            "per_call_frames_per_sec": None if per_call is None else round(per_call, 2),
            "per_call_batched_same_frames": None if per_call_batched is None else round(per_call_batched, 2),
            "per_call": (f"TopFu::operator() per call: tf_process_frame on the timed region's first {nc} frames from a "
                         "fresh context, one call per frame (demo.cpp:102-105 semantics: each returns on its frame's ICP verdict, its "
                         "last two launches go out with the next call, carrying that frame's preprocessing; the time ends after "
                         "the last frame's whole work); "
                         "per_call_batched_same_frames: tf_process_frames on the same frames from a fresh context")
                        if per_call is not None else None,
            "icp_integrate_ms_per_frame": None if icp_integ is None else round(icp_integ, 4),
            "stage_ms_per_frame": {k: (None if v is None else round(v, 4)) for k, v in per_stage.items()},
            "stage_breakdown": (f"separate replay of the timed region's first {n_breakdown} frames in a fresh context, "
                                f"every stage timed (HIP events; averages per executed launch)") if n_breakdown else None,
            "frames_ok": int(ok.sum()), "resets": int(tot["resets"]),
            "ok_frames_per_sec": round(int(ok.sum()) * (total_frames / total_steps_frames) / elapsed_max, 2),
            "visible_blocks_mean": round(nvis_mean, 1),
            "visible_blocks_mean_is": "visible-list length per frame that integrated (tracked frames and frame-0 "
                                      "frames after a reset), timed region",
            "workload_check": None if cfg["walk"] else {
                "camera_inside_room": "every generated frame (asserted in orbit_frames, >= 0.2 m from every wall)",
                "orbit_deg_timed": [round(min(synth.orbit_angle_deg(k) for k in range(args.warmup * F, n_frames)), 2),
                                    round(max(synth.orbit_angle_deg(k) for k in range(args.warmup * F, n_frames)), 2)],
                "timed_frames": [args.warmup * F, n_frames]},
            "render_tiles_mean": round(tot["tiles_sum"] / max(1, tot["frames_tracked"]), 1),
            "visible_blocks_last": st["noVisibleEntries"],
            "allocated_blocks_last": int(tf_params.n_blocks - 1 - st["lastFreeBlockId"]),
            "last_frame_ok": bool(ok[-1]),
            "swapped_out_per_frame": round(tot["swapped_out"] / max(1, tot["frames"]), 2) if args.swapping else None,
            "swapped_in_merged_per_frame": round(tot["swapped_in_merged"] / max(1, tot["frames"]), 2) if args.swapping else None,
            "swap_state_1to2_per_frame": round(tot["swapped_in"] / max(1, tot["frames"]), 2) if args.swapping else None,
            "swap_counts_are": ("swapped_out: blocks copied VBA -> GlobalCache and freed; swapped_in_merged: GlobalCache "
                                "-> VBA merges of stored blocks; swap_state_1to2: IntegrateGlobalIntoLocal state "
                                "transitions, most of them new blocks with nothing stored") if args.swapping else None,
            "roofline": roof,
            "hbm_stream_copy_GBs": stream_gbs,
            "roofline_stages": roof_all,
            "icp_schedule": "persistent" if tf_persistent else "per_iteration",
            "pose_algebra": {0: "canonical", 2: "opencv2", 4: "opencv4"}[tf_alg],
            "pose_algebra_is": ("the reference's own (cv::determinant, cv::solve DECOMP_SVD, Affine3f as OpenCV "
                                "3.x-4.x / 2.4.9 publish them; projective_icp.cpp:197-209), bit-exact against the oracle's "
                                "restatement") if tf_alg else "canonical (not the reference's arithmetic)",
            "other_algebra": other,
            "icp_fallbacks": int(tot["icp_fallbacks"]),
            "cpu_baseline": cpu,
            "multi_gpu": multi if world > 1 else None,
        }
        print(json.dumps(out))
        check_distinct_devices(multi if world > 1 else None)
    dev.free()
    if rgb is not None:
        rgb.free()
    rep.close()


if __name__ == "__main__":
    main()
