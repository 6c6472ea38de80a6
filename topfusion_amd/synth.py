"""Synthetic depth streams for the benchmark configs.

The reference ships no data (its demo reads E:\\Teddy\\Frames\\%04d.pgm,
apps/demo.cpp:93-97), so every workload is rendered analytically:

* C1  "room corner": back wall z = 1.8 m, floor y = +0.6 m (camera y points
  down), left wall x = -0.8 m; pose = identity; optional 1 mm noise and 1 %
  holes (seed 42).
* C2  orbit: the camera starts at the identity and orbits a pivot 1.2 m ahead
  about the vertical axis at 0.25 deg/frame (~5 mm/frame); room + sphere
  r = 0.3 m (seed 7 + stream index).
* C3  1280x960 with intrinsics x2, same scene.

Depth is uint16 millimetres (the reference's cuda::Depth, types.hpp:62).
"""
import numpy as np

# TopFuParams::default_params intrinsics, topfu.cpp:24
FX, FY, CX, CY = 504.261, 503.905, 352.457, 272.202


def intrinsics(cols=640, rows=480):
    s = cols / 640.0
    return FX * s, FY * s, CX * s, CY * s


def _rot_y(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]], np.float64)


def render_depth(R, t, cols=640, rows=480, sphere=True, noise_mm=0.0, holes=0.0, seed=0, intr=None):
    """Ray-cast the analytic room (+ sphere) from camera pose (R, t) (camera->world).

    Returns uint16 depth in mm (camera-frame z), 0 where nothing is hit."""
    fx, fy, cx, cy = intr if intr is not None else intrinsics(cols, rows)
    u = np.arange(cols, dtype=np.float64)
    v = np.arange(rows, dtype=np.float64)
    uu, vv = np.meshgrid(u, v)
    dc = np.stack([(uu - cx) / fx, (vv - cy) / fy, np.ones_like(uu)], axis=-1)   # z = 1 in camera frame
    dw = dc @ R.T                                                               # world direction
    o = np.asarray(t, np.float64)
    best = np.full((rows, cols), np.inf)
    # planes: (normal axis, offset) -- back wall, far walls, floor, ceiling
    planes = [(2, 1.8), (1, 0.6), (0, -0.8), (0, 1.1), (1, -0.9), (2, -0.6)]
    with np.errstate(divide="ignore", invalid="ignore"):
        for ax, off in planes:
            tt = (off - o[ax]) / dw[..., ax]
            tt = np.where(tt > 1e-6, tt, np.inf)
            best = np.minimum(best, tt)
        if sphere:
            c = np.array([0.15, 0.25, 1.3])
            r = 0.3
            oc = o - c
            b = dw @ oc
            a = np.einsum("ijk,ijk->ij", dw, dw)
            cc = oc @ oc - r * r
            disc = b * b - a * cc
            sq = np.sqrt(np.maximum(disc, 0))
            t0 = (-b - sq) / a
            t0 = np.where((disc >= 0) & (t0 > 1e-6), t0, np.inf)
            best = np.minimum(best, t0)
    z = best  # dc has z = 1 so the ray parameter is the camera-frame depth
    rng = np.random.default_rng(seed)
    mm = z * 1000.0
    if noise_mm > 0:
        mm = mm + rng.normal(0.0, noise_mm, mm.shape)
    mm = np.where(np.isfinite(mm), np.rint(mm), 0)
    mm = np.clip(mm, 0, 65535).astype(np.uint16)
    if holes > 0:
        mm[rng.random(mm.shape) < holes] = 0
    return mm


def room_corner(cols=640, rows=480, noise_mm=1.0, holes=0.01, seed=42):
    """C1: single frame at the identity pose."""
    return render_depth(np.eye(3), np.zeros(3), cols, rows, sphere=False, noise_mm=noise_mm, holes=holes, seed=seed)


def orbit_pose(k, deg_per_frame=0.25, pivot_dist=1.2):
    """Ground-truth camera->world pose of frame k of the C2 orbit."""
    a = np.deg2rad(deg_per_frame * k)
    R = _rot_y(a)
    pivot = np.array([0.0, 0.0, pivot_dist])
    t = pivot - R @ pivot
    return R, t


def orbit_sequence(n, cols=640, rows=480, seed=7, noise_mm=1.0, holes=0.0, deg_per_frame=0.25):
    """C2: n frames of the orbit, uint16 array (n, rows, cols)."""
    out = np.empty((n, rows, cols), np.uint16)
    for k in range(n):
        R, t = orbit_pose(k, deg_per_frame)
        out[k] = render_depth(R, t, cols, rows, sphere=True, noise_mm=noise_mm, holes=holes, seed=seed * 100003 + k)
    return out
