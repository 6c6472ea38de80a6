"""Synthetic depth streams for the benchmark configs.

The reference ships no data (its demo reads E:\\Teddy\\Frames\\%04d.pgm,
apps/demo.cpp:93-97), so every workload is rendered analytically:

* C1  "room corner": back wall z = 1.8 m, floor y = +0.6 m (camera y points
  down), left wall x = -0.8 m; pose = identity; optional 1 mm noise and 1 %
  holes (seed 42).
* C2  orbit: the camera starts at the identity and orbits a pivot 1.2 m ahead
  about the vertical axis at 0.25 deg/frame (~5 mm/frame), swinging +-25 deg so it
  stays inside the room for any stream length; room + sphere r = 0.3 m (seed 7 +
  stream index).
* C3  1280x960 with intrinsics x2, same scene.

Depth is uint16 millimetres (the reference's cuda::Depth, types.hpp:62).
"""
import os

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


def render_colour(R, t, cols=640, rows=480, sphere=True, intr=None):
    """The colour camera's view of the same room (pose R, t camera->world): a smooth texture of the
    surface point hit by each pixel's ray, uint8 (rows, cols, 4), alpha 255, black where nothing is
    hit -- the RGB stream for the colour TSDF (Voxel_s_rgb)."""
    fx, fy, cx, cy = intr if intr is not None else intrinsics(cols, rows)
    u = np.arange(cols, dtype=np.float64)
    v = np.arange(rows, dtype=np.float64)
    uu, vv = np.meshgrid(u, v)
    dc = np.stack([(uu - cx) / fx, (vv - cy) / fy, np.ones_like(uu)], axis=-1)
    dw = dc @ np.asarray(R, np.float64).T
    o = np.asarray(t, np.float64)
    best = np.full((rows, cols), np.inf)
    planes = [(2, 1.8), (1, 0.6), (0, -0.8), (0, 1.1), (1, -0.9), (2, -0.6)]
    with np.errstate(divide="ignore", invalid="ignore"):
        for ax, off in planes:
            tt = (off - o[ax]) / dw[..., ax]
            best = np.minimum(best, np.where(tt > 1e-6, tt, np.inf))
        if sphere:
            c = np.array([0.15, 0.25, 1.3])
            oc = o - c
            b = dw @ oc
            a = np.einsum("ijk,ijk->ij", dw, dw)
            disc = b * b - a * (oc @ oc - 0.09)
            t0 = (-b - np.sqrt(np.maximum(disc, 0))) / a
            best = np.minimum(best, np.where((disc >= 0) & (t0 > 1e-6), t0, np.inf))
    hit = np.isfinite(best)
    p = o + dw * np.where(hit, best, 0)[..., None]
    out = np.zeros((rows, cols, 4), np.uint8)
    out[..., 0] = np.rint(127.5 + 120 * np.sin(2 * np.pi * p[..., 0] / 0.13))
    out[..., 1] = np.rint(127.5 + 120 * np.sin(2 * np.pi * (p[..., 1] + p[..., 2]) / 0.17))
    out[..., 2] = np.rint(127.5 + 120 * np.cos(2 * np.pi * (p[..., 2] - p[..., 0]) / 0.23))
    out[..., 3] = 255
    out[~hit] = 0
    return out


def room_corner(cols=640, rows=480, noise_mm=1.0, holes=0.01, seed=42):
    """C1: single frame at the identity pose."""
    return render_depth(np.eye(3), np.zeros(3), cols, rows, sphere=False, noise_mm=noise_mm, holes=holes, seed=seed)


ORBIT_AMPLITUDE_DEG = 25.0
# the walls of render_depth's room (x, y, z extents); the sphere sits inside
ROOM_WALLS_LO = np.array([-0.8, -0.9, -0.6])
ROOM_WALLS_HI = np.array([1.1, 0.6, 1.8])


def orbit_angle_deg(k, deg_per_frame=0.25, amplitude_deg=ORBIT_AMPLITUDE_DEG):
    """Orbit angle of frame k: a ping-pong (triangle wave) at deg_per_frame between
    -amplitude and +amplitude, starting at 0 and swinging to +amplitude first.  The first
    amplitude/deg_per_frame frames equal a plain orbit, and the camera never
    leaves the room however long the stream is (a plain orbit at 0.25 deg/frame crosses the
    left wall at 42 deg, frame 168).  amplitude_deg=None gives the plain, unbounded orbit."""
    if amplitude_deg is None:
        return deg_per_frame * k
    a = deg_per_frame * k
    period = 4.0 * amplitude_deg
    ph = a % period
    if ph <= amplitude_deg:
        return ph
    if ph <= 3.0 * amplitude_deg:
        return 2.0 * amplitude_deg - ph
    return ph - period


def orbit_pose(k, deg_per_frame=0.25, pivot_dist=1.2, amplitude_deg=ORBIT_AMPLITUDE_DEG):
    """Ground-truth camera->world pose of frame k of the C2 orbit: a rotation about the vertical
    axis through a pivot pivot_dist ahead of the start (0.25 deg ~ 5 mm per frame), swinging
    +-amplitude_deg (orbit_angle_deg).  With the defaults the camera centre stays >= 0.29 m
    inside every wall (orbit_in_room)."""
    a = np.deg2rad(orbit_angle_deg(k, deg_per_frame, amplitude_deg))
    R = _rot_y(a)
    pivot = np.array([0.0, 0.0, pivot_dist])
    t = pivot - R @ pivot
    return R, t


def orbit_in_room(R, t, margin=0.2):
    """True if the camera centre t lies inside the room's walls with `margin` metres to spare."""
    t = np.asarray(t, np.float64)
    return bool(np.all(t > ROOM_WALLS_LO + margin) and np.all(t < ROOM_WALLS_HI - margin))


def orbit_sequence(n, cols=640, rows=480, seed=7, noise_mm=1.0, holes=0.0, deg_per_frame=0.25):
    """C2: n frames of the orbit, uint16 array (n, rows, cols)."""
    out = np.empty((n, rows, cols), np.uint16)
    for k in range(n):
        R, t = orbit_pose(k, deg_per_frame)
        assert orbit_in_room(R, t), f"orbit frame {k}: camera outside the room"
        out[k] = render_depth(R, t, cols, rows, sphere=True, noise_mm=noise_mm, holes=holes, seed=seed * 100003 + k)
    return out


# ----------------------------------------------------------------------------------------
# C5: hash stress -- 10 mm voxels, random-walk trajectory (seed 13, steps
# <= 1 cm / 0.5 deg).  The walk stays inside the room box (reflected at its faces) so every
# ray hits a surface within the view frustum.
# ----------------------------------------------------------------------------------------
ROOM_LO = np.array([-0.55, -0.65, -0.35])     # camera-centre box inside the room (walls at
ROOM_HI = np.array([0.85, 0.35, 0.8])         # x -0.8/1.1, y -0.9/0.6, z -0.6/1.8; sphere kept clear)


def _axis_angle(axis, ang):
    axis = axis / np.linalg.norm(axis)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * (K @ K)


def random_walk_poses(n, seed=13, step_m=0.01, step_deg=0.5):
    """Camera->world poses (R[n,3,3], t[n,3]) of the C5 random walk: frame 0 at the identity,
    then per frame a translation of length <= step_m in a uniformly random direction and a
    rotation of angle <= step_deg about a uniformly random axis (float64)."""
    rng = np.random.default_rng(seed)
    R = np.empty((n, 3, 3))
    t = np.empty((n, 3))
    Rc, tc = np.eye(3), np.zeros(3)
    for k in range(n):
        R[k], t[k] = Rc, tc
        d = rng.normal(size=3)
        tc = tc + d / np.linalg.norm(d) * step_m * rng.random()
        tc = np.where(tc < ROOM_LO, 2 * ROOM_LO - tc, tc)          # reflect at the box faces
        tc = np.where(tc > ROOM_HI, 2 * ROOM_HI - tc, tc)
        Rc = _axis_angle(rng.normal(size=3), np.deg2rad(step_deg) * rng.random()) @ Rc
    return R, t


def random_walk_sequence(n, cols=640, rows=480, seed=13, noise_mm=1.0, step_m=0.01, step_deg=0.5):
    """C5 frames on the host (numpy renderer, for the parity tests), uint16 (n, rows, cols)."""
    R, t = random_walk_poses(n, seed, step_m, step_deg)
    out = np.empty((n, rows, cols), np.uint16)
    for k in range(n):
        out[k] = render_depth(R[k], t[k], cols, rows, sphere=True, noise_mm=noise_mm, seed=seed * 100003 + k)
    return out


# ----------------------------------------------------------------------------------------
# A voxel-block hash built directly from a list of block positions (the C3 HBM-scale scene)
# ----------------------------------------------------------------------------------------
def hash_index(x, y, z, n_buckets):
    """hashIndex (VoxelBlockHash.hpp / tf_internal.h): ((x*73856093) ^ (y*19349669) ^
    (z*83492791)) & (n_buckets - 1) in uint32 arithmetic, vectorised."""
    x = np.asarray(x).astype(np.int64).astype(np.uint32)
    y = np.asarray(y).astype(np.int64).astype(np.uint32)
    z = np.asarray(z).astype(np.int64).astype(np.uint32)
    with np.errstate(over="ignore"):
        h = (x * np.uint32(73856093)) ^ (y * np.uint32(19349669)) ^ (z * np.uint32(83492791))
    return (h & np.uint32(n_buckets - 1)).astype(np.int64)


def build_hash(pos, n_buckets, n_excess, dtype):
    """A valid hash table holding the blocks `pos` (int (n, 3)), as the reference's allocation
    would lay them out (SceneReconstructionEngine_host.cu allocateVoxelBlocksList): the first
    block of a bucket in the bucket entry, the others in excess entries taken from the top of
    the excess free list (excessList[lastFreeExcessListId--]) and chained through `offset`
    (excess id + 1); block i gets VBA block ptr i.  Returns (hash, entry index of each block,
    lastFreeExcessListId)."""
    pos = np.asarray(pos, np.int64)
    n = len(pos)
    hidx = hash_index(pos[:, 0], pos[:, 1], pos[:, 2], n_buckets)
    order = np.lexsort((np.arange(n), hidx))            # by bucket, then by block index
    hs = hidx[order]
    first = np.ones(n, bool)
    first[1:] = hs[1:] != hs[:-1]
    n_ex = int((~first).sum())
    if n_ex > n_excess:
        raise ValueError(f"{n_ex} colliding blocks exceed the {n_excess}-entry excess list")
    ex_id = np.full(n, -1, np.int64)
    ex_id[~first] = n_excess - 1 - np.arange(n_ex)
    entry_sorted = np.where(first, hs, n_buckets + ex_id)
    # offset of each entry: the next block of the same bucket's excess id + 1, else 0
    nxt = np.zeros(n, np.int64)
    same_next = np.zeros(n, bool)
    same_next[:-1] = ~first[1:]
    nxt[:-1] = ex_id[1:] + 1
    offset_sorted = np.where(same_next, nxt, 0)
    h = np.zeros(n_buckets + n_excess, dtype)
    h["ptr"] = -2
    blk = order
    h["x"][entry_sorted] = pos[blk, 0]
    h["y"][entry_sorted] = pos[blk, 1]
    h["z"][entry_sorted] = pos[blk, 2]
    h["offset"][entry_sorted] = offset_sorted
    h["ptr"][entry_sorted] = blk
    entry = np.empty(n, np.int64)
    entry[blk] = entry_sorted
    return h, entry.astype(np.int32), n_excess - 1 - n_ex


# ----------------------------------------------------------------------------------------
# C5E: the hash stress proper -- an unbounded procedurally tiled hall (capacity
# saturation, silent allocation failure, eviction churn).  The C5 walk above is confined to one
# room, whose whole surface fits in a few thousand 10 mm blocks; this scene keeps new surface
# entering the view however far the camera goes.
#
#   floor y = HALL_FLOOR, ceiling y = HALL_CEIL (world y points down, as the camera's);
#   a lattice of HALL_PERIOD-metre cells in x / z, each holding (by an integer hash of the cell)
#   a box standing on the floor, a box hanging from the ceiling, or nothing.  Floor boxes end at
#   y >= 0.2, ceiling boxes at y <= -0.35 and the camera stays in y in [-0.15, 0.1], so the camera
#   is never inside a box.
#
# Everything here is integer hashing and IEEE +, -, *, / in float64 (no transcendental function
# of the pixel), so synth/tf_synth.hip renders the same uint16 millimetres bit for bit; noise is
# the sum of four hashed uniforms (Irwin-Hall, std noise_mm).
# ----------------------------------------------------------------------------------------
HALL_FLOOR, HALL_CEIL, HALL_PERIOD, HALL_REACH = 0.55, -0.75, 0.8, 3
HALL_CAM_Y = (-0.15, 0.10)
_SQRT3 = 1.7320508075688772


def _mix32(h):
    """lowbias32 integer finaliser on uint32 (numpy arrays or scalars), wrapping arithmetic."""
    h = np.asarray(h, np.uint32)
    with np.errstate(over="ignore"):
        h = h ^ (h >> np.uint32(16))
        h = h * np.uint32(0x7FEB352D)
        h = h ^ (h >> np.uint32(15))
        h = h * np.uint32(0x846CA68B)
        h = h ^ (h >> np.uint32(16))
    return h


def _u32(v):
    return (np.asarray(v, np.int64) & 0xFFFFFFFF).astype(np.uint32)


def _unit(h):
    """uint32 -> float64 in [0, 1), exact."""
    return np.asarray(h, np.uint32).astype(np.float64) * (1.0 / 4294967296.0)


def hall_cell(i, j):
    """The box of lattice cell (i, j): (kind, lo[3], hi[3]); kind 0 none, 1 floor box, 2 ceiling box."""
    i = np.asarray(i, np.int64)
    j = np.asarray(j, np.int64)
    with np.errstate(over="ignore"):
        h = _mix32(_u32(i) * np.uint32(0x9E3779B1) ^ _mix32(_u32(j) + np.uint32(0x632BE5AB)))
        u = [_unit(h)]
        for k in range(5):
            h = _mix32(h + np.uint32(0x9E3779B9))
            u.append(_unit(h))
    kind = np.where(u[0] < 0.45, 1, np.where(u[0] < 0.8, 2, 0))
    cx = (i.astype(np.float64) + 0.5) * HALL_PERIOD + (u[1] - 0.5) * 0.2
    cz = (j.astype(np.float64) + 0.5) * HALL_PERIOD + (u[2] - 0.5) * 0.2
    hx = 0.08 + 0.14 * u[3]
    hz = 0.08 + 0.14 * u[4]
    ylo = np.where(kind == 1, 0.2 + 0.2 * u[5], HALL_CEIL)
    yhi = np.where(kind == 1, HALL_FLOOR, -0.35 - 0.2 * u[5])
    lo = np.stack([cx - hx, ylo, cz - hz], -1)
    hi = np.stack([cx + hx, yhi, cz + hz], -1)
    return kind, lo, hi


def _slab(o, d, lo, hi):
    """Ray / axis-aligned box entry distance (inf if missed or behind); o (3,), d (..., 3)."""
    tn = np.full(d.shape[:-1], -np.inf)
    tf = np.full(d.shape[:-1], np.inf)
    with np.errstate(divide="ignore", invalid="ignore"):
        for a in range(3):
            da = d[..., a]
            t1 = (lo[a] - o[a]) / da
            t2 = (hi[a] - o[a]) / da
            inside = (o[a] >= lo[a]) & (o[a] <= hi[a])
            par = da == 0
            t1 = np.where(par, np.where(inside, -np.inf, np.inf), t1)
            t2 = np.where(par, np.where(inside, np.inf, -np.inf), t2)
            tn = np.maximum(tn, np.minimum(t1, t2))
            tf = np.minimum(tf, np.maximum(t1, t2))
    return np.where((tn <= tf) & (tn > 1e-6), tn, np.inf)


def hall_noise(seed, frame, cols, rows):
    """Irwin-Hall(4) noise of frame `frame`, unit variance, (rows, cols) float64."""
    pix = np.arange(rows * cols, dtype=np.int64).reshape(rows, cols)
    with np.errstate(over="ignore"):
        base = _mix32(_mix32(_u32(seed) + np.uint32(0x2545F491)) ^ _u32(frame))
        s = np.zeros((rows, cols))
        for k in range(4):
            s = s + _unit(_mix32(base ^ _mix32(_u32(pix * 4 + k) + np.uint32(0x68E31DA4))))
    return (s - 2.0) * _SQRT3


def render_hall(R, t, cols=640, rows=480, noise_mm=1.0, seed=13, frame=0, intr=None):
    """uint16 depth (mm) of the hall from camera->world pose (R, t); 0 where nothing is hit.
    The reference renderer of synth/tf_synth.hip (tfs_render_hall): same bits."""
    fx, fy, cx, cy = intr if intr is not None else intrinsics(cols, rows)
    R = np.asarray(R, np.float64)
    o = np.asarray(t, np.float64)
    u = np.arange(cols, dtype=np.float64)
    v = np.arange(rows, dtype=np.float64)
    uu, vv = np.meshgrid(u, v)
    xc, yc = (uu - cx) / fx, (vv - cy) / fy
    # d = R @ (xc, yc, 1), written out so the order of the operations is fixed
    d = np.stack([(R[0, 0] * xc + R[0, 1] * yc) + R[0, 2], (R[1, 0] * xc + R[1, 1] * yc) + R[1, 2],
                  (R[2, 0] * xc + R[2, 1] * yc) + R[2, 2]], -1)
    best = np.full((rows, cols), np.inf)
    with np.errstate(divide="ignore", invalid="ignore"):
        for y0 in (HALL_FLOOR, HALL_CEIL):
            tt = (y0 - o[1]) / d[..., 1]
            best = np.minimum(best, np.where(tt > 1e-6, tt, np.inf))
    ci, cj = int(np.floor(o[0] / HALL_PERIOD)), int(np.floor(o[2] / HALL_PERIOD))
    for di in range(-HALL_REACH, HALL_REACH + 1):
        for dj in range(-HALL_REACH, HALL_REACH + 1):
            kind, lo, hi = hall_cell(ci + di, cj + dj)
            if int(kind) == 0:
                continue
            best = np.minimum(best, _slab(o, d, lo, hi))
    mm = best * 1000.0
    if noise_mm > 0:
        mm = mm + noise_mm * hall_noise(seed, frame, cols, rows)
    mm = np.where(np.isfinite(mm), np.rint(mm), 0.0)
    return np.clip(mm, 0, 65535).astype(np.uint16)


def hall_walk_poses(n, seed=13, step_m=0.01, step_deg=0.5):
    """Camera->world poses (R[n,3,3], t[n,3]) of the C5E walk through the hall: frame 0 at the
    identity; per frame a translation of at most step_m (~0.75 step_m on average) along a heading
    that turns by a bounded Ornstein-Uhlenbeck rate, the camera yawing with the heading and
    pitching / rolling a few degrees, every relative rotation <= step_deg.  Unconfined in x / z,
    y in HALL_CAM_Y (reflected).  float64."""
    rng = np.random.default_rng(seed)
    R = np.empty((n, 3, 3))
    t = np.empty((n, 3))
    pos = np.zeros(3)
    yaw = pitch = roll = 0.0
    w_yaw = w_pitch = w_roll = 0.0
    vy = 0.0
    d2r = np.pi / 180.0
    lim_yaw, lim_pitch, lim_roll = 0.40 * step_deg * d2r, 0.20 * step_deg * d2r, 0.10 * step_deg * d2r
    for k in range(n):
        cy_, sy_ = np.cos(yaw), np.sin(yaw)
        cp, sp = np.cos(pitch), np.sin(pitch)
        cr, sr = np.cos(roll), np.sin(roll)
        Ry = np.array([[cy_, 0, sy_], [0, 1, 0], [-sy_, 0, cy_]])
        Rx = np.array([[1, 0, 0], [0, cp, -sp], [0, sp, cp]])
        Rz = np.array([[cr, -sr, 0], [sr, cr, 0], [0, 0, 1]])
        R[k], t[k] = Ry @ Rx @ Rz, pos
        # turn rates: mean-reverting, bounded; pitch / roll pulled back to level
        w_yaw = float(np.clip(0.995 * w_yaw + rng.normal(0, 0.08) * lim_yaw, -lim_yaw, lim_yaw))
        w_pitch = float(np.clip(0.98 * w_pitch - 0.002 * pitch + rng.normal(0, 0.1) * lim_pitch, -lim_pitch, lim_pitch))
        w_roll = float(np.clip(0.98 * w_roll - 0.002 * roll + rng.normal(0, 0.1) * lim_roll, -lim_roll, lim_roll))
        yaw, pitch, roll = yaw + w_yaw, pitch + w_pitch, roll + w_roll
        speed = step_m * (0.6 + 0.3 * rng.random())                  # <= 0.9 step_m horizontally
        vy = float(np.clip(0.95 * vy + rng.normal(0, 0.05) * 0.2 * step_m, -0.2 * step_m, 0.2 * step_m))
        pos = pos + np.array([speed * np.sin(yaw), vy, speed * np.cos(yaw)])
        lo, hi = HALL_CAM_Y
        if pos[1] < lo:
            pos[1], vy = 2 * lo - pos[1], -vy
        if pos[1] > hi:
            pos[1], vy = 2 * hi - pos[1], -vy
    return R, t


def hall_sequence(n, cols=640, rows=480, seed=13, noise_mm=1.0, first=0):
    """C5E frames first..first+n-1 on the host (numpy), uint16 (n, rows, cols)."""
    R, t = hall_walk_poses(first + n, seed)
    intr = intrinsics(cols, rows)
    return np.stack([render_hall(R[k], t[k], cols, rows, noise_mm, seed, k, intr) for k in range(first, first + n)])


def world_to_camera_rt(R, t):
    """[R|t] camera->world -> row-major 3x4 world->camera (float32), what the engine entry points
    (tf_scene_alloc, tf_scene_fuse_frames) take; float32 inverse of the float32 pose as
    cv::Affine3f::inv computes it (tf_pose.h tf_rigid_inv)."""
    R = np.asarray(R, np.float32)
    t = np.asarray(t, np.float32)
    out = np.zeros(R.shape[:-2] + (3, 4), np.float32)
    Rt = np.swapaxes(R, -1, -2)
    out[..., :3, :3] = Rt
    # -(R^T t) summed in the order of tf_rigid_inv: (a0j*t0 + a1j*t1) + a2j*t2
    for j in range(3):
        out[..., j, 3] = -((R[..., 0, j] * t[..., 0] + R[..., 1, j] * t[..., 1]) + R[..., 2, j] * t[..., 2])
    return out


# ----------------------------------------------------------------------------------------
# GPU rendering of the synthetic streams (synth/libtfsynth.so, built by __graft_entry__.build()):
# the frames go straight into HBM through the same HIP runtime libtfusion_hip.so links.
# ----------------------------------------------------------------------------------------
_SYNTH_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "synth", "libtfsynth.so")
_synth = None


def synth_lib():
    """ctypes handle of synth/libtfsynth.so (raises if it was not built)."""
    global _synth
    if _synth is None:
        import ctypes
        if not os.path.exists(_SYNTH_SO):
            raise RuntimeError(f"{_SYNTH_SO} not built: run `make -C synth` (or __graft_entry__.build())")
        from topfusion_amd import _lib
        _lib.load()                      # the product library first: one HIP runtime for both
        L = ctypes.CDLL(_SYNTH_SO)
        P, S, I, D = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_double
        L.tfs_render_hall.argtypes = [P, S, P, I, I, I, I, D, D, D, D, ctypes.c_uint, D]
        L.tfs_render_room.argtypes = [P, S, P, I, I, I, I, D, D, D, D, ctypes.c_uint, D, I]
        L.tfs_render_room_rgb.argtypes = [P, S, P, I, I, I, D, D, D, D, I]
        L.tfs_copy_gbs.argtypes = [S, I]
        L.tfs_copy_gbs.restype = D
        L.tfs_malloc.argtypes = [ctypes.POINTER(P), S]
        L.tfs_free.argtypes = [P]
        L.tfs_download.argtypes = [P, P, S]
        L.tfs_upload.argtypes = [P, P, S]
        for f in ("tfs_render_hall", "tfs_render_room", "tfs_render_room_rgb", "tfs_malloc", "tfs_free", "tfs_download", "tfs_upload", "tfs_sync"):
            getattr(L, f).restype = I
        _synth = L
    return _synth


class DeviceStream:
    """n uint16 depth frames (rows x cols) in one device allocation (libtfsynth's hipMalloc)."""

    def __init__(self, n, cols, rows):
        import ctypes
        self.n, self.cols, self.rows = n, cols, rows
        self.frame_bytes = cols * rows * 2
        p = ctypes.c_void_p()
        assert synth_lib().tfs_malloc(ctypes.byref(p), max(16, n * self.frame_bytes)) == 0, "tfs_malloc"
        self.ptr = p.value

    def frame_ptr(self, k):
        return self.ptr + k * self.frame_bytes

    def download(self, k0=0, n=1):
        import ctypes
        out = np.empty((n, self.rows, self.cols), np.uint16)
        assert synth_lib().tfs_download(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(self.frame_ptr(k0)),
                                        n * self.frame_bytes) == 0
        return out

    def upload(self, frames, k0=0):
        import ctypes
        a = np.ascontiguousarray(frames, np.uint16).reshape(-1, self.rows, self.cols)
        assert synth_lib().tfs_upload(ctypes.c_void_p(self.frame_ptr(k0)), a.ctypes.data_as(ctypes.c_void_p), a.nbytes) == 0

    def free(self):
        import ctypes
        if self.ptr:
            synth_lib().tfs_free(ctypes.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def render_hall_device(stream, R, t, first=0, seed=13, noise_mm=1.0, k0=0):
    """Frames first..first+len(R)-1 of the hall (poses R, t camera->world) rendered on the GPU into
    stream slots k0.. (synth/tf_synth.hip: render_hall's bits)."""
    import ctypes
    n = len(R)
    P = np.zeros((n, 12), np.float64)
    P[:, :9] = np.asarray(R, np.float64).reshape(n, 9)
    P[:, 9:] = np.asarray(t, np.float64)
    fx, fy, cx, cy = intrinsics(stream.cols, stream.rows)
    rc = synth_lib().tfs_render_hall(ctypes.c_void_p(stream.frame_ptr(k0)), stream.frame_bytes,
                                     P.ctypes.data_as(ctypes.c_void_p), n, first, stream.cols, stream.rows,
                                     fx, fy, cx, cy, seed, noise_mm)
    assert rc == 0, f"tfs_render_hall: {rc}"


def render_room(R, t, cols=640, rows=480, noise_mm=1.0, seed=7, frame=0, sphere=True, intr=None):
    """The C2 / C5 room (render_depth's geometry: six walls, the sphere r = 0.3 m at (0.15, 0.25,
    1.3)) with the hall's hashed Irwin-Hall noise instead of numpy's generator, every operation in
    a fixed order: the reference renderer of synth/tf_synth.hip (tfs_render_room), same bits.
    This is what the bench and the GPU tests render on the device."""
    fx, fy, cx, cy = intr if intr is not None else intrinsics(cols, rows)
    R = np.asarray(R, np.float64)
    o = np.asarray(t, np.float64)
    u = np.arange(cols, dtype=np.float64)
    v = np.arange(rows, dtype=np.float64)
    uu, vv = np.meshgrid(u, v)
    xc, yc = (uu - cx) / fx, (vv - cy) / fy
    d = [(R[0, 0] * xc + R[0, 1] * yc) + R[0, 2], (R[1, 0] * xc + R[1, 1] * yc) + R[1, 2],
         (R[2, 0] * xc + R[2, 1] * yc) + R[2, 2]]
    best = np.full((rows, cols), np.inf)
    with np.errstate(divide="ignore", invalid="ignore"):
        for ax, off in ROOM_PLANES:
            tt = (off - o[ax]) / d[ax]
            best = np.minimum(best, np.where(tt > 1e-6, tt, np.inf))
        if sphere:
            oc = (o[0] - 0.15, o[1] - 0.25, o[2] - 1.3)
            b = (d[0] * oc[0] + d[1] * oc[1]) + d[2] * oc[2]
            a = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]
            cc = ((oc[0] * oc[0] + oc[1] * oc[1]) + oc[2] * oc[2]) - 0.09
            disc = b * b - a * cc
            t0 = (-b - np.sqrt(np.maximum(disc, 0.0))) / a
            best = np.minimum(best, np.where((disc >= 0) & (t0 > 1e-6), t0, np.inf))
    mm = best * 1000.0
    if noise_mm > 0:
        mm = mm + noise_mm * hall_noise(seed, frame, cols, rows)
    mm = np.where(np.isfinite(mm), np.rint(mm), 0.0)
    return np.clip(mm, 0, 65535).astype(np.uint16)


ROOM_PLANES = ((2, 1.8), (1, 0.6), (0, -0.8), (0, 1.1), (1, -0.9), (2, -0.6))   # render_depth's walls


def render_room_device(stream, R, t, first=0, seed=7, noise_mm=1.0, k0=0, sphere=True, intr=None):
    """Frames first.. of the room at poses (R, t) camera->world, rendered on the GPU into stream
    slots k0.. (synth/tf_synth.hip: render_room's bits)."""
    import ctypes
    n = len(R)
    P = np.zeros((n, 12), np.float64)
    P[:, :9] = np.asarray(R, np.float64).reshape(n, 9)
    P[:, 9:] = np.asarray(t, np.float64)
    fx, fy, cx, cy = intr if intr is not None else intrinsics(stream.cols, stream.rows)
    rc = synth_lib().tfs_render_room(ctypes.c_void_p(stream.frame_ptr(k0)), stream.frame_bytes,
                                     P.ctypes.data_as(ctypes.c_void_p), n, first, stream.cols, stream.rows,
                                     fx, fy, cx, cy, seed, noise_mm, 1 if sphere else 0)
    assert rc == 0, f"tfs_render_room: {rc}"


def orbit_device(n, cols=640, rows=480, seed=7, noise_mm=1.0):
    """C2 / C3: n frames of the orbit (orbit_pose; asserted inside the room) rendered on the GPU."""
    R = np.empty((n, 3, 3))
    t = np.empty((n, 3))
    for k in range(n):
        R[k], t[k] = orbit_pose(k)
        assert orbit_in_room(R[k], t[k]), f"orbit frame {k}: camera outside the room"
    s = DeviceStream(n, cols, rows)
    for b0 in range(0, n, 1024):
        b1 = min(n, b0 + 1024)
        render_room_device(s, R[b0:b1], t[b0:b1], first=b0, seed=seed, noise_mm=noise_mm, k0=b0)
    return s


def walk_device(n, cols=640, rows=480, seed=13, noise_mm=1.0):
    """C5: n frames of the room random walk (random_walk_poses) rendered on the GPU."""
    R, t = random_walk_poses(n, seed=seed)
    s = DeviceStream(n, cols, rows)
    for b0 in range(0, n, 1024):
        b1 = min(n, b0 + 1024)
        render_room_device(s, R[b0:b1], t[b0:b1], first=b0, seed=seed, noise_mm=noise_mm, k0=b0)
    return s


def hall_device(n, cols=640, rows=480, seed=13, noise_mm=1.0):
    """C5E: n frames of the hall walk rendered on the GPU; returns (stream, R, t)."""
    R, t = hall_walk_poses(n, seed)
    s = DeviceStream(n, cols, rows)
    for b0 in range(0, n, 1024):
        b1 = min(n, b0 + 1024)
        render_hall_device(s, R[b0:b1], t[b0:b1], first=b0, seed=seed, noise_mm=noise_mm, k0=b0)
    return s, R, t


def orbit_colour_device(n, cols=640, rows=480):
    """The colour camera's view (registered with the depth camera) of the first n orbit frames,
    rendered on the GPU (synth/tf_synth.hip k_render_room_rgb): uchar4 frames in one device
    allocation; returns (DeviceStream-like buffer, its device address)."""
    import ctypes
    R = np.empty((n, 3, 3))
    t = np.empty((n, 3))
    for k in range(n):
        R[k], t[k] = orbit_pose(k)
    P = np.zeros((n, 12), np.float64)
    P[:, :9] = R.reshape(n, 9)
    P[:, 9:] = t
    buf = DeviceStream(2 * n, cols, rows)              # 4 bytes per pixel = two uint16 frames' worth
    fx, fy, cx, cy = intrinsics(cols, rows)
    rc = synth_lib().tfs_render_room_rgb(ctypes.c_void_p(buf.ptr), cols * rows * 4, P.ctypes.data_as(ctypes.c_void_p), n,
                                         cols, rows, fx, fy, cx, cy, 1)
    assert rc == 0, f"tfs_render_room_rgb: {rc}"
    return buf
