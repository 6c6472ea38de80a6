"""The synthetic workloads (topfusion_amd/synth.py): the C2 orbit keeps the
camera inside the room, looking at the room, for every frame the bench generates."""
import numpy as np

from topfusion_amd import synth


def test_orbit_angle_ping_pong():
    """0.25 deg per frame at most, starting at 0 and equal to the plain orbit for the first
    100 frames, bounded by +-25 deg for any stream length."""
    a = np.array([synth.orbit_angle_deg(k) for k in range(2000)])
    assert a[0] == 0.0
    assert np.allclose(a[:101], 0.25 * np.arange(101))
    assert np.abs(np.diff(a)).max() <= 0.25 + 1e-9
    assert a.max() == 25.0 and a.min() == -25.0
    assert synth.orbit_angle_deg(1000, amplitude_deg=None) == 250.0


def test_orbit_camera_inside_room_bench_frames():
    """Every frame of the driver's bench shape ((5 + 20) x 32 = 800) and well beyond: the camera
    centre is >= 0.2 m inside every wall, and the old plain orbit is not (it crossed the left wall
    at frame 168)."""
    for k in range(0, 4000):
        R, t = synth.orbit_pose(k)
        assert synth.orbit_in_room(R, t), k
    R, t = synth.orbit_pose(200, amplitude_deg=None)
    assert not synth.orbit_in_room(R, t)


def test_orbit_frames_see_the_room():
    """Sampled frames over a whole ping-pong period: >= 80 % of the pixels hold a surface within
    the ICP truncation range 0.2-2.0 m (TopFuParams::icp_truncate_depth_dist), and the sphere is in
    view at the start."""
    W, H = 160, 120
    intr = synth.intrinsics(W, H)
    for k in range(0, 400, 20):
        d = synth.render_depth(*synth.orbit_pose(k), W, H, intr=intr).astype(np.float64)
        frac = ((d >= 200) & (d <= 2000)).mean()
        assert frac >= 0.8, (k, frac)
    d0 = synth.render_depth(*synth.orbit_pose(0), W, H, intr=intr)
    dn = synth.render_depth(*synth.orbit_pose(0), W, H, sphere=False, intr=intr)
    assert (d0 < dn).sum() > 0.05 * W * H


def test_hall_walk_bounds_and_reach():
    """C5E walk (synth.hall_walk_poses): <= 1 cm and <= 0.5 deg per frame, the
    camera between the floor-box tops and the ceiling-box bottoms (never inside a box), and
    unconfined -- tens of metres of new hall over the bench's 51 k frames."""
    R, t = synth.hall_walk_poses(51000, seed=13)
    steps = np.linalg.norm(np.diff(t, axis=0), axis=1)
    assert steps.max() <= 0.01
    tr = np.einsum("kij,kij->k", R[:-1], R[1:])          # trace(R_k^T R_k+1)
    ang = np.degrees(np.arccos(np.clip((tr - 1) / 2, -1, 1)))
    assert ang.max() <= 0.5
    lo, hi = synth.HALL_CAM_Y
    assert t[:, 1].min() >= lo and t[:, 1].max() <= hi
    assert lo > -0.35 and hi < 0.2                          # ceiling boxes end at <= -0.35, floor boxes start at >= 0.2
    extent = np.ptp(t[:, 0]) + np.ptp(t[:, 2])
    assert extent > 50.0, extent
    R2, t2 = synth.hall_walk_poses(300, seed=13)
    assert np.array_equal(R2, R[:300]) and np.array_equal(t2, t[:300])   # a prefix of a longer walk


def test_hall_frames_in_range():
    """Hall frames carry surface inside computeDists' 2.047 m range (what allocation sees)."""
    R, t = synth.hall_walk_poses(3001, seed=13)
    W, H = 160, 120
    intr = synth.intrinsics(W, H)
    for k in (0, 1500, 3000):
        d = synth.render_hall(R[k], t[k], W, H, 1.0, 13, k, intr)
        assert ((d > 0) & (d < 2047)).mean() > 0.2, k


def test_world_to_camera_rt_is_rigid_inverse():
    R, t = synth.hall_walk_poses(50, seed=13)
    w2c = synth.world_to_camera_rt(R, t)
    for k in (0, 17, 49):
        M = np.eye(4)
        M[:3, :3], M[:3, 3] = R[k], t[k]
        N = np.eye(4)
        N[:3] = w2c[k]
        assert np.allclose(N @ M, np.eye(4), atol=1e-5)
