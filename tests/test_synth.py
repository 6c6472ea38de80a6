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
