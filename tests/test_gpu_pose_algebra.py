"""The reference's own pose algebra on the GPU (tf_set_pose_algebra / TFUSION_ICP_SOLVE):
OpenCV's cv::determinant, cv::solve(DECOMP_SVD) and Affine3f(rvec, t) as OpenCV 3.x-4.x
(opencv4) and 2.4.9 (opencv2) publish them (projective_icp.cpp:197-209), bit-exact against the
oracle's restatement of the same algorithms (oracle/tf_oracle.c, TFO_POSE_OPENCV*, portable
transcendental functions -- which gave the same bits as glibc's over the whole C2 window,
profiles/r05/pose_algebra_gap_C2.json)."""
import numpy as np
import pytest

from parity_util import DeviceFrames, assert_bit_exact
from test_gpu_parity import _compare_frame_state, compare_scene
from topfusion_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture
def cv_oracle(oracle_mod):
    """The oracle module with its pose algebra restored to canonical afterwards."""
    yield oracle_mod
    oracle_mod.set_pose_algebra("canonical")


def _pair(oracle_mod, W, H, algebra):
    from topfusion_amd import TopFu, default_params
    fx, fy, cx, cy = synth.intrinsics(W, H)
    args = dict(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy)
    g = TopFu(default_params(**args))
    g.set_pose_algebra(algebra)
    oracle_mod.set_pose_algebra(algebra, libm=False)
    return g, args


def test_pose_algebra_api():
    from topfusion_amd import TopFu, default_params, _lib as L
    fx, fy, cx, cy = synth.intrinsics(320, 240)
    g = TopFu(default_params(cols=320, rows=240, fx=fx, fy=fy, cx=cx, cy=cy))
    assert g.pose_algebra() == 0
    for a, v in (("opencv4", 4), ("opencv2", 2), ("svd", 4), ("canonical", 0)):
        g.set_pose_algebra(a)
        assert g.pose_algebra() == v
    with pytest.raises(L.TfError):
        g.set_pose_algebra(3)
    g.close()


def test_opencv4_algebra_bench_timed_window(cv_oracle):
    """The bench's C2 input and schedule over its whole run (frames 0..799 in 25 tf_process_frames
    steps of 32) under the OpenCV 3.x-4.x algebra: every frame's ok flag equal, the whole state
    bit-exact after frames 191, 479 and 799."""
    import bench
    W, H, F, steps = 640, 480, 32, 25
    g, args = _pair(cv_oracle, W, H, "opencv4")
    assert g.icp_persistent()
    o = cv_oracle.Oracle(cv_oracle.default_params(**args), omp=True)
    dev = bench.orbit_frames(steps * F, W, H, 7)
    fb = W * H * 2
    n_reset = 0
    for step in range(steps):
        okg = g.process_frames(dev.ptr + step * F * fb, F)
        host = dev.download(step * F, F)
        oko = np.array([o(host[k]) for k in range(F)])
        assert np.array_equal(okg, oko), (step, okg, oko)
        n_reset += int((~oko).sum())
        if step in (5, 14, 24):
            tag = f"opencv4 bench frames {step * F}..{(step + 1) * F - 1}"
            _compare_frame_state(g, o, tag, grey=bool(oko[-1]))
            compare_scene(g, o, tag)
    assert n_reset == 79, n_reset          # the oracle's count under OpenCV 4 (profiles/r05/pose_algebra_gap_C2.json)
    g.close()
    dev.free()


@pytest.mark.parametrize("schedule", ["persistent", "per_iteration"])
def test_opencv2_algebra_per_call(cv_oracle, monkeypatch, schedule):
    """OpenCV 2.4.9's variant, per-call frames (TopFu::operator()), on both ICP schedules: every
    frame's bool, iteration count and pose bit-exact, the scene at the end."""
    if schedule == "per_iteration":
        monkeypatch.setenv("TFUSION_ICP_PERSISTENT", "0")
    W, H, N = 320, 240, 24
    g, args = _pair(cv_oracle, W, H, "opencv2")
    assert g.icp_persistent() == (schedule == "persistent")
    o = cv_oracle.Oracle(cv_oracle.default_params(**args))
    frames = synth.orbit_sequence(N, W, H, seed=7)
    dev = DeviceFrames(frames)
    for k in range(N):
        okg, oko = g(dev.ptr + k * W * H * 2), o(frames[k])
        assert okg == oko, (k, okg, oko)
        sg, so = g.stats(), o.counters()
        assert sg["icp_iterations"] == so["icp_iterations"], k
        assert_bit_exact(f"opencv2 {schedule} frame {k} pose", g.getCameraPose()[:3, :4], o.pose())
    compare_scene(g, o, f"opencv2 {schedule}")
    g.close()
    dev.free()
