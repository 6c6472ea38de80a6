"""The ICP iterations' pose algebras on the GPU (tf_set_pose_algebra / TFUSION_ICP_SOLVE): the
reference's own -- OpenCV's cv::determinant, cv::solve(DECOMP_SVD) and Affine3f(rvec, t) as
OpenCV 3.x-4.x (opencv4, the default) and 2.4.9 (opencv2) publish them
(projective_icp.cpp:197-209) -- and the canonical one, each bit-exact against the oracle's
restatement of the same algorithms (oracle/tf_oracle.c, TFO_POSE_*, portable transcendental
functions, which gave the same bits as glibc's over the whole C2 window,
profiles/r05/pose_algebra_gap_C2.json).  Parity with OpenCV itself is unpinned: the restatement
follows OpenCV's published algorithms and has not been checked against an OpenCV build (none is
available here and the reference ships no fixtures)."""
import numpy as np
import pytest

from parity_util import DeviceFrames, assert_bit_exact
from test_gpu_parity import _compare_frame_state, compare_scene
from topfusion_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture
def cv_oracle(oracle_mod):
    """The oracle module with its pose algebra restored to the default (opencv4) afterwards."""
    yield oracle_mod
    oracle_mod.set_pose_algebra("opencv4")


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
    assert g.pose_algebra() == 4                # the reference's algebra by default
    for a, v in (("opencv4", 4), ("opencv2", 2), ("svd", 4), ("canonical", 0)):
        g.set_pose_algebra(a)
        assert g.pose_algebra() == v
    with pytest.raises(L.TfError):
        g.set_pose_algebra(3)
    g.close()


def test_canonical_algebra_bench_timed_window(cv_oracle):
    """The bench's C2 input and schedule over its whole run (frames 0..799 in 25 tf_process_frames
    steps of 32) under the canonical algebra (LU + block Schur + sinc Rodrigues; the default,
    OpenCV 4's, is test_gpu_parity.test_bench_timed_window): every frame's ok flag equal, the whole
    state bit-exact after frames 191, 479 and 799."""
    import bench
    W, H, F, steps = 640, 480, 32, 25
    g, args = _pair(cv_oracle, W, H, "canonical")
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
            tag = f"canonical bench frames {step * F}..{(step + 1) * F - 1}"
            _compare_frame_state(g, o, tag, grey=bool(oko[-1]))
            compare_scene(g, o, tag)
    assert n_reset == 80, n_reset          # the oracle's count under the canonical algebra (pose_algebra_gap_C2.json)
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


def _solve_systems_inputs():
    """ICP systems (27 sums each): every iteration the oracle ran on the bench's first 120 C2
    frames under OpenCV 4's algebra (tests/golden/icp_systems_C2_opencv4.f32, made by
    tools/svd_systems.py), random ICP-like systems at three scales, and degenerate ones -- A = 0
    and rank 1..5 (zero singular values: the random completion)."""
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    cap = np.fromfile(os.path.join(here, "golden", "icp_systems_C2_opencv4.f32"), np.float32).reshape(-1, 27)
    rng = np.random.default_rng(20261018)
    iu = [(a, c) for a in range(6) for c in range(a, 7)]
    out = [cap]
    for scale, rows in ((1.0, 40), (1e-6, 12), (1e6, 8), (1.0, 7)):
        v = (rng.random((3000, rows, 7), np.float32) - 0.5) * np.float32(scale)
        s = np.stack([np.einsum("nr,nr->n", v[:, :, a], v[:, :, c]) for a, c in iu], axis=1)
        out.append(s.astype(np.float32))
    deg = []
    for rank in range(6):
        for _ in range(20):
            v = rng.random((rank, 7), np.float32) - 0.5
            deg.append(np.array([np.dot(v[:, a], v[:, c]) for a, c in iu], np.float32))
    out.append(np.stack(deg))
    return np.ascontiguousarray(np.concatenate(out), np.float32)


@pytest.mark.parametrize("algebra", ["opencv4", "opencv2", "canonical"])
def test_solve_systems_bit_exact(oracle_mod, algebra):
    """tf_icp_solve_systems (the persistent ICP's det + solve device code; OpenCV: the lane-parallel
    Jacobi SVD with its fast (c, s) sequence and exact fallback) against the oracle's serial
    cv::determinant / cv::solve(DECOMP_SVD) (canonical: LU + block Schur), every bit of x and det."""
    import ctypes
    from parity_util import DeviceBuffer
    from topfusion_amd import _lib as L
    sums = _solve_systems_inputs()
    n = sums.shape[0]
    code = {"canonical": 0, "opencv2": 2, "opencv4": 4}[algebra]
    d_in = DeviceFrames(sums)
    d_x = DeviceBuffer(n * 6 * 4)
    d_det = DeviceBuffer(n * 8)
    L.check(L.load().tf_icp_solve_systems(code, d_in.ptr, n, d_x.ptr, d_det.ptr, None), "tf_icp_solve_systems")
    d_x.sync()
    x = np.empty((n, 6), np.float32)
    det = np.empty(n, np.float64)
    assert d_x._hip.hipMemcpy(x.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(d_x.ptr), ctypes.c_size_t(x.nbytes), 2) == 0
    assert d_x._hip.hipMemcpy(det.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(d_det.ptr), ctypes.c_size_t(det.nbytes), 2) == 0
    Lo = oracle_mod.lib()
    ox = np.empty((n, 6), np.float32)
    od = np.empty(n, np.float64)
    iu = [(a, c) for a in range(6) for c in range(a, 7)]
    for q in range(n):
        A = np.zeros((6, 6), np.float32)
        b = np.zeros(6, np.float32)
        for (a, c), v in zip(iu, sums[q]):
            if c == 6:
                b[a] = v
            else:
                A[a, c] = A[c, a] = v
        xq = np.zeros(6, np.float32)
        if code == 0:
            Lo.tfo_solve6(A.ctypes.data, b.ctypes.data, xq.ctypes.data)
            od[q] = Lo.tfo_det6(A.ctypes.data)
        else:
            Lo.tfo_cv_solve_svd6(A.ctypes.data, b.ctypes.data, xq.ctypes.data)
            od[q] = Lo.tfo_cv_det6(A.ctypes.data, code)
        ox[q] = xq
    assert_bit_exact(f"{algebra} solve x", x, ox)
    assert_bit_exact(f"{algebra} det", det, od)
    for buf in (d_in, d_x, d_det):
        buf.free()
