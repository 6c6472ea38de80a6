"""Per-call frames (tf_process_frame = TopFu::operator(), topfu.cpp:161-330) called back to back
with no host synchronisation between them, as demo.cpp's loop and bench.py's per-call rate do.

A per-call frame returns once its verdict -- the bool and poses_.back() -- is known (the persistent
ICP launch writes it into host memory), with its allocation, integration, raycasts and frame end
still running, so the next call's launches queue behind them; its last two launches are enqueued by
the next call with that frame's preprocessing in their grid tails, or by any other entry point
first (DESIGN §6 "Per-call rate").  Every frame's bool and pose, and the whole state at the end,
must be bit-exact with the oracle run frame by frame -- with and without the early return
(TFUSION_PERCALL_EARLY) and the deferred launches (TFUSION_PERCALL_DEFER), with a batch, renders
and host-depth frames mixed in between.
"""
import ctypes

import numpy as np
import pytest

from parity_util import DeviceFrames, assert_bit_exact
from topfusion_amd import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("early,defer", [("1", "1"), ("1", "0"), ("0", "1")])
def test_per_call_back_to_back(oracle_mod, monkeypatch, early, defer):
    from test_gpu_parity import _compare_frame_state, compare_scene
    from topfusion_amd import TopFu, default_params
    from topfusion_amd import _lib as L
    monkeypatch.setenv("TFUSION_PERCALL_EARLY", early)
    monkeypatch.setenv("TFUSION_PERCALL_DEFER", defer)
    W, H, n = 640, 480, 48
    fx, fy, cx, cy = synth.intrinsics(W, H)
    args = dict(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy)
    g = TopFu(default_params(**args))
    o = oracle_mod.Oracle(oracle_mod.default_params(**args), omp=True)
    seq = synth.orbit_sequence(n, W, H, seed=7)
    seq[21] = np.zeros_like(seq[21])                  # an ICP failure -> reset inside the run
    dev = DeviceFrames(seq)
    lib, fb = L.load(), W * H * 2
    got_ok, got_pose = [], []
    k = 0
    while k < n:
        if k == 30:                                   # a batch in between
            okb = g.process_frames(dev.ptr + k * fb, 6)
            got_ok += list(okb)
            got_pose += [None] * 6
            k += 6
            continue
        pose = np.zeros(12, np.float32)
        if k in (12, 40):                             # host-depth frames (tf_process_frame_host)
            s = lib.tf_process_frame_host(g._h, seq[k].ctypes.data_as(ctypes.c_void_p), W * 2,
                                          pose.ctypes.data_as(ctypes.c_void_p), None)
        else:
            s = lib.tf_process_frame(g._h, ctypes.c_void_p(dev.ptr + k * fb), W * 2,
                                     pose.ctypes.data_as(ctypes.c_void_p), None)
        L.check(s, "tf_process_frame", allow=(L.TF_OK, L.TF_ICP_FAIL))
        got_ok.append(s == L.TF_OK)
        got_pose.append(pose)
        if k in (8, 25):                              # renderImage between frames (stream-ordered)
            L.check(lib.tf_render_image_type(g._h, 0, None, 0), "tf_render_image_type")
        k += 1
    n_fail = 0
    for k in range(n):
        oko = o(seq[k])
        assert got_ok[k] == oko, f"frame {k}: gpu {got_ok[k]} oracle {oko}"
        n_fail += int(not oko)
        if got_pose[k] is not None:
            assert_bit_exact(f"frame {k} pose", got_pose[k].reshape(3, 4), o.pose())
    assert n_fail >= 1
    _compare_frame_state(g, o, "per-call final", grey=bool(got_ok[-1]))
    compare_scene(g, o, "per-call final")
    g.close()
    dev.free()
