"""Device-side failures (include/tfusion_hip.h, "Device-side failures"), each forced
deterministically by a fault-injection switch read at tf_create:

* TFUSION_ICP_FAULT=launch:iteration -- that persistent ICP launch reports a lost peer (as when
  another process holds part of the device and not all 256 workgroups are co-resident).  The
  frame is re-run on the per-iteration schedule and continues: every frame bit-exact with the
  oracle, whichever path (batch, per-call returning on the verdict, per-call synchronous).
* TFUSION_FILL_FAULT=launch -- that k_raycast_pair launch's wait for the range image fails (past
  the ICP: the frame is half done).  The context reports TF_HIP_ERROR from then on -- on the next
  call for a per-call frame that had already returned -- until tf_reset."""
import numpy as np
import pytest

from parity_util import DeviceFrames
from test_gpu_parity import _compare_frame_state, compare_scene, make_pair
from topfusion_amd import synth

pytestmark = pytest.mark.gpu

W, H, N = 320, 240, 8


@pytest.mark.parametrize("mode", ["batch", "per_call", "per_call_sync"])
def test_icp_lost_peer_fallback(oracle_mod, monkeypatch, mode):
    from topfusion_amd import _lib as L
    monkeypatch.setenv("TFUSION_ICP_FAULT", "3:5")        # frame 2's persistent launch, at iteration 5
    if mode == "per_call_sync":
        monkeypatch.setenv("TFUSION_PERCALL_EARLY", "0")
    g, o = make_pair(oracle_mod, W, H)
    assert g.icp_persistent()
    frames = synth.orbit_sequence(N, W, H, seed=7)
    dev = DeviceFrames(frames)
    fb = W * H * 2
    if mode == "batch":
        okg = g.process_frames(dev.ptr, N)
    else:
        okg = np.array([g(dev.ptr + k * fb) for k in range(N)])
    oko = np.array([o(frames[k]) for k in range(N)])
    assert np.array_equal(okg, oko), (okg, oko)
    assert okg[2], "frame 2 must be a tracked frame for the fault to hit"
    pg = g.getCameraPose()[:3, :4]
    assert np.array_equal(pg.view(np.uint32), o.pose().view(np.uint32))
    _compare_frame_state(g, o, f"lost peer ({mode})", grey=bool(oko[-1]))
    compare_scene(g, o, f"lost peer ({mode})")
    assert g.totals()["icp_fallbacks"] == 1
    assert g.stats()["icp_iterations"] == o.counters()["icp_iterations"]
    g.close()
    dev.free()


@pytest.mark.parametrize("mode", ["batch", "per_call"])
def test_error_past_icp_is_sticky(monkeypatch, mode):
    from topfusion_amd import TopFu, default_params, _lib as L
    monkeypatch.setenv("TFUSION_ED_LDS_MAX_N", "0")       # the fill's atomic path: CreateICPMaps' tiles wait on it
    monkeypatch.setenv("TFUSION_FILL_FAULT", "3")         # frame 2's k_raycast_pair: the wait fails
    fx, fy, cx, cy = synth.intrinsics(W, H)
    g = TopFu(default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy))
    frames = synth.orbit_sequence(N, W, H, seed=7)
    dev = DeviceFrames(frames)
    fb = W * H * 2
    if mode == "batch":
        with pytest.raises(L.TfError) as ei:
            g.process_frames(dev.ptr, N)
        assert ei.value.status == L.TF_HIP_ERROR
    else:
        for k in range(3):
            assert g(dev.ptr + k * fb)                     # frame 2 returns on its verdict, before its tail runs
        with pytest.raises(L.TfError) as ei:
            g(dev.ptr + 3 * fb)                            # reported by the next call
        assert ei.value.status == L.TF_HIP_ERROR
    I = np.tile(np.eye(4, dtype=np.float32)[:3], (2, 1, 1))
    for call in (g.stats, g.getCameraPose, lambda: g(dev.ptr), g.hash, g.vba,
                 lambda: g.fuse_frames(dev.ptr, I)):
        with pytest.raises(L.TfError) as ei:               # sticky: every call until tf_reset (ADVICE r4:
            call()                                         # downloads and engine batches too)
        assert ei.value.status == L.TF_HIP_ERROR
    g.reset()
    ok = g.process_frames(dev.ptr, N)                      # the context works again
    assert ok.all()
    assert g.stats()["frame_counter"] == N
    g.close()
    dev.free()


def test_vis_build_lost_wait_is_sticky_on_engine_path(monkeypatch):
    """TFUSION_VIS_FAULT=l: the l-th k_vis_build launch's wait for the lower chunks' counts fails.
    An engine-level batch (tf_scene_fuse_frames) has no frame end, so the kernel itself marks the
    context in error: the batch and every later call report TF_HIP_ERROR until tf_reset
    clears it."""
    from topfusion_amd import TopFu, default_params, _lib as L
    monkeypatch.setenv("TFUSION_VIS_FAULT", "2")
    fx, fy, cx, cy = synth.intrinsics(W, H)
    g = TopFu(default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy))
    frames = np.stack([synth.room_corner(W, H, seed=42 + k) for k in range(3)])
    dev = DeviceFrames(frames)
    I = np.tile(np.eye(4, dtype=np.float32)[:3], (3, 1, 1))
    with pytest.raises(L.TfError) as ei:
        g.fuse_frames(dev.ptr, I)
    assert ei.value.status == L.TF_HIP_ERROR
    for call in (g.stats, g.hash, lambda: g.fuse_frames(dev.ptr, I[:1])):
        with pytest.raises(L.TfError) as ei:
            call()
        assert ei.value.status == L.TF_HIP_ERROR
    g.reset()
    rec = g.fuse_frames(dev.ptr, I)                        # the fault fired once: the context works again
    assert (rec["noVisibleEntries"] > 0).all()
    g.close()
    dev.free()


def test_engine_batch_no_ops_after_lost_wait(monkeypatch):
    """once an engine batch's k_vis_build wait fails (TFUSION_VIS_FAULT=2: frame 1 of
    the batch), the rest of the batch changes nothing -- frame 1 integrates nothing over its
    unbuilt list, and frames 2.. allocate nothing (their records show frame 1's free-list top,
    where a clean context on the same frames allocates new blocks) -- and the next call returns
    TF_HIP_ERROR without enqueuing anything.  The records are read through the C-ABI, which fills
    them before it reports the error."""
    import ctypes
    from topfusion_amd import TopFu, default_params, _lib as L
    fx, fy, cx, cy = synth.intrinsics(W, H)
    n = 4
    frames = np.stack([synth.room_corner(W, H, seed=42 + k) for k in range(n)])
    dev = DeviceFrames(frames)
    poses = np.tile(np.eye(4, dtype=np.float32)[:3], (n, 1, 1))
    poses[:, 0, 3] = 0.12 * np.arange(n)                    # each frame 12 cm further along x: new blocks

    def batch(g):
        rec = np.zeros(n, L.FUSE_RECORD_DTYPE)
        P = np.ascontiguousarray(poses.reshape(n, 12))
        st = L.load().tf_scene_fuse_frames(g._h, None, ctypes.c_void_p(dev.ptr), W * H * 2, 0,
                                           P.ctypes.data_as(ctypes.c_void_p), n, rec.ctypes.data_as(ctypes.c_void_p))
        return st, rec

    clean = TopFu(default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy))
    st0, rec0 = batch(clean)
    assert st0 == L.TF_OK
    assert rec0["lastFreeBlockId"][2] < rec0["lastFreeBlockId"][1]      # the clean run allocates at frame 2
    clean.close()
    monkeypatch.setenv("TFUSION_VIS_FAULT", "2")
    g = TopFu(default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy))
    st1, rec1 = batch(g)
    assert st1 == L.TF_HIP_ERROR
    assert rec1["lastFreeBlockId"][0] == rec0["lastFreeBlockId"][0]     # frame 0 as the clean run
    assert (rec1["lastFreeBlockId"][2:] == rec1["lastFreeBlockId"][1]).all(), rec1["lastFreeBlockId"]
    st2, rec2 = batch(g)
    assert st2 == L.TF_HIP_ERROR and (rec2["lastFreeBlockId"] == 0).all()   # nothing enqueued, records untouched
    g.reset()
    st3, rec3 = batch(g)
    assert st3 == L.TF_OK and (rec3["lastFreeBlockId"] == rec0["lastFreeBlockId"]).all()
    g.close()
    dev.free()
