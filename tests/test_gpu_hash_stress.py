"""C5 hash stress at the engine level (BASELINE configs[4]; bench.py --config C5E):
capacity saturation and the silent allocation failures of allocateVoxelBlocksList
(SceneReconstructionEngine_host.cu:358-413), bit for bit against the oracle at 640x480 with the
reference capacities (65 536 blocks, 2^20 buckets, 2^17 excess entries).

The frames are the bench's: the unconfined walk through the tiled hall (synth.render_hall),
rendered on the GPU (synth/tf_synth.hip, checked here against the numpy renderer), fused by
tf_scene_fuse_frames (checked against the per-call engine entry points).  The saturated regime
starts ~12 k frames in; the GPU runs the walk up to just before it, its whole scene state
(hash, voxels, both free lists, the visible list and types, the counters) is handed to the
oracle, and both run on, frame by frame, past the first failure."""
import ctypes

import numpy as np
import pytest

from parity_util import DeviceBuffer, assert_bit_exact, assert_struct_exact
from topfusion_amd import synth

pytestmark = pytest.mark.gpu

W, H, VOX = 640, 480, 0.01


def _params(mod, swapping=False, **kw):
    fx, fy, cx, cy = synth.intrinsics(W, H)
    args = dict(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy, voxelSize=VOX, **kw)
    if swapping:
        args.update(use_swapping=1, swap_transfer_blocks=0x1000)
    return mod.default_params(**args)


def _walk(n, seed=13):
    R, t = synth.hall_walk_poses(n, seed)
    return R, t, synth.world_to_camera_rt(R, t)


def _oracle_frame(o, frame, w2c, swapping):
    from oracle import oracle as O
    d = O.compute_dists(frame)
    o.alloc(w2c, d)
    o.integrate(w2c, d)
    if swapping:
        o.swap()


def _check_record(tag, rec, o, swapping):
    c = o.counters()
    f1, f2 = o.alloc_failures()
    got = (int(rec["lastFreeBlockId"]), int(rec["lastFreeExcessListId"]), int(rec["noVisibleEntries"]),
           int(rec["alloc_failed_type1"]), int(rec["alloc_failed_type2"]))
    want = (c["lastFreeBlockId"], c["lastFreeExcessListId"], c["noVisibleEntries"], f1, f2)
    assert got == want, f"{tag}: record (lastFree, lastFreeExcess, noVisible, fail1, fail2) gpu {got} oracle {want}"
    if swapping:
        si, so, sr = o.swap_counts()
        g3 = (int(rec["swapped_in"]), int(rec["swapped_out"]), int(rec["swap_realloc"]))
        assert g3 == (si, so, sr), f"{tag}: swap counts gpu {g3} oracle {(si, so, sr)}"


def _compare_all(tag, g, o, swapping):
    from test_gpu_parity import compare_scene
    compare_scene(g, o, tag)
    assert_bit_exact(f"{tag} allocationList", g.alloc_list(), o.alloc_list())
    assert_bit_exact(f"{tag} excessAllocationList", g.excess_list(), o.excess_list())
    if swapping:
        assert_bit_exact(f"{tag} swap state", g.swap_state(), o.swap_state())
        fg, fo = g.swap_stored_flags(), o.swap_stored_flags()
        assert_bit_exact(f"{tag} stored flags", fg, fo)
        ids = np.nonzero(fo)[0]
        if len(ids):
            sg = g.swap_stored().reshape(-1, 512)[ids]
            so = o.swap_stored().reshape(-1, 512)[ids]
            assert_struct_exact(f"{tag} stored blocks", sg, so, ["sdf", "w"])


def _handoff(g, o, swapping):
    """The oracle's scene := the GPU context's (engine-level state only)."""
    from topfusion_amd import _lib as L
    st = g.stats()
    kw = {}
    if swapping:
        kw = dict(swap_state=g.swap_state(), swap_stored_flags=g.swap_stored_flags(), swap_stored=g.swap_stored())
    o.load_scene_state(g.hash(), g.vba(), g.alloc_list(), g.excess_list(),
                       g.download(L.TF_BUF_VISIBLE_IDS).view(np.int32), g.visible_type(),
                       (st["lastFreeBlockId"], st["lastFreeExcessListId"], st["noVisibleEntries"]), **kw)


def test_hall_renderer_gpu_equals_numpy():
    """synth/tf_synth.hip renders synth.render_hall's uint16 millimetres bit for bit (noise
    included), at the walk's start and deep into it."""
    R, t, _ = _walk(7780)
    ks = [0, 1, 7779]
    s = synth.DeviceStream(len(ks), W, H)
    for i, k in enumerate(ks):
        synth.render_hall_device(s, R[k:k + 1], t[k:k + 1], first=k, k0=i)
    got = s.download(0, len(ks))
    s.free()
    for i, k in enumerate(ks):
        want = synth.render_hall(R[k], t[k], W, H, 1.0, 13, k)
        assert_bit_exact(f"hall frame {k}", got[i], want)
        assert ((want > 0) & (want < 2047)).mean() > 0.2, k        # surface in computeDists' range


@pytest.mark.parametrize("fuse_tail", ["1", "0"])
def test_fuse_frames_equals_per_call_engine(oracle_mod, monkeypatch, fuse_tail):
    """tf_scene_fuse_frames == tf_imgproc_compute_dists + tf_scene_alloc + tf_scene_integrate per
    frame (GPU vs GPU, whole state), and both == the oracle, over 24 hall frames.  fuse_tail 1
    (default): four launches per frame, frame k+1's head (dists, matrices, setToType3) in frame k's
    integration grid; 0: the seven-launch form."""
    monkeypatch.setenv("TFUSION_FUSE_TAIL", fuse_tail)
    from topfusion_amd import TopFu, _lib as L
    n = 24
    R, t, w2c = _walk(n)
    s = synth.DeviceStream(n, W, H)
    synth.render_hall_device(s, R, t)
    gf = TopFu(_params(L))
    rec = gf.fuse_frames(s.ptr, w2c)
    gp = TopFu(_params(L))
    lib = L.load()
    dists = DeviceBuffer(W * H * 4)
    intr = np.array(synth.intrinsics(W, H), np.float32)
    fp = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data_as(ctypes.c_void_p)
    o = oracle_mod.Oracle(_params(oracle_mod), omp=True)
    frames = s.download(0, n)
    for k in range(n):
        L.check(lib.tf_imgproc_compute_dists(ctypes.c_void_p(s.frame_ptr(k)), W * 2, ctypes.c_void_p(dists.ptr), W * 4, W, H,
                                             None), "compute_dists")
        L.check(lib.tf_scene_alloc(gp._h, fp(intr), fp(w2c[k]), ctypes.c_void_p(dists.ptr), W * 4, 0, 0), "tf_scene_alloc")
        L.check(lib.tf_scene_integrate(gp._h, fp(intr), fp(w2c[k]), ctypes.c_void_p(dists.ptr), W * 4), "tf_scene_integrate")
        _oracle_frame(o, frames[k], w2c[k], False)
        _check_record(f"fuse frame {k}", rec[k], o, False)
    _compare_all("fuse vs oracle", gf, o, False)
    _compare_all("per-call vs oracle", gp, o, False)
    assert rec["noVisibleEntries"][-1] > 100
    dists.free()
    s.free()
    gf.close()
    gp.close()


def test_c5e_saturation_640x480(oracle_mod):
    """The bench's C5E walk through the VBA's exhaustion: the GPU fuses the walk until fewer than
    1200 free blocks are left, hands its state to the oracle, and both run >= 40 frames past the
    first silent failure, every frame's counters, failure counts and visible types compared, the
    whole scene (hash, voxels, free lists, visible list) every 16 frames and at the end."""
    from topfusion_amd import TopFu, _lib as L
    N = 14000
    R, t, w2c = _walk(N)
    s = synth.DeviceStream(N, W, H)
    synth.render_hall_device(s, R, t)
    g = TopFu(_params(L))
    k = 0
    while k < N:                                        # fast-forward in batches while blocks last
        rec = g.fuse_frames(s.frame_ptr(k), w2c[k:k + 200])
        k += 200
        assert (rec["alloc_failed_type1"] == 0).all(), "failed before the hand-off"
        if rec["lastFreeBlockId"][-1] < 1200:
            break
    assert k < N - 400, "the walk did not approach saturation"
    o = oracle_mod.Oracle(_params(oracle_mod), omp=True)
    _handoff(g, o, False)
    _compare_all(f"hand-off at frame {k}", g, o, False)
    first_fail, f1_tot, f2_tot = None, 0, 0
    while first_fail is None or k < first_fail + 40:
        assert k < N, "no allocation failure within the rendered frames"
        rec = g.fuse_frames(s.frame_ptr(k), w2c[k:k + 1])[0]
        _oracle_frame(o, s.download(k, 1)[0], w2c[k], False)
        tag = f"C5E frame {k}"
        _check_record(tag, rec, o, False)
        assert_bit_exact(f"{tag} visible_type", g.visible_type(), o.visible_type())
        f1, f2 = o.alloc_failures()
        f1_tot, f2_tot = f1_tot + f1, f2_tot + f2
        if first_fail is None and f1 + f2 > 0:
            first_fail = k
            _compare_all(f"{tag} (first failure)", g, o, False)
        elif k % 16 == 0:
            _compare_all(tag, g, o, False)
        k += 1
    _compare_all(f"C5E frame {k - 1}", g, o, False)
    assert g.stats()["lastFreeBlockId"] == -1          # the VBA is full: 65 536 blocks allocated
    assert f1_tot > 0 and f2_tot > 0                     # both kinds of request fail once blocks run out
    s.free()
    g.close()


def _prefill_far(n_buckets, n_excess, excess_left):
    """A hash table of 'swapped-out' entries (ptr -1) far below the hall (block y = 300), as many
    as leave `excess_left` excess entries free -- the walk's new blocks then exhaust the excess
    list.  Returns (table, lastFreeExcessListId)."""
    from topfusion_amd.topfu import HASH_DTYPE
    xs, zs = np.meshgrid(np.arange(-400, 400), np.arange(-400, 400), indexing="ij")
    pos = np.stack([xs.ravel(), np.full(xs.size, 300), zs.ravel()], 1)
    pos = pos[np.random.default_rng(5).permutation(len(pos))]
    hb = synth.hash_index(pos[:, 0], pos[:, 1], pos[:, 2], n_buckets)
    _, first = np.unique(hb, return_index=True)
    is_first = np.zeros(len(pos), bool)
    is_first[first] = True
    n_ex = np.arange(1, len(pos) + 1) - np.cumsum(is_first)      # excess entries a prefix needs
    L = int(np.searchsorted(n_ex, n_excess - excess_left, side="right"))
    h, _, last_free_excess = synth.build_hash(pos[:L], n_buckets, n_excess, HASH_DTYPE)
    h["ptr"][h["ptr"] >= 0] = -1
    return h, last_free_excess


@pytest.mark.parametrize("swapping", [False, True])
def test_c5e_prefilled_capacity(oracle_mod, swapping):
    """Both capacities nearly spent before the walk starts: ~500 k swapped-out entries far away
    hold all but 60 excess entries, and only 300 voxel blocks are free.  The first frames exhaust
    both, with and without the swapping engine (whose evictions then free blocks for later
    frames); 64 frames, every frame's counters / failures / swap counts / visible types and the
    whole scene every 16 frames compared."""
    from topfusion_amd import TopFu, _lib as L
    n = 64
    R, t, w2c = _walk(n)
    s = synth.DeviceStream(n, W, H)
    synth.render_hall_device(s, R, t)
    frames = s.download(0, n)
    pg = _params(L, swapping)
    g = TopFu(pg)
    o = oracle_mod.Oracle(_params(oracle_mod, swapping), omp=True)
    h, lfe = _prefill_far(pg.n_buckets, pg.n_excess, 60)
    g.upload(L.TF_BUF_HASH, h)
    o.upload_hash(h)
    g.set_counters(300, lfe, 0)
    o.set_counters(300, lfe, 0)
    fails = np.zeros((n, 2), np.int64)
    for k in range(n):
        rec = g.fuse_frames(s.frame_ptr(k), w2c[k:k + 1])[0]
        _oracle_frame(o, frames[k], w2c[k], swapping)
        tag = f"prefilled{' swapping' if swapping else ''} frame {k}"
        _check_record(tag, rec, o, swapping)
        assert_bit_exact(f"{tag} visible_type", g.visible_type(), o.visible_type())
        fails[k] = o.alloc_failures()
        if k % 16 == 15:
            _compare_all(tag, g, o, swapping)
    assert fails[:, 0].sum() > 0 and fails[:, 1].sum() > 0, fails.sum(0)
    assert g.stats()["lastFreeExcessListId"] == -1 or fails[:, 1].sum() > 0
    s.free()
    g.close()
