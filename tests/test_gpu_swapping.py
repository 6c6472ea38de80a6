"""GPU parity of voxel-block swapping: the GlobalCache in HBM, the swapping
branches of AllocateSceneFromDepth (enlarged frustum, swap-state marking,
reAllocateSwappedOutVoxelBlocks; SceneReconstructionEngine_host.cu:159-189, 417-479) and the
swapping engine of the lineage (IntegrateGlobalIntoLocal / SaveToGlobalMemory, DESIGN.md
§Swapping), against the oracle's restatement, bit for bit: hash, free list, visible list and
types, VBA, swap states, stored flags, stored blocks and the per-call transfer counts.

The engine's algorithm is not in the reference tree (CUDAInstantiations.cu:8 comments
ITMSwappingEngine_CUDA out), so these results are pinned to the oracle's restatement only."""
import os
import tempfile

import numpy as np
import pytest

from parity_util import assert_bit_exact, assert_struct_exact, hash_block_set
from topfusion_amd import synth

pytestmark = pytest.mark.gpu

CENTRE = np.array([0.15, -0.15, 0.6])      # inside the room, clear of the sphere
SMALL_HASH = dict(n_buckets=0x8000, n_excess=0x2000)


def _yaw_pose(deg):
    """camera -> world: rotation about the vertical axis through CENTRE (float64)."""
    a = np.deg2rad(deg)
    c, s = np.cos(a), np.sin(a)
    R = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    return R, CENTRE.copy()


def _rt32(R, t):
    m = np.zeros((3, 4), np.float32)
    m[:, :3], m[:, 3] = R, t
    return m


def _pair(oracle_mod, W, H, **kw):
    from topfusion_amd import TopFu, default_params
    fx, fy, cx, cy = synth.intrinsics(W, H)
    args = dict(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy, use_swapping=1, **kw)
    return TopFu(default_params(**args)), oracle_mod.Oracle(oracle_mod.default_params(**args))


def _compare(g, o, tag, stored=False):
    hg, ho = g.hash(), o.hash()
    assert hash_block_set(hg) == hash_block_set(ho), f"{tag} block sets"
    assert_struct_exact(f"{tag} hash", hg, ho, ["x", "y", "z", "offset", "ptr"])
    sg, so = g.stats(), o.counters()
    for k in ("lastFreeBlockId", "lastFreeExcessListId", "noVisibleEntries"):
        assert sg[k] == so[k], f"{tag} {k}: gpu {sg[k]} oracle {so[k]}"
    assert_bit_exact(f"{tag} visible ids", g.visible_ids(), o.visible_ids())
    assert_bit_exact(f"{tag} visible types", g.visible_type(), o.visible_type())
    assert_struct_exact(f"{tag} vba", g.vba(), o.vba(), ["sdf", "w"])
    assert_bit_exact(f"{tag} swap state", g.swap_state(), o.swap_state())
    fg, fo = g.swap_stored_flags(), o.swap_stored_flags()
    assert_bit_exact(f"{tag} stored flags", fg, fo)
    if stored:
        ids = np.nonzero(fo)[0]
        sgv = g.swap_stored().reshape(-1, 512)[ids]
        sov = o.swap_stored().reshape(-1, 512)[ids]
        assert_struct_exact(f"{tag} stored blocks", sgv, sov, ["sdf", "w"])
    return hg


def _invariants(h, n_blocks, last_free, flags, state):
    """Free-list bookkeeping a swapped scene must keep: every live block held once, the free
    count + live blocks = capacity, swapped-out entries (ptr -1) stored and in state 0/1."""
    live = h["ptr"][h["ptr"] >= 0]
    assert len(np.unique(live)) == len(live), "a VBA block held twice"
    assert last_free + 1 + len(live) == n_blocks, (last_free, len(live), n_blocks)
    out = np.nonzero(h["ptr"] == -1)[0]
    assert flags[out].all(), "a swapped-out entry without stored data"
    assert (state[out] != 2).all(), "a swapped-out entry marked active"


@pytest.mark.parametrize("n_blocks,transfer,split", [(8192, 1024, False), (2600, 96, False), (2600, 96, True)])
def test_swapping_engine_path(oracle_mod, n_blocks, transfer, split):
    """A camera turning in place through 400 deg and back (40 deg a frame, ground-truth poses)
    over SceneReconstructionEngine_CUDA::{AllocateSceneFromDepth, IntegrateIntoScene} + the
    swapping engine, with a VBA too small for the room (blocks must be evicted to make room)
    and a transfer cap below the per-frame demand (backlogs carry over).  The small case also
    runs the free list dry, so swapped-out entries stay without a block (state 1, ptr -1).
    split: IntegrateGlobalIntoLocal and SaveToGlobalMemory as two calls (tf_scene_swap_in /
    _out, as a SwappingEngine caller makes them) against the oracle's two halves."""
    import ctypes
    from topfusion_amd import _lib
    L = _lib.load()
    W, H = 320, 240
    g, o = _pair(oracle_mod, W, H, n_blocks=n_blocks, swap_transfer_blocks=transfer, vis_capacity=65536, **SMALL_HASH)
    fx, fy, cx, cy = synth.intrinsics(W, H)
    intr = np.array([fx, fy, cx, cy], np.float32)
    from test_gpu_engines import Pitched, _f, _ok
    dists = Pitched(H, W, np.float32)
    angles = list(range(0, 400, 40)) + list(range(360, -1, -40))
    tot = np.zeros(3, np.int64)
    merged = 0
    for k, deg in enumerate(angles):
        R, t = _yaw_pose(deg)
        depth = synth.render_depth(R, t, W, H, noise_mm=1.0, seed=1000 + k)
        dd = oracle_mod.compute_dists(depth)
        w2c = oracle_mod.rigid_inv(_rt32(R, t))
        dists.put(dd)
        _ok(L.tf_scene_alloc(g._h, _f(intr), _f(w2c), dists.ptr, dists.step, 0, 0), "tf_scene_alloc")
        o.alloc(w2c, dd)
        _ok(L.tf_scene_integrate(g._h, _f(intr), _f(w2c), dists.ptr, dists.step), "tf_scene_integrate")
        o.integrate(w2c, dd)
        flags_before = o.swap_stored_flags()
        state_before = o.swap_state()
        if split:
            g.swap_in()
            o.swap_in()
            assert g.swap_counts()[0] == o.swap_counts()[0], f"frame {k} swapped in"
            g.swap_out()
            o.swap_out()
        else:
            g.swap()
            o.swap()
        cg, co = g.swap_counts(), o.swap_counts()
        assert cg == co, f"frame {k} ({deg} deg) swap counts (in, out, realloc): gpu {cg} oracle {co}"
        tot += co
        # swap-ins that merged stored data this frame
        merged += int(((state_before == 1) & (flags_before == 1) & (o.swap_state() == 2)).sum())
        h = _compare(g, o, f"frame {k} ({deg} deg)", stored=(k % 5 == 4 or k == len(angles) - 1))
        _invariants(h, n_blocks, o.counters()["lastFreeBlockId"], o.swap_stored_flags(), o.swap_state())
    assert tot[0] > 0 and tot[1] > 0 and tot[2] > 0, f"swapped in / out / reallocated: {tot}"
    assert merged > 0, "no stored block was merged back"
    if n_blocks < 4000:
        h = o.hash()
        assert ((h["ptr"] == -1) & (o.swap_state() == 1)).any(), "free list never ran dry"
    dists.free()
    g.close()


def _back_and_forth(n_out):
    """orbit angles 0 .. n_out-1 frames at 1 deg / frame, then back to 0"""
    return [float(k) for k in range(n_out)] + [float(k) for k in range(n_out - 2, -1, -1)]


def test_swapping_tracked_frames(oracle_mod):
    """TopFu::operator() with a swapping scene (Scene(params, true)): ICP, the enlarged-frustum
    allocation, integration, the swapping engine and the raycasts, frame by frame over an
    orbit that swings 30 deg out and back at 1 deg a frame, through tf_process_frame (the
    reference's ICP fails every ~7 frames on this orbit -- the same resets with and without
    swapping -- and each reset empties the cache); per-frame results, pose,
    counters and range image each frame, the whole scene + GlobalCache at checkpoints, and the
    device totals against the oracle's per-frame transfer counts."""
    from test_gpu_parity import _compare_frame_state
    W, H = 320, 240
    g, o = _pair(oracle_mod, W, H, n_blocks=12288, swap_transfer_blocks=1024, **SMALL_HASH)
    angles = _back_and_forth(31)
    tin = tout = 0
    for k, deg in enumerate(angles):
        R, t = synth.orbit_pose(1, deg_per_frame=deg)
        d = synth.render_depth(R, t, W, H, noise_mm=1.0, seed=7000 + k)
        okg, oko = g(d), o(d)
        assert okg == oko, f"frame {k}: gpu {okg} oracle {oko}"
        c = o.swap_counts()
        tin, tout = tin + c[0], tout + c[1]
        assert g.swap_counts() == c, f"frame {k} swap counts: gpu {g.swap_counts()} oracle {c}"
        _compare_frame_state(g, o, f"frame {k}", grey=bool(oko) and k > 0)
        if k % 15 == 14:
            _compare(g, o, f"frame {k}", stored=True)
    _compare(g, o, "final", stored=True)
    tg = g.totals()
    assert (tg["swapped_in"], tg["swapped_out"]) == (tin, tout), (tg, tin, tout)
    assert tout > 0 and tin > 0, (tin, tout)
    g.close()


def test_swapping_batched_and_save_load(oracle_mod):
    """The batch path (tf_process_frames, two-frame lookahead) with swapping: final state
    bit-exact; then the GlobalCache saved to a file and loaded into a fresh context."""
    from parity_util import DeviceFrames
    from topfusion_amd import TopFu
    W, H = 320, 240
    g, o = _pair(oracle_mod, W, H, n_blocks=12288, swap_transfer_blocks=1024, **SMALL_HASH)
    angles = _back_and_forth(21)
    seq = np.stack([synth.render_depth(*synth.orbit_pose(1, deg_per_frame=a), W, H, noise_mm=1.0, seed=9000 + k)
                    for k, a in enumerate(angles)])
    dev = DeviceFrames(seq)
    okg = g.process_frames(dev.ptr, len(angles))
    oko = np.array([o(seq[k]) for k in range(len(angles))])
    assert np.array_equal(okg, oko), (okg, oko)
    dev.free()
    # the reference's frame-mixing resets empty the GlobalCache: where the sequence ended on one,
    # the orbit continues (one-frame batches) until blocks are stored again, so save / load has data
    k = len(angles)
    while o.swap_stored_flags().sum() == 0 and k < len(angles) + 40:
        d = synth.render_depth(*synth.orbit_pose(1, deg_per_frame=float(k - len(angles))), W, H, noise_mm=1.0, seed=9000 + k)
        one = DeviceFrames(d[None])
        assert bool(g.process_frames(one.ptr, 1)[0]) == o(d), k
        one.free()
        k += 1
    _compare(g, o, "batched final", stored=True)
    assert o.swap_stored_flags().sum() > 0
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "cache.bin")
        g.swap_save(path)
        assert os.path.getsize(path) == g.n_total * (1 + 512 * 4)
        g2 = TopFu(g.params())
        g2.swap_load(path)
        assert_bit_exact("loaded stored flags", g2.swap_stored_flags(), g.swap_stored_flags())
        assert_bit_exact("loaded store", g2.swap_stored().view(np.uint32), g.swap_stored().view(np.uint32))
        g2.close()
    g.close()


def test_swapping_c5_random_walk(oracle_mod):
    """C5 geometry (10 mm voxels, the seed-13 random walk) on a swapping scene whose VBA runs
    out (2048 blocks): allocation saturates, out-of-view blocks are evicted to the cache at
    the transfer cap, and the walk's ICP-failure resets (the reference's own, as without
    swapping) empty it; every frame's result, counters, transfer counts and pose against the
    oracle, the whole scene + GlobalCache after an eviction frame and at the end."""
    W, H, n = 320, 240, 24
    g, o = _pair(oracle_mod, W, H, voxelSize=0.01, n_blocks=2048, swap_transfer_blocks=256,
                 n_buckets=0x10000, n_excess=0x4000)
    seq = synth.random_walk_sequence(n, W, H, seed=13)
    outs = 0
    for k in range(n):
        okg, oko = g(seq[k]), o(seq[k])
        assert okg == oko, f"frame {k}: gpu {okg} oracle {oko}"
        sg, so = g.last_stats, o.counters()
        for key in ("lastFreeBlockId", "lastFreeExcessListId", "noVisibleEntries", "icp_iterations", "frame_counter",
                    "n_resets"):
            assert sg[key] == so[key], f"frame {k} {key}: gpu {sg[key]} oracle {so[key]}"
        c = o.swap_counts()
        assert g.swap_counts() == c, f"frame {k} swap counts: gpu {g.swap_counts()} oracle {c}"
        outs += c[1]
        assert_bit_exact(f"frame {k} pose", g.getCameraPose()[:3, :4], o.pose())
        if c[1] and o.swap_stored_flags().any():
            _compare(g, o, f"frame {k} (evicted {c[1]})", stored=True)
    _compare(g, o, "C5 swapping final", stored=True)
    assert outs > 0 and o.counters()["n_resets"] >= 1
    tg = g.totals()
    assert tg["swapped_out"] == outs, (tg, outs)
    assert tg["swapped_in_merged"] == o.swap_merged_total(), (tg, o.swap_merged_total())
    g.close()


def test_engine_reset_scene_keeps_global_cache(oracle_mod):
    """SceneReconstructionEngine::ResetScene (SceneReconstructionEngine_host.cu:51-73) clears the
    hash, the VBA and the free lists but leaves the GlobalCache alone, as the reference's does
    (the TopFu-level resets -- construction, TopFu::reset, the ICP-failure reset -- empty it so no
    block of the old scene is swapped into the new one).  After evictions, the engine reset keeps
    every stored flag and block, bit-exact with the oracle, and the frames after it still match."""
    W, H = 320, 240
    g, o = _pair(oracle_mod, W, H, voxelSize=0.01, n_blocks=2048, swap_transfer_blocks=256,
                 n_buckets=0x10000, n_excess=0x4000)
    seq = synth.random_walk_sequence(22, W, H, seed=13)
    for k in range(16):
        assert g(seq[k]) == o(seq[k]), k
    stored_before = o.swap_stored_flags().copy()
    g.stage_reset_scene()
    o.reset_scene()
    _compare(g, o, "after engine ResetScene", stored=True)
    assert stored_before.sum() > 0
    assert_bit_exact("stored flags kept", g.swap_stored_flags(), stored_before)
    assert g.stats()["lastFreeBlockId"] == 2047
    for k in range(16, 22):
        assert g(seq[k]) == o(seq[k]), k
    _compare(g, o, "frames after the reset", stored=True)
    g.close()
