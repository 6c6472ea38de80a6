"""GPU parity of the colour TSDF: Voxel_s_rgb voxels (VoxelTypes.hpp:39-67)
whose colour half is updated by computeUpdatedVoxelColorInfo (SceneReconstructionEngine.hpp:
116-148) with interpolateBilinear (PixelUtils.hpp:8-32) where the lineage's
ComputeUpdatedVoxelInfo<true, ...> (:163-176) calls it, through M_rgb = calib_inv * M_d
(SceneReconstructionEngine_host.cu:217); and RenderImage's RENDER_COLOUR_FROM_VOLUME
(renderColour_device, VisualisationEngine_CUDA.cu:254-256; readFromSDF_color4u_interpolated,
RepresentationAccess.hpp:260-294).  Every comparison against the oracle, bit for bit.

The reference's colour call sites are commented out (ComputeUpdatedVoxelInfo<true, ...>,
the rgb arguments of IntegrateIntoScene), so these results are pinned to the oracle's
restatement of the functions the reference does hold."""
import ctypes

import numpy as np
import pytest

from parity_util import DeviceBuffer, DeviceFrames, assert_bit_exact, assert_struct_exact, hash_block_set
from topfusion_amd import synth

pytestmark = pytest.mark.gpu

# a colour camera 2.5 cm beside the depth camera, turned by 1 deg, with its own intrinsics
_A = np.deg2rad(1.0)
D_RT = np.array([[np.cos(_A), 0, np.sin(_A), 0.025], [0, 1, 0, 0.0], [-np.sin(_A), 0, np.cos(_A), 0.004]], np.float32)


def _rgb_intr(W, H):
    fx, fy, cx, cy = synth.intrinsics(W, H)
    return (fx * 1.03, fy * 1.03, cx - 3.5, cy + 2.25)


def _params(oracle_mod, W, H, registered=False, **kw):
    from topfusion_amd import default_params
    fx, fy, cx, cy = synth.intrinsics(W, H)
    args = dict(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy, voxel_rgb=1, **kw)
    if not registered:
        args.update(rgb_intr=_rgb_intr(W, H), depth_to_rgb=D_RT.reshape(12))
    return default_params(**args), oracle_mod.default_params(**args)


def _colour_view(R_d, t_d, W, H, registered=False):
    """The RGB image the colour camera sees when the depth camera is at (R_d, t_d) (camera ->
    world): X_rgb = D X_d, so the colour camera's pose is c2w_d * D^-1."""
    if registered:
        return synth.render_colour(R_d, t_d, W, H)
    RD, tD = D_RT[:, :3].astype(np.float64), D_RT[:, 3].astype(np.float64)
    R = R_d @ RD.T
    t = t_d - R @ tD
    return synth.render_colour(R, t, W, H, intr=_rgb_intr(W, H))


def _compare_scene(g, o, tag):
    hg, ho = g.hash(), o.hash()
    assert hash_block_set(hg) == hash_block_set(ho), f"{tag} block sets"
    assert_struct_exact(f"{tag} hash", hg, ho, ["x", "y", "z", "offset", "ptr"])
    assert_struct_exact(f"{tag} vba", g.vba(), o.vba(), ["sdf", "w"])
    cg, co = g.vba_rgb(), o.vba_rgb()
    assert_bit_exact(f"{tag} colour plane", cg, co)
    return co


def test_colour_engine_path(oracle_mod):
    """SceneReconstructionEngine_CUDA::{AllocateSceneFromDepth, IntegrateIntoScene + rgb} at the
    orbit's ground-truth poses with an unregistered colour camera (own intrinsics, 2.5 cm / 1 deg
    off), pitched caller buffers; then RenderImage(RENDER_COLOUR_FROM_VOLUME) from new raycasts."""
    from topfusion_amd import TopFu, _lib
    from test_gpu_engines import Pitched, _f, _ok
    L = _lib.load()
    W, H = 320, 240
    pg, po = _params(oracle_mod, W, H)
    g, o = TopFu(pg), oracle_mod.Oracle(po)
    fx, fy, cx, cy = synth.intrinsics(W, H)
    intr = np.array([fx, fy, cx, cy], np.float32)
    dists = Pitched(H, W, np.float32)
    rgbb = Pitched(H, W, np.uint8, 4)
    for k in (0, 6, 12, 18, 24):
        R, t = synth.orbit_pose(k)
        c2w = np.zeros((3, 4), np.float32)
        c2w[:, :3], c2w[:, 3] = R, t
        w2c = oracle_mod.rigid_inv(c2w)
        dd = oracle_mod.compute_dists(synth.render_depth(R, t, W, H, noise_mm=1.0, seed=300 + k))
        rgb = _colour_view(R, t, W, H)
        dists.put(dd)
        rgbb.put(rgb)
        _ok(L.tf_scene_alloc(g._h, _f(intr), _f(w2c), dists.ptr, dists.step, 0, 0), "tf_scene_alloc")
        o.alloc(w2c, dd)
        _ok(L.tf_scene_integrate_rgb(g._h, _f(intr), _f(w2c), dists.ptr, dists.step, ctypes.c_void_p(rgbb.ptr),
                                     rgbb.step), "tf_scene_integrate_rgb")
        o.integrate(w2c, dd, rgb)
        co = _compare_scene(g, o, f"pose {k}")
    coloured = int(((co >> 24) > 0).sum())
    assert coloured > 10000, coloured
    assert int((co >> 24).max()) >= 4                       # repeated observations averaged
    img = Pitched(H, W, np.uint8, 4)
    for k in (24, 10):
        R, t = synth.orbit_pose(k)
        c2w = np.zeros((3, 4), np.float32)
        c2w[:, :3], c2w[:, 3] = R, t
        _ok(L.tf_vis_render_image(g._h, _f(intr), _f(c2w), 2, 1, img.ptr, img.step), "tf_vis_render_image colour")
        o.raycast(c2w, 0)
        want = np.zeros((H, W, 4), np.uint8)
        o.L.tfo_render_type(o.ctx, _f(c2w.reshape(12)), 2, want.ctypes.data_as(ctypes.c_void_p))
        got = img.get()
        assert_bit_exact(f"RENDER_COLOUR_FROM_VOLUME at pose {k}", got, want)
        lit = want[..., 3] == 255
        assert lit.mean() > 0.5
        # the volume's colour is the scene's: what a camera at this pose would see (a few levels of blur)
        seen = synth.render_colour(R, t, W, H)
        assert np.median(np.abs(want[lit][:, :3].astype(int) - seen[lit][:, :3].astype(int))) <= 4
    for b in (dists, rgbb, img):
        b.free()
    g.close()


def test_colour_tracked_frames(oracle_mod):
    """TopFu::operator()(depth, image) on a colour context, frame by frame: device frames through
    tf_process_frame_rgb (a registered colour camera, the Kinect-style default), host frames
    through tf_process_frame_rgb_host; per-frame bool, counters, pose, range image, raycast and
    ICP maps, the scene and its colour plane, and the colour render of the last pose."""
    from topfusion_amd import TopFu
    from test_gpu_parity import _compare_frame_state
    W, H, n = 320, 240, 12
    for registered in (True, False):
        pg, po = _params(oracle_mod, W, H, registered=registered)
        g, o = TopFu(pg), oracle_mod.Oracle(po)
        seq = synth.orbit_sequence(n, W, H, seed=7)
        rgbs = np.stack([_colour_view(*synth.orbit_pose(k), W, H, registered=registered) for k in range(n)])
        dev_d, dev_c = DeviceFrames(seq), DeviceFrames(rgbs)
        for k in range(n):
            if k % 2 == 0:
                okg = g(dev_d.ptr + k * W * H * 2, rgb=dev_c.ptr + k * W * H * 4)
            else:
                okg = g(seq[k], rgb=rgbs[k])
            oko = o(seq[k], rgbs[k])
            assert okg == oko, f"frame {k}: gpu {okg} oracle {oko}"
            _compare_frame_state(g, o, f"registered={registered} frame {k}", grey=bool(oko) and k > 0)
        _compare_scene(g, o, f"registered={registered} final")
        got = g.renderImage(2)
        want = o.render_image_type(2)
        assert_bit_exact(f"registered={registered} renderImage colour", got, want)
        assert (want[..., 3] == 255).mean() > 0.5
        dev_d.free()
        dev_c.free()
        g.close()


def test_colour_batched_frames(oracle_mod):
    """tf_process_frames_rgb: 36 frames (two enqueue groups, two-frame lookahead, the orbit's
    ICP-failure resets at frames 9, 19 and 30 clearing the colour plane with the scene) at
    640x480, final state bit-exact with the oracle run frame by frame, including the whole
    colour plane."""
    from topfusion_amd import TopFu
    from test_gpu_parity import _compare_frame_state
    W, H, n = 640, 480, 36
    pg, po = _params(oracle_mod, W, H)
    g, o = TopFu(pg), oracle_mod.Oracle(po)
    seq = synth.orbit_sequence(n, W, H, seed=7)
    rgbs = np.stack([_colour_view(*synth.orbit_pose(k), W, H) for k in range(n)])
    dev_d, dev_c = DeviceFrames(seq), DeviceFrames(rgbs)
    okg = g.process_frames(dev_d.ptr, n, rgb_frames=dev_c.ptr)
    oko = np.array([o(seq[k], rgbs[k]) for k in range(n)])
    assert np.array_equal(okg, oko), (okg, oko)
    assert oko[-1] and (~oko).sum() >= 2, oko
    _compare_frame_state(g, o, "batched colour", grey=True)
    co = _compare_scene(g, o, "batched colour final")
    assert int(((co >> 24) > 0).sum()) > 10000
    dev_d.free()
    dev_c.free()
    g.close()


def test_colour_argument_checks():
    """An RGB image on a Voxel_s context, or a swapping colour context (the GlobalCache holds
    Voxel_s blocks), is TF_INVALID_ARG; RENDER_COLOUR_FROM_VOLUME on Voxel_s is greyscale."""
    from topfusion_amd import TopFu, default_params
    from topfusion_amd import _lib as L
    lib = L.load()
    W, H = 320, 240
    fx, fy, cx, cy = synth.intrinsics(W, H)
    g = TopFu(default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy))
    d = synth.orbit_sequence(1, W, H, seed=7)[0]
    rgb = np.zeros((H, W, 4), np.uint8)
    s = lib.tf_process_frame_rgb_host(g._h, d.ctypes.data_as(ctypes.c_void_p), W * 2,
                                           rgb.ctypes.data_as(ctypes.c_void_p), W * 4, None, None)
    assert s == L.TF_INVALID_ARG
    g(d)
    assert g(synth.orbit_sequence(2, W, H, seed=7)[1])
    assert_bit_exact("colour-from-volume on Voxel_s", g.renderImage(2), g.renderImage(0))
    g.close()
    p = default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy, voxel_rgb=1, use_swapping=1)
    h = ctypes.c_void_p()
    assert lib.tf_create(ctypes.byref(p), ctypes.byref(h)) == L.TF_INVALID_ARG
