"""GPU parity at the benchmark configurations' own sizes, on the bench's own
inputs (bench.py builds them), against the OpenMP build of the oracle:

* C3 at 2^21 - 1 active blocks (4 GiB of voxels, 1280x960, 2 mm): the C3I / C3R scene
  (bench.c3_scene: every block in the visible list), two IntegrateIntoScene passes
  (SceneReconstructionEngine.hpp:23-71) and one k_raycast_pair launch -- CreateICPMaps'
  castRay<true> + renderImage's castRay + grey (VisualisationEngine_Shared.hpp:99-172) -- with
  the whole VBA, the raycast, the grey image and the visibility marks bit-exact.
* C5 at 640x480, 10 mm, the seed-13 random walk rendered on the GPU as the bench renders it, the
  bench's 32-frame tf_process_frames steps, swapping off and on (GlobalCache in HBM at the
  reference capacities, SDF_TRANSFER_BLOCK_NUM blocks per direction)."""
import numpy as np
import pytest

from parity_util import assert_bit_exact, assert_struct_exact
from topfusion_amd import synth

pytestmark = pytest.mark.gpu


def test_c3_two_million_blocks_integrate_raycast(oracle_mod):
    import bench
    from topfusion_amd import _lib as L
    g, p, W, H, vox, nb, ids, last_free_excess = bench.c3_scene()
    assert nb == (1 << 21) - 1
    fx, fy, cx, cy = synth.intrinsics(W, H)
    o = oracle_mod.Oracle(oracle_mod.default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy, voxelSize=vox,
                                                    **bench.C3_CAPACITY), omp=True)
    o.upload_hash(g.hash())
    o.upload_visible_ids(ids)
    o.set_counters(-1, last_free_excess, nb)
    wall = np.full((H, W), 1500, np.uint16)
    dists = oracle_mod.compute_dists(wall)
    assert_bit_exact("C3 dists", g.dists(), dists)
    I = np.eye(4, dtype=np.float32)[:3]
    for k in range(2):
        g.time_stage("integrate", I, 1)
        o.integrate(I, dists)
    vg = g.vba()
    vo = o.vba()
    touched = int((vo["w"] > 0).sum())
    assert touched > 10_000_000, touched               # the wall's band crosses many blocks
    assert_struct_exact("C3 VBA after 2 passes", vg, vo, ["sdf", "w"])
    del vg, vo
    # the C3R raycast pair from the range image RenderState starts with, visibility cleared
    rng = np.empty((H, W, 2), np.float32)
    rng[..., 0], rng[..., 1] = p.viewFrustum_min, p.viewFrustum_max
    g.upload(L.TF_BUF_RANGE, rng)
    g.upload(L.TF_BUF_VISIBLE_TYPE, np.zeros(g.nbytes(L.TF_BUF_VISIBLE_TYPE), np.uint8))
    g.time_stage("raycast_render", I, 1)
    o.raycast(I, 1)
    grey_o = o.render_grey(I)
    ray_g = g.raycast_result()
    assert (ray_g[..., 3] > 0).mean() > 0.9             # the wall is hit
    assert_bit_exact("C3 raycast", ray_g, o.raycast_result())
    assert_bit_exact("C3 grey", g.frame_grey(), grey_o)
    assert_bit_exact("C3 visibility marks", g.visible_type(), o.visible_type())
    g.close()


def _c5_compare(g, o, tag, swapping):
    from test_gpu_parity import _compare_frame_state, compare_scene
    _compare_frame_state(g, o, tag, grey=False)
    compare_scene(g, o, tag)
    if swapping:
        assert_bit_exact(f"{tag} swap state", g.swap_state(), o.swap_state())
        fg, fo = g.swap_stored_flags(), o.swap_stored_flags()
        assert_bit_exact(f"{tag} stored flags", fg, fo)
        ids = np.nonzero(fo)[0]
        if len(ids):
            sg = g.swap_stored().reshape(-1, 512)[ids]
            so = o.swap_stored().reshape(-1, 512)[ids]
            assert_struct_exact(f"{tag} stored blocks", sg, so, ["sdf", "w"])


@pytest.mark.parametrize("swapping", [False, True])
def test_c5_bench_frames_640x480(oracle_mod, swapping):
    import bench
    from topfusion_amd import TopFu, default_params
    W, H, F, steps = 640, 480, 32, 2
    dev = bench.walk_frames(steps * F, W, H, 13)
    host = dev.download(0, steps * F)
    fx, fy, cx, cy = synth.intrinsics(W, H)
    args = dict(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy, voxelSize=0.01)
    if swapping:
        args.update(use_swapping=1, swap_transfer_blocks=0x1000)
    g = TopFu(default_params(**args))
    o = oracle_mod.Oracle(oracle_mod.default_params(**args), omp=True)
    fb = W * H * 2
    swapped_out = 0
    for s in range(steps):
        okg = g.process_frames(dev.ptr + s * F * fb, F)
        oko = []
        for k in range(s * F, (s + 1) * F):
            oko.append(o(host[k]))
            if swapping:
                swapped_out += o.swap_counts()[1]
        oko = np.array(oko)
        assert np.array_equal(okg, oko), (s, okg, oko)
        _c5_compare(g, o, f"C5 640x480 frames {s * F}..{(s + 1) * F - 1}", swapping)
    if swapping:
        assert swapped_out > 0                          # blocks left the enlarged frustum and were evicted
        assert g.totals()["swapped_out"] == swapped_out
        assert g.totals()["swapped_in_merged"] == o.swap_merged_total()
    g.close()
    dev.free()
