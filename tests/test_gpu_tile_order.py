"""The raycast tiles' dispatch order (k_raycast_pair's longest-first order, tf_ctx::tile_order) is a
schedule only: with it on (the default), off (TFUSION_TILE_ORDER=0) or with the XCD shares as
interleaved tile rows (TFUSION_TILE_MAP=rows), every frame of the bench's C2 stream gives the same
bits as the oracle -- range image, raycast, grey image, visibility types, ICP maps, poses and
scene.  The order is built from the previous frames' workgroup times, so the frames after the
first few run on a reordered grid."""
import numpy as np
import pytest

from test_gpu_parity import _compare_frame_state, compare_scene, make_pair
from topfusion_amd import synth

pytestmark = pytest.mark.gpu

W, H, N = 640, 480, 12


@pytest.mark.parametrize("env", [{}, {"TFUSION_TILE_ORDER": "0"}, {"TFUSION_TILE_MAP": "rows"}],
                         ids=["longest-first", "plain", "rows"])
def test_tile_order_is_a_schedule(oracle_mod, monkeypatch, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g, o = make_pair(oracle_mod, W, H)
    frames = synth.orbit_sequence(N, W, H, seed=7)
    dev = synth.DeviceStream(N, W, H)
    dev.upload(frames)
    tracked = 0
    for k in range(N):                    # one frame per batch: every frame's state is compared
        okg = bool(g.process_frames(dev.frame_ptr(k), 1)[0])
        oko = bool(o(frames[k]))
        assert okg == oko, (k, okg, oko)
        tracked += okg and k > 0
        _compare_frame_state(g, o, f"frame {k} {env}", grey=oko)
    assert tracked >= 6
    compare_scene(g, o, f"{env}")
    g.close()
    dev.free()
