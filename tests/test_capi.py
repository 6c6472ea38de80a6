"""CPU tests of the drop-in boundary: libtfusion_hip.so loads in a GPU-less container,
exports every function include/tfusion_hip.h declares, its structs match the ctypes mirror
byte for byte, and the host-only entry points behave (no compute calls without a GPU)."""
import ctypes
import os
import subprocess
import tempfile

import pytest

from topfusion_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_function():
    L = _lib.load()
    names = _lib.header_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_ctypes_signatures_cover_header():
    """Every declared function has a ctypes signature in topfusion_amd/_lib.py."""
    src = open(_lib.__file__).read()
    for n in _lib.header_functions():
        if n == "tf_debug_icp_ts":
            continue
        assert f'"{n}"' in src, n


def _c_layout(struct, fields):
    prog = "#include <stdio.h>\n#include <stddef.h>\n#include \"tfusion_hip.h\"\nint main(void){\n"
    prog += f'printf("%zu\\n", sizeof({struct}));\n'
    for f in fields:
        prog += f'printf("%zu\\n", offsetof({struct}, {f}));\n'
    prog += "return 0;}\n"
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write(prog)
        exe = os.path.join(d, "l")
        subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    return [int(v) for v in out]


@pytest.mark.parametrize("cls,cname", [(_lib.TfParams, "tf_params"), (_lib.TfStats, "tf_stats")])
def test_struct_layout_matches_header(cls, cname):
    fields = [f for f, _ in cls._fields_]
    got = _c_layout(cname, fields)
    assert got[0] == ctypes.sizeof(cls)
    for f, off in zip(fields, got[1:]):
        assert getattr(cls, f).offset == off, f


def test_default_params_match_reference_defaults():
    """TopFuParams::default_params (topfu.cpp:12-53) via the C-ABI and via the oracle."""
    from oracle import oracle as O
    p = _lib.default_params()
    q = O.default_params()
    for f, _ in _lib.TfParams._fields_:
        a, b = getattr(p, f), getattr(q, f)
        if f == "icp_iter_num":
            assert list(a) == list(b) == [10, 5, 4, 0]
        elif f in ("rgb_intr", "depth_to_rgb"):
            assert list(a) == list(b), f
        else:
            assert a == b, f
    assert (p.cols, p.rows) == (640, 480)
    assert p.voxelSize == pytest.approx(0.005) and p.mu == pytest.approx(0.02) and p.maxW == 100


def test_status_strings_and_invalid_args():
    L = _lib.load()
    assert L.tf_status_string(_lib.TF_OK) == b"ok"
    assert L.tf_status_string(_lib.TF_ICP_FAIL).startswith(b"icp failed")
    assert L.tf_default_params(None) == _lib.TF_INVALID_ARG
    ctx = ctypes.c_void_p()
    assert L.tf_create(None, ctypes.byref(ctx)) == _lib.TF_INVALID_ARG
    bad = _lib.default_params(n_buckets=1000)          # not a power of two
    assert L.tf_create(ctypes.byref(bad), ctypes.byref(ctx)) == _lib.TF_INVALID_ARG


def test_no_silent_cpu_fallback(monkeypatch):
    """The product fails loudly when the HIP library is missing."""
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libtfusion_hip.so")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.load()


def test_product_does_not_import_oracle():
    """Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may touch oracle/."""
    pkg = os.path.join(ROOT, "topfusion_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".h", ".cpp", ".hpp")):
                src = open(os.path.join(dp, f), errors="ignore").read()
                bad = ("import oracle", "from oracle", "tf_oracle.h", "liboracle", "tfo_")
                assert not any(b in src for b in bad), f


def test_random_walk_synth():
    """C5 trajectory: deterministic, steps bounded by 1 cm / 0.5 deg, camera inside the room box;
    the fixed-order room renderer (synth.render_room, what synth/tf_synth.hip renders) agrees with
    the host renderer to the millimetre's rounding without noise."""
    import numpy as np
    from topfusion_amd import synth
    R, t = synth.random_walk_poses(400, seed=13)
    R2, t2 = synth.random_walk_poses(400, seed=13)
    assert np.array_equal(R, R2) and np.array_equal(t, t2)
    assert np.all(t >= synth.ROOM_LO - 1e-12) and np.all(t <= synth.ROOM_HI + 1e-12)
    step = np.linalg.norm(np.diff(t, axis=0), axis=1)
    assert step.max() <= 0.01 + 1e-12
    rel = np.einsum("nij,nkj->nik", R[1:], R[:-1])                  # R_{k+1} R_k^T
    ang = np.degrees(np.arccos(np.clip((np.trace(rel, axis1=1, axis2=2) - 1) / 2, -1, 1)))
    assert ang.max() <= 0.5 + 1e-6
    host = synth.random_walk_sequence(2, 96, 72, seed=13, noise_mm=0.0).astype(np.int64)
    intr = synth.intrinsics(96, 72)
    room = np.stack([synth.render_room(R[k], t[k], 96, 72, 0.0, 13, k, intr=intr) for k in range(2)]).astype(np.int64)
    assert np.abs(host - room).max() <= 1 and (host != room).mean() < 1e-3
    n = synth.hall_noise(7, 3, 320, 240)
    assert abs(n.mean()) < 0.01 and abs(n.std() - 1.0) < 0.01 and np.abs(n).max() <= 2 * synth._SQRT3


def test_entry_points_flush_deferred_frame():
    """A per-call frame leaves its last two launches to the next call (tf_capi.hip flush_tail): every
    other C-ABI entry point that takes a context must enqueue them first (TF_FLUSH), so that it
    sees the whole frame.  Static check of tf_capi.hip: the only entry points without it are the
    per-call frame itself (it flushes with its own frame's lookahead) and the host-only ones."""
    import re
    src = open(os.path.join(ROOT, "topfusion_amd", "csrc", "tf_capi.hip")).read()
    host_only = {"tf_destroy", "tf_get_params", "tf_get_stream", "tf_get_schedule", "tf_get_pose_algebra", "tf_profile_enable",
                 "tf_profile_stages", "tf_profile_sample", "tf_profile_reset", "tf_profile_read"}
    per_call = {"tf_process_frame", "tf_process_frame_host"}
    checked = 0
    for m in re.finditer(r'extern "C" [^(]*\b(tf_\w+)\(([^)]*)\)\s*\{', src):
        name, args = m.group(1), m.group(2)
        if "tf_ctx* c" not in args or name in host_only:
            continue
        body = src[m.end():src.index("\n}", m.end()) if "\n}" in src[m.end():] else len(src)]
        head = body[:400]
        if name in per_call:
            assert "process_frame_early" in head and "TF_FLUSH(c)" in head, name
        else:
            assert "TF_FLUSH(c)" in head, f"{name} does not flush a deferred per-call frame"
        checked += 1
    assert checked >= 40, checked
    # tf_get_stream hands the stream out: a caller synchronising it itself must see whole frames
    gs = src[src.index('extern "C" void* tf_get_stream'):]
    assert "flush_tail(c)" in gs[:300]
