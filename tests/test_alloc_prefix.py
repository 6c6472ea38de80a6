"""The ordered-prefix form of allocateVoxelBlocksList's capacity exhaustion (k_alloc_apply,
topfusion_amd/csrc/tf_scene.hip) against the serial loop it replaces
(SceneReconstructionEngine_host.cu:358-413), on random request sequences: every request's outcome,
its free-list / excess-list slots, the final counters and the failure counts.  The kernel computes
exactly this per request from its chunk prefix counts; the GPU tests check the kernel itself."""
import numpy as np
import pytest


def serial(types, v0, e0):
    """The reference loop: requests in index order, type 1 / 2."""
    v, e = v0, e0
    out = []
    for t in types:
        if t == 1:
            vba = v
            v -= 1
            if vba >= 0:
                out.append((True, vba, None))
            else:
                v += 1
                out.append((False, None, None))
        else:
            vba, exl = v, e
            v -= 1
            e -= 1
            if vba >= 0 and exl >= 0:
                out.append((True, vba, exl))
            else:
                v += 1
                e += 1
                out.append((False, None, None))
    return out, v, e


def prefix(types, v0, e0):
    """k_alloc_apply's per-request decision from prefix counts only."""
    types = np.asarray(types)
    is2 = types == 2
    q = np.concatenate([[0], np.cumsum(is2)[:-1]])              # type-2 requests before k
    g = np.arange(len(types))                                    # requests before k
    S = (g - q) + np.minimum(q, e0 + 1)
    ok = (S <= v0) & (~is2 | (q <= e0))
    out = [(bool(o), int(v0 - s) if o else None, (int(e0 - qq) if (o and t2) else None))
           for o, s, qq, t2 in zip(ok, S, q, is2)]
    f1 = int((~ok & ~is2).sum())
    f2 = int((~ok & is2).sum())
    n = len(types)
    v = v0 - (n - f1 - f2)
    e = e0 - (int(is2.sum()) - f2)
    return out, v, e, f1, f2


@pytest.mark.parametrize("seed", range(40))
def test_prefix_equals_serial(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(0, 400))
    p2 = rng.random()
    types = np.where(rng.random(n) < p2, 2, 1)
    v0 = int(rng.integers(-1, n + 5))
    e0 = int(rng.integers(-1, n + 5))
    want, wv, we = serial(types, v0, e0)
    got, gv, ge, f1, f2 = prefix(types, v0, e0)
    assert got == want
    assert (gv, ge) == (wv, we)
    assert f1 == sum(1 for (o, _, _), t in zip(want, types) if not o and t == 1)
    assert f2 == sum(1 for (o, _, _), t in zip(want, types) if not o and t == 2)


def test_edges():
    for v0, e0 in ((-1, -1), (-1, 5), (5, -1), (0, 0), (3, 100), (100, 2)):
        for types in ([], [1], [2], [2, 2, 1, 1, 2, 1], [1] * 10, [2] * 10):
            want, wv, we = serial(types, v0, e0)
            got, gv, ge, _, _ = prefix(types, v0, e0)
            assert got == want and (gv, ge) == (wv, we), (v0, e0, types)
