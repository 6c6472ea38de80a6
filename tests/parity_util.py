"""Comparison helpers for the GPU-vs-oracle parity tests."""
import numpy as np


def same_bits(a, b):
    """Elementwise bit equality; any two NaNs compare equal (NaN payloads differ by ISA)."""
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    if a.dtype.kind == "f":
        ai = a.view(np.uint32 if a.dtype.itemsize == 4 else np.uint64)
        bi = b.view(np.uint32 if b.dtype.itemsize == 4 else np.uint64)
        return (ai == bi) | (np.isnan(a) & np.isnan(b))
    return a == b


def assert_bit_exact(name, got, want, max_report=8):
    eq = same_bits(got, want)
    if not np.all(eq):
        bad = np.argwhere(~eq)
        msg = [f"{name}: {len(bad)} of {eq.size} elements differ"]
        for idx in bad[:max_report]:
            t = tuple(idx)
            msg.append(f"  at {t}: got {np.asarray(got)[t]!r} want {np.asarray(want)[t]!r}")
        raise AssertionError("\n".join(msg))


def assert_struct_exact(name, got, want, fields):
    for f in fields:
        assert_bit_exact(f"{name}.{f}", got[f], want[f])


def hash_block_set(h):
    """Allocated blocks as a sorted set of positions (order-free view of the hash table)."""
    alloc = h[h["ptr"] >= 0]
    return sorted(zip(alloc["x"].tolist(), alloc["y"].tolist(), alloc["z"].tolist()))
