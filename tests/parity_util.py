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


class DeviceFrames:
    """Device copy of a host array through the HIP runtime libtfusion_hip.so itself links
    (no torch: torch ships its own HIP runtime, and two runtimes in one process do not share
    a device context in every initialisation order)."""

    def __init__(self, arr):
        import ctypes
        from topfusion_amd import _lib
        _lib.load()                                   # the product library (and its libamdhip64)
        self._hip = ctypes.CDLL("libamdhip64.so.7")
        a = np.ascontiguousarray(arr)
        self.nbytes = a.nbytes
        p = ctypes.c_void_p()
        assert self._hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(a.nbytes)) == 0, "hipMalloc"
        self.ptr = p.value
        assert self._hip.hipMemcpy(ctypes.c_void_p(self.ptr), a.ctypes.data_as(ctypes.c_void_p),
                                   ctypes.c_size_t(a.nbytes), 1) == 0, "hipMemcpy H2D"   # hipMemcpyHostToDevice

    def free(self):
        import ctypes
        if self.ptr:
            self._hip.hipFree(ctypes.c_void_p(self.ptr))
            self.ptr = None


class DeviceBuffer(DeviceFrames):
    """A device allocation of `nbytes` (zero-filled), with host <-> device copies; 2-D copies
    with a row step (bytes) for pitched layouts."""

    def __init__(self, nbytes):
        super().__init__(np.zeros(int(nbytes), np.uint8))

    def upload2d(self, arr, step):
        import ctypes
        a = np.ascontiguousarray(arr)
        rows = a.shape[0]
        row_bytes = a.nbytes // rows
        assert step * rows <= self.nbytes and row_bytes <= step
        assert self._hip.hipMemcpy2D(ctypes.c_void_p(self.ptr), ctypes.c_size_t(step), a.ctypes.data_as(ctypes.c_void_p),
                                     ctypes.c_size_t(row_bytes), ctypes.c_size_t(row_bytes), ctypes.c_size_t(rows), 1) == 0

    def download2d(self, shape, dtype, step):
        import ctypes
        out = np.empty(shape, dtype)
        rows = shape[0]
        row_bytes = out.nbytes // rows
        assert self._hip.hipMemcpy2D(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(row_bytes), ctypes.c_void_p(self.ptr),
                                     ctypes.c_size_t(step), ctypes.c_size_t(row_bytes), ctypes.c_size_t(rows), 2) == 0
        return out

    def sync(self):
        assert self._hip.hipDeviceSynchronize() == 0
