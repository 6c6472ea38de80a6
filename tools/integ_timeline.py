"""Workgroup timeline of one frame-path k_integrate launch (diagnostic build: bash
tools/build_variant.sh itl -DTF_INTEG_TIMELINE).  On the GPU box:
  TFUSION_HIP_LIB=tools/_build/itl/libtfusion_hip.so python tools/integ_timeline.py
Runs the C2 orbit, then one tracked frame, and prints the projection and integration workgroups'
start / duration spread and the launch's span."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
from topfusion_amd import TopFu, default_params, synth
from topfusion_amd import _lib
W, H, N0 = 640, 480, 160
fx, fy, cx, cy = synth.intrinsics(W, H)
dev = bench.orbit_frames(N0 + 40, W, H, 7)
tf = TopFu(default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy), device=0)
tf.process_frames(dev.ptr, N0)
k = N0
while True:
    ok = tf.process_frames(dev.frame_ptr(k), 1)
    k += 1
    if ok[0] or k >= N0 + 40:
        break
bench.device_sync()
buf = (ctypes.c_ulonglong * (4096 * 2))()
_lib.load().tf_debug_integ_timeline(buf, ctypes.sizeof(buf))
tl = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 2).astype(np.int64)
n_ed = 256
used = tl[:, 0] > 0
idx = np.nonzero(used)[0]
t0 = tl[used, 0].min()
st = (tl[:, 0] - t0) / 100.0
en = (tl[:, 1] - t0) / 100.0
print(f"frame {k - 1}: visible {tf.stats()['noVisibleEntries']}, {len(idx)} workgroups, span {en[used].max():.2f} us")
for name, sel in (("projection", idx[idx < n_ed]), ("integrate", idx[idx >= n_ed])):
    if len(sel) == 0:
        continue
    d = en[sel] - st[sel]
    print(f"  {name:10s} n={len(sel):5d} dur p10/p50/p90/max {np.percentile(d, 10):6.2f}/{np.median(d):6.2f}/{np.percentile(d, 90):6.2f}/{d.max():6.2f}"
          f"  start p50/max {np.median(st[sel]):6.2f}/{st[sel].max():6.2f}  end p50/max {np.median(en[sel]):6.2f}/{en[sel].max():6.2f}")
sel = idx[idx >= n_ed]
d = en[sel] - st[sel]
b = sel - n_ed
print("integrate duration by workgroup index (quintiles of bid): " +
      " ".join(f"{np.median(d[(b >= q * 154) & (b < (q + 1) * 154)]):.2f}" for q in range(5)))
n = tf.stats()["noVisibleEntries"]
passes = np.array([-(-(n - (bb * 2)) // 3072) for bb in b])
for p_ in sorted(set(passes.tolist())):
    m = passes == p_
    print(f"  {p_} passes: n={m.sum()} dur p50/max {np.median(d[m]):.2f}/{d[m].max():.2f}")
edges = np.arange(0, en[used].max() + 1, 1.0)
print("resident every 1 us:", [int(((st[used] <= e) & (en[used] > e)).sum()) for e in edges])
# by XCD (blockIdx.x mod 8 under round-robin dispatch; TFUSION_INTEG_BANDS: band x on XCD x)
xs = sel % 8
print("integrate end by XCD (p50/max us), workgroups: " +
      " ".join(f"x{x}:{np.median(en[sel][xs == x]):.1f}/{en[sel][xs == x].max():.1f}" for x in range(8)))
# (the XCD-band experiment's builds, tools/experiments/integ_xcd_bands.patch: its band counts and edges)
if hasattr(_lib.load(), "tf_debug_bands"):
    cnt = (ctypes.c_int * 9)()
    edg = (ctypes.c_float * 18)()
    _lib.load().tf_debug_bands(tf._h, cnt, edg)
    print("band_on", cnt[0], "counts", list(cnt[1:]), "edges", [round(x, 1) for x in edg[0:9]], [round(x, 1) for x in edg[9:18]])
