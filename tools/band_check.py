"""XCD bands (k_vis_build, TFUSION_INTEG_BANDS): the visible blocks' centre columns after the C2 orbit
and one tracked frame, recomputed on the host from the hash, the visible list and the pose, against
the device's band counts and edges (tf_debug_bands; diagnostic builds of the experiment in
tools/experiments/integ_xcd_bands.patch only).  On the GPU box:
  python tools/band_check.py"""
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
p = default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy)
tf = TopFu(p, device=0)
tf.process_frames(dev.ptr, N0)
k = N0
while True:
    ok = tf.process_frames(dev.frame_ptr(k), 1)
    k += 1
    if ok[0] or k >= N0 + 40:
        break
bench.device_sync()
ids = tf.visible_ids()
h = tf.hash()[ids]
c2w = tf.getCameraPose().astype(np.float64)
w2c = np.linalg.inv(c2w)
f = 8 * p.voxelSize
P = np.stack([(h["x"] + 0.5) * f, (h["y"] + 0.5) * f, (h["z"] + 0.5) * f, np.ones(len(h))], 0)
C = w2c @ P
u = np.where(C[2] > 0, fx * C[0] / np.where(C[2] > 0, C[2], 1) + cx, cx)
cnt = (ctypes.c_int * 9)()
edg = (ctypes.c_float * 18)()
_lib.load().tf_debug_bands(tf._h, cnt, edg)
print(f"frame {k - 1}: visible {len(ids)}; device band_on {cnt[0]} counts {list(cnt[1:])}")
print("edges buffers", [round(x, 1) for x in edg[0:9]], [round(x, 1) for x in edg[9:18]])
for e in (np.array(edg[0:9]), np.array(edg[9:18])):
    b = np.searchsorted(e[1:8], u, side="right")
    print("host counts with", np.round(e, 1).tolist(), np.bincount(b, minlength=8).tolist())
print("u percentiles 0/1/10/50/90/99/100:", np.round(np.percentile(u, [0, 1, 10, 50, 90, 99, 100]), 1).tolist())
print("z percentiles:", np.round(np.percentile(C[2], [0, 1, 50, 99, 100]), 3).tolist())
print("u histogram (80 px):", np.histogram(np.clip(u, -80, 719), bins=np.arange(-80, 721, 80))[0].tolist())
# vis_build timeline (TF_VIS_TIMELINE builds)
try:
    buf = (ctypes.c_ulonglong * (1024 * 8))()
    if _lib.load().tf_debug_vis_timeline(buf, ctypes.sizeof(buf)) == 0:
        tl8 = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8).astype(np.int64)
        spins = tl8[:, 7].copy()
        tl = tl8[:, [0, 1, 2, 5, 3, 4]]
        used = tl[:, 0] > 0
        t0 = tl[used, 0].min()
        t = (tl[used] - t0) / 100.0
        names = ["start", "count pub", "bands pub", "counts read", "bands read", "end"]
        print("k_vis_build workgroups", int(used.sum()))
        for j, nm in enumerate(names):
            print(f"  {nm:11s} p10/p50/p90/max {np.percentile(t[:, j], 10):6.2f}/{np.median(t[:, j]):6.2f}/{np.percentile(t[:, j], 90):6.2f}/{t[:, j].max():6.2f}")
        print("  last workgroup:", np.round(t[-1], 2).tolist())
        print("  band re-polls per workgroup p50/max:", int(np.median(spins[used])), int(spins[used].max()))
except AttributeError:
    pass
