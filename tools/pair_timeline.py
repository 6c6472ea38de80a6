"""Workgroup timeline of one k_raycast_pair launch (diagnostic build: bash tools/build_variant.sh
ptl -DTF_PAIR_TIMELINE).  On the GPU box:
  TFUSION_HIP_LIB=tools/_build/ptl/libtfusion_hip.so python tools/pair_timeline.py
Runs the C2 orbit through the batch path, then one tracked frame at a time, and prints for the
last frame's pair launch: the span, per branch kind the workgroups' durations and start times,
resident workgroups over time, and the longest workgroups with their waves' end times."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
from topfusion_amd import TopFu, default_params, synth
from topfusion_amd import _lib
W, H = 640, 480
N0 = int(sys.argv[1]) if len(sys.argv) > 1 else 160
fx, fy, cx, cy = synth.intrinsics(W, H)
dev = bench.orbit_frames(N0 + 40, W, H, 7)
tf = TopFu(default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy), device=0)
tf.process_frames(dev.ptr, N0)
k = N0
if os.environ.get("PTL_BATCH"):      # (the ptl_la build: the last launch of a 32-frame batch with lookahead)
    tf.process_frames(dev.frame_ptr(k), 32)
    k += 32
else:
    while True:
        ok = tf.process_frames(dev.frame_ptr(k), 1)
        k += 1
        if ok[0] and tf.stats()["frame_counter"] > 1 or k >= N0 + 40:
            break
bench.device_sync()
PTL = 8192
buf = (ctypes.c_ulonglong * (PTL * 7))()
_lib.load().tf_debug_pair_timeline(buf, ctypes.sizeof(buf))
tl = np.frombuffer(buf, dtype=np.uint64).reshape(PTL, 7).astype(np.int64)
used = tl[:, 0] > 0
tl = tl[used]
kind = tl[:, 6] & 0xff
xcc = (tl[:, 6] >> 8) & 0xf
t0 = tl[:, 0].min()
st = (tl[:, 0] - t0) / 100.0
en = (tl[:, 5] - t0) / 100.0
wv = (tl[:, 1:5] - t0) / 100.0
dur = en - st
names = {0: "fill", 1: "icp-maps rays", 2: "render rays", 3: "pyr/normals", 4: "bilateral", 5: "idle"}
print(f"frame {k - 1} visible {tf.stats().get('visible_entries', '?')}: {len(tl)} workgroups, span {en.max():.2f} us")
for kd in sorted(set(kind.tolist())):
    m = kind == kd
    d = dur[m]
    print(f"  {names.get(kd, kd):14s} n={m.sum():5d} dur p50/p90/max {np.median(d):6.2f}/{np.percentile(d, 90):6.2f}/{d.max():6.2f}"
          f"  start p50/p90/max {np.median(st[m]):6.2f}/{np.percentile(st[m], 90):6.2f}/{st[m].max():6.2f}"
          f"  end max {en[m].max():6.2f}")
    if kd in (1, 2):
        w = (wv[m] - st[m][:, None]).ravel()
        print(f"      wave lifetimes p50/p90/p99/max {np.median(w):6.2f}/{np.percentile(w, 90):6.2f}/{np.percentile(w, 99):6.2f}/{w.max():6.2f}")
        spread = (wv[m].max(1) - wv[m].min(1))
        print(f"      slowest - fastest wave of a tile p50/p90 {np.median(spread):6.2f}/{np.percentile(spread, 90):6.2f}")
edges = np.arange(0, en.max() + 2, 2.0)
act = [int(((st <= e) & (en > e)).sum()) for e in edges]
print("resident workgroups every 2 us:", act)
print("ray workgroups ending after t:", [int(((kind == 1) | (kind == 2))[en > t].sum()) for t in (10, 20, 30, 40, 50, 60)])
order = np.argsort(-en)[:12]
for i in order:
    print(f"  wg kind {names.get(int(kind[i]), kind[i]):14s} xcc {int(xcc[i])} start {st[i]:6.2f} end {en[i]:6.2f} waves " +
          " ".join(f"{x:6.2f}" for x in wv[i]))
