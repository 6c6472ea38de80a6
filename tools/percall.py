"""Per-call (TopFu::operator()) cost breakdown on the GPU box: the same 64 orbit frames (device
resident) through (a) TopFu.__call__ (Python wrapper + stats dict), (b) tf_process_frame via
ctypes with preallocated arguments, (c) tf_process_frames as one batch -- each from a fresh context."""
import ctypes, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from topfusion_amd import TopFu, default_params, synth, _lib as L
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
W, H, n = 640, 480, int(os.environ.get("PERCALL_FRAMES", "64"))
skip = int(os.environ.get("PERCALL_SKIP", "0"))
fx, fy, cx, cy = synth.intrinsics(W, H)
pk = dict(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy)
dev = bench.orbit_frames(skip + n, W, H, 7)
fb = W * H * 2
base = dev.ptr + skip * fb
out = {}
# (a)
tf = TopFu(default_params(**pk))
bench.device_sync(); t0 = time.perf_counter()
for k in range(n):
    tf(base + k * fb)
out["python_call_fps"] = n / (time.perf_counter() - t0)
tf.close()
# (b)
tf = TopFu(default_params(**pk))
lib = L.load()
pose = (ctypes.c_float * 12)()
h = tf._h
bench.device_sync(); t0 = time.perf_counter()
for k in range(n):
    lib.tf_process_frame(h, ctypes.c_void_p(base + k * fb), W * 2, pose, None)
out["ctypes_call_fps"] = n / (time.perf_counter() - t0)
tf.close()
# (c)
tf = TopFu(default_params(**pk))
bench.device_sync(); t0 = time.perf_counter()
ok = tf.process_frames(base, n)
bench.device_sync()
out["batched_fps"] = n / (time.perf_counter() - t0)
out["resets"] = int((~ok.astype(bool)).sum())
tf.close()
out["frames"] = n; out["skip"] = skip
print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in out.items()}))
