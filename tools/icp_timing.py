"""Per-phase ICP iteration timing (debug build, `make -C topfusion_amd/csrc timing`).
Run on the GPU box: TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so python tools/icp_timing.py"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
from topfusion_amd import TopFu, default_params, synth
from topfusion_amd import _lib
W, H = 640, 480
fx, fy, cx, cy = synth.intrinsics(W, H)
frames = synth.orbit_sequence(60, W, H, seed=7)
dev = synth.DeviceStream(len(frames), frames.shape[2], frames.shape[1])
dev.upload(frames)
tf = TopFu(default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy), device=0)
tf.process_frames(dev.ptr, 60)
bench.device_sync()
L = _lib.load()
ts = (ctypes.c_ulonglong * 16)()
L.tf_debug_icp_ts(ts)
n = max(ts[0], 1)
names = {1: "ticket won", 2: "final tree loads+LDS", 3: "tree+unpack", 4: "det", 5: "solve", 6: "rodrigues+compose+store"}
print("launches", n)
for k in range(1, 7):
    print(f"{names[k]:28s} cumulative {ts[k] / n * 10 / 1000:8.3f} us (from last-WG entry)")

m = ts[7]
if m:
    print("persistent iterations", m)
    for k, name in ((8, "WG0 own column published"), (9, "WG0 all 256 columns gathered"), (10, "WG0 tail done"),
                    (12, "WG255 own column published"), (13, "WG255 broadcast seen")):
        print(f"{name:30s} {ts[k] / m * 10 / 1000:8.3f} us after iteration start")
