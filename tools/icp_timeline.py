"""Timeline of the persistent ICP kernel's last launch (debug build, `make -C topfusion_amd/csrc
timing`).  On the GPU box:
  TFUSION_HIP_LIB=tools/_build/libtfusion_hip_timing.so python tools/icp_timeline.py"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
from topfusion_amd import TopFu, default_params, synth
from topfusion_amd import _lib
W, H = 640, 480
fx, fy, cx, cy = synth.intrinsics(W, H)
frames = synth.orbit_sequence(8, W, H, seed=7)
dev = synth.DeviceStream(len(frames), frames.shape[2], frames.shape[1])
dev.upload(frames)
tf = TopFu(default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy), device=0)
tf.process_frames(dev.ptr, 3)
bench.device_sync()
NW = 256
S = 2 * NW + 10
buf = (ctypes.c_ulonglong * (64 * S))()
_lib.load().tf_debug_icp_timeline(buf)
tl = np.frombuffer(buf, dtype=np.uint64).reshape(64, S).astype(np.int64)
its = tf.stats()["icp_iterations"]
print("iterations", its, "(times in us, 100 MHz clock, relative to WG0's iteration start)")
for i in range(its):
    t0 = tl[i, 0]
    st = (tl[i, :NW] - t0) / 100.0
    pub = (tl[i, NW:2 * NW] - t0) / 100.0
    g = (tl[i, 2 * NW] - t0) / 100.0
    tail = (tl[i, 2 * NW + 1] - t0) / 100.0
    ph = [(tl[i, 2 * NW + k] - t0) / 100.0 for k in (6, 2, 3, 7, 4, 5)]
    nxt = (tl[i + 1, :NW] - t0) / 100.0 if i + 1 < its else None
    line = (f"it {i:2d}: start[min/med/max] {st.min():5.2f}/{np.median(st):5.2f}/{st.max():5.2f} "
            f"pub {pub.min():5.2f}/{np.median(pub):5.2f}/{pub.max():5.2f} (max wg {int(pub.argmax())}) "
            f"wg0 pub {pub[0]:5.2f} gathered {g:5.2f} [tree+readlane {ph[0]:5.2f} unpack {ph[1]:5.2f} solve {ph[2]:5.2f} "
            f"rodrigues {ph[3]:5.2f} compose {ph[4]:5.2f} det {ph[5]:5.2f}] tail {tail:5.2f}")
    if nxt is not None:
        line += f" next-start {nxt.min():5.2f}/{np.median(nxt):5.2f}/{nxt.max():5.2f}"
        if tl[i + 1, 2 * NW + 8] > 0:               # the next iteration starts a level: its set-up
            line += (f" [level set-up {(tl[i + 1, 2 * NW + 8] - t0) / 100.0:5.2f}"
                     f" maps in {(tl[i + 1, 2 * NW + 9] - t0) / 100.0:5.2f}]")
    print(line)
# the tail's halves on the shader clock, each run twice back to back (the second run's code is
# in the instruction cache): workgroup 0, per iteration
try:
    tb = (ctypes.c_longlong * 256)()
    _lib.load().tf_debug_icp_tail_cycles(tb)
    tc = np.frombuffer(tb, dtype=np.int64).reshape(64, 4)[:its]
    print("tail cycles (shader clock) per iteration: solve, solve again, rodrigues, rodrigues again")
    for i in range(its):
        print(f"  it {i:2d}: {tc[i, 0]:6d} {tc[i, 1]:6d} {tc[i, 2]:6d} {tc[i, 3]:6d}")
    print(f"  median: {int(np.median(tc[:, 0]))} {int(np.median(tc[:, 1]))} {int(np.median(tc[:, 2]))} {int(np.median(tc[:, 3]))}")
except Exception as ex:
    print("tail cycles:", ex)
# the shader clock workgroup 0 ran at (s_memtime against the 100 MHz s_memrealtime)
try:
    cb = (ctypes.c_ulonglong * 128)()
    _lib.load().tf_debug_icp_clock(cb)
    ck = np.frombuffer(cb, dtype=np.uint64).reshape(64, 2).astype(np.int64)
    n = its
    if n > 1:
        dm = ck[n - 1, 0] - ck[0, 0]
        dr = ck[n - 1, 1] - ck[0, 1]
        print(f"shader clock over iterations 0..{n - 1}: {dm / dr * 100.0:.0f} MHz ({dm} s_memtime ticks in {dr / 100.0:.2f} us)")
except Exception as ex:
    print("clock:", ex)
