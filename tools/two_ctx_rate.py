"""Batched C2 rate of a context while a second context lives on the same device (the persistent
ICP launches are then ordered across the two by a stream event, tf_capi.hip icp_order_*), against
the same frames on a context alone.  On the GPU box:
  TFUSION_HIP_LIB=... python tools/two_ctx_rate.py
Prints one JSON line: alone / with a second context, frames/s, median of 3."""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
from topfusion_amd import TopFu, default_params, synth
W, H, F, N0, N = 640, 480, 32, 160, 256
fx, fy, cx, cy = synth.intrinsics(W, H)
dev = bench.orbit_frames(N0 + N, W, H, 7)
pk = dict(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy)


def rate(second):
    tf = TopFu(default_params(**pk), device=0)
    other = TopFu(default_params(**pk), device=0) if second else None
    tf.process_frames(dev.ptr, N0)                # warm state: frames 0..N0-1 untimed
    r = bench.batched_rate(tf, dev.frame_ptr(N0), N, F)
    tf.close()
    if other:
        other.close()
    return r


out = {}
for second in (False, True, False, True, False, True):
    out.setdefault("with_second_context" if second else "alone", []).append(rate(second))
print(json.dumps({k: round(float(np.median(v)), 1) for k, v in out.items()} | {"runs": out}))
