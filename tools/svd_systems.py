"""Capture the 6x6 systems (27 sums: StreamHelper layout, projective_icp.cpp:51-61) of every ICP
iteration the oracle runs on the bench's C2 frames under the OpenCV 3.x-4.x pose algebra, and
the Jacobi-SVD sweep statistics of those solves (oracle/tf_oracle.c, tfo_cv_jacobi_svd).

    python tools/svd_systems.py --frames 300 --out tools/_build/svd_systems_C2.npy

Test infrastructure: CPU only; the systems feed tools/micro/svd_lanes.hip (the lane-parallel
Jacobi against the serial one, bit for bit, and its latency)."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O            # noqa: E402
from topfusion_amd import synth           # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--algebra", default="opencv4")
    ap.add_argument("--out", default=os.path.join(ROOT, "tools", "_build", "svd_systems_C2.npy"))
    args = ap.parse_args()
    W, H = 640, 480
    fx, fy, cx, cy = synth.intrinsics(W, H)
    O.set_pose_algebra(args.algebra)
    o = O.Oracle(O.default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy, voxelSize=0.005), omp=True)
    L = o.L
    cap = args.frames * 19
    buf = np.zeros((cap, 27), np.float32)
    L.tfo_capture_sums(buf.ctypes.data, cap)
    st = (ctypes.c_longlong * 36)()
    L.tfo_cv_svd_stats(st, 1)
    ok = 0
    for k in range(args.frames):
        R, t = synth.orbit_pose(k)
        ok += o(synth.render_room(R, t, W, H, seed=7, frame=k))
    n = L.tfo_captured_sums()
    L.tfo_capture_sums(None, 0)
    L.tfo_cv_svd_stats(st, 1)
    s = list(st)
    np.save(args.out, buf[:n])
    print(json.dumps({"frames": args.frames, "ok": ok, "systems": n, "jacobi_calls": s[0], "sweeps": s[1],
                      "rotations": s[2], "max_sweep_index": s[3],
                      "sweeps_hist": {i: s[4 + i] for i in range(32) if s[4 + i]}}))


if __name__ == "__main__":
    main()
