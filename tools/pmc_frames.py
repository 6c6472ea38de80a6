"""PMC driver (run under rocprofv3 --pmc): the bench's C2 frames through the bench's own path --
frames 0..WARM-1 as warm-up batches, then the timed region's frames in 32-frame tf_process_frames
steps -- and a JSON of what each frame was (frame-0 path / tracked / ICP-failure reset) and the
timed region's visible-block and voxel-lane totals, so tools/pmc_frames_summary.py can attribute
every dispatch's counters to one frame and one frame type, on the timed frames only.

    rocprofv3 --pmc FETCH_SIZE ... -- python3 tools/pmc_frames.py OUT.json [steps=20] [warmup=5]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    import bench
    from topfusion_amd import TopFu, default_params, synth
    W, H, F = 640, 480, 32
    n = (warm + steps) * F
    dev = bench.orbit_frames(n, W, H, 7)
    bench.device_sync()
    fx, fy, cx, cy = synth.intrinsics(W, H)
    tf = TopFu(default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy))
    tf.profile(True)             # (also counts the integration's voxel lanes; events do not change any kernel's traffic)
    fb = W * H * 2
    ok = []
    for s in range(warm + steps):
        if s == warm:
            bench.device_sync()
            tf.reset_totals()
        ok.extend(int(v) for v in tf.process_frames(dev.ptr + s * F * fb, F))
    tot = tf.totals()
    # frame types: frame 0 of a run (the first, and every frame after a reset) takes the
    # integrate-only path; a tracked frame's ICP succeeded; a reset frame's ICP failed
    kind = []
    for k, v in enumerate(ok):
        if k == 0 or ok[k - 1] == 0:
            kind.append("frame0")
        else:
            kind.append("tracked" if v else "reset")
    integrated = max(1, tot["frames"] - tot["resets"])
    json.dump({"frames": n, "timed_first": warm * F, "kind": kind,
               "timed_totals": tot, "nvis_mean_integrated": tot["visible_sum"] / integrated,
               "lanes_per_integrated_frame": [tot["integrate_lanes_read"] / integrated,
                                              tot["integrate_lanes_written"] / integrated]}, open(out, "w"))
    tf.close()


if __name__ == "__main__":
    main()
