"""Ray-march step statistics of the C2 bench frames (diagnostic; needs the TF_RAY_STATS build:
bash tools/build_variant.sh raystats -DTF_RAY_STATS, run with TFUSION_HIP_LIB pointing at it).

Per tracked frame: steps per ray in unallocated space (a grid lookup only) and steps that read
voxels, for CreateICPMaps' castRay<true> and renderImage's castRay; per 64-lane wave (4 rows of a
16x16 tile) the longest ray, which sets the wave's time."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from topfusion_amd import TopFu, default_params, synth
    from topfusion_amd import _lib as L
    W, H, F = 640, 480, 32
    first, nsamp = 160, int(sys.argv[1]) if len(sys.argv) > 1 else 24
    dev = bench.orbit_frames(first + nsamp, W, H, 7)
    bench.device_sync()
    fx, fy, cx, cy = synth.intrinsics(W, H)
    tf = TopFu(default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy))
    fb = W * H * 2
    tf.process_frames(dev.ptr, first)
    lib = L.load()
    lib.tf_debug_ray_stats.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(2 * 1280 * 960, np.uint32)
    rows = []
    for k in range(first, first + nsamp):
        ok = tf.process_frames(dev.ptr + k * fb, 1)
        if not ok[0]:
            continue
        assert lib.tf_debug_ray_stats(buf.ctypes.data, buf.nbytes) == 0
        res = {"frame": k}
        for half, name in ((0, "icp"), (1, "render")):
            a = buf[half * 1280 * 960: half * 1280 * 960 + W * H].reshape(H, W)
            free = (a & 0xffff).astype(np.int64)
            found = (a >> 16).astype(np.int64)
            tot = free + found
            # waves: 16x16 tiles, 4 rows each
            t = tot.reshape(H // 16, 16, W // 16, 16).transpose(0, 2, 1, 3).reshape(-1, 4, 64)
            wmax = t.max(axis=2).ravel()
            res[name] = {"ray_free": float(free.mean()), "ray_found": float(found.mean()), "ray_total": float(tot.mean()),
                         "wave_max_mean": float(wmax.mean()), "wave_max_p50": float(np.percentile(wmax, 50)),
                         "wave_max_p90": float(np.percentile(wmax, 90)), "wave_max_max": int(wmax.max()),
                         "ray_total_max": int(tot.max()), "wave_free_max_mean":
                         float((free.reshape(H // 16, 16, W // 16, 16).transpose(0, 2, 1, 3).reshape(-1, 4, 64)).max(axis=2).mean())}
        rows.append(res)
        print(json.dumps(res), flush=True)
    for name in ("icp", "render"):
        keys = rows[0][name].keys()
        print(name, {k: round(float(np.mean([r[name][k] for r in rows])), 2) for k in keys})
    tf.close()


if __name__ == "__main__":
    main()
