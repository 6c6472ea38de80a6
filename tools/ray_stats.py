"""Ray-march step statistics of the C2 bench frames (diagnostic; needs the TF_RAY_STATS build:
bash tools/build_variant.sh raystats -DTF_RAY_STATS, run with TFUSION_HIP_LIB pointing at it).

Per tracked frame: steps per ray in unallocated space (a grid lookup only), steps that read
voxels and, of those, band steps (the eight interpolation corners read too), for CreateICPMaps'
castRay<true> and renderImage's castRay; per 64-lane wave (an 8x8 quadrant of a 16x16 tile) the
longest ray, which sets the wave's time, and the composition of the longest waves' longest rays
with a round-trip count (1 per free step, 2 per voxel step, 2 more per band step)."""
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
    buf = np.zeros(4 * 1280 * 960, np.uint32)
    rows = []
    for k in range(first, first + nsamp):
        ok = tf.process_frames(dev.ptr + k * fb, 1)
        if not ok[0]:
            continue
        assert lib.tf_debug_ray_stats(buf.ctypes.data, buf.nbytes) == 0
        res = {"frame": k}
        for half, name in ((0, "icp"), (1, "render")):
            a = buf[half * 1280 * 960: half * 1280 * 960 + W * H].reshape(H, W)
            free = (a & 0x3ff).astype(np.int64)
            found = ((a >> 10) & 0x7ff).astype(np.int64)
            band = (a >> 21).astype(np.int64)
            one = buf[(2 + half) * 1280 * 960: (2 + half) * 1280 * 960 + W * H].reshape(H, W).astype(np.int64)
            tot = free + found
            rt = free + 2 * found + 2 * band

            def waves(v):   # 8x8 quadrants: (H/8, 8, W/8, 8) -> (waves, 64)
                return v.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
            wt, wf, wb, wr, wo = waves(tot), waves(free), waves(band), waves(rt), waves(one)
            wmax = wt.max(axis=1)
            arg = wt.argmax(axis=1)
            top = np.argsort(-wmax)[:max(1, len(wmax) // 100)]          # the longest 1 % of waves
            lr = lambda v: v[top, arg[top]]
            res[name] = {"ray_free": float(free.mean()), "ray_found": float(found.mean()), "ray_band": float(band.mean()),
                         "ray_total": float(tot.mean()),
                         "wave_max_mean": float(wmax.mean()), "wave_max_p50": float(np.percentile(wmax, 50)),
                         "wave_max_p90": float(np.percentile(wmax, 90)), "wave_max_max": int(wmax.max()),
                         "wave_rt_max_mean": float(wr.max(axis=1).mean()), "wave_rt_max_max": int(wr.max()),
                         "top1pct_ray_steps": float(lr(wt).mean()), "top1pct_ray_free": float(lr(wf).mean()),
                         "top1pct_ray_band": float(lr(wb).mean()), "top1pct_ray_rt": float(lr(wr).mean()),
                         "ray_found_sdf1": float(one.mean()), "top1pct_ray_found_sdf1": float(lr(wo).mean()),
                         "top1pct_live_lanes_at_half": float(np.mean([(wt[w] > wmax[w] // 2).sum() for w in top]))}
        if k == first + nsamp - 1 or len(rows) == 0:
            try:
                vis = tf.visible_ids()
                ptr = tf.hash()["ptr"][vis]
                ptr = ptr[ptr >= 0]
                sdf = tf.vba()["sdf"].reshape(-1, 512)[ptr]
                res["visible_blocks"] = int(len(ptr))
                res["uniform_sdf1_blocks"] = int((sdf == 0x7fff).all(axis=1).sum())
            except Exception as ex:
                res["uniform_note"] = repr(ex)[:160]
        rows.append(res)
        print(json.dumps(res), flush=True)
    for name in ("icp", "render"):
        keys = rows[0][name].keys()
        print(name, {k: round(float(np.mean([r[name][k] for r in rows])), 2) for k in keys})
    tf.close()


if __name__ == "__main__":
    main()
