"""Where a GPU build first leaves the oracle on the 320x240 orbit (diagnostic): after every frame,
pose, counters, hash, visible list, voxels and range image, the first difference reported.
On the GPU box:  [TFUSION_HIP_LIB=...] python tools/seq_diverge.py [frames]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from topfusion_amd import TopFu, default_params, synth
from oracle import oracle as om
from parity_util import same_bits

cols, rows = 320, 240
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
fx, fy, cx, cy = synth.intrinsics(cols, rows)
args = dict(cols=cols, rows=rows, fx=fx, fy=fy, cx=cx, cy=cy)
g, o = TopFu(default_params(**args)), om.Oracle(om.default_params(**args))
seq = synth.orbit_sequence(n, cols, rows, seed=7)
for k in range(n):
    okg, oko = g(seq[k]), o(seq[k])
    rep = []
    if okg != oko: rep.append(f"ok {okg}/{oko}")
    if not same_bits(g.getCameraPose()[:3, :4], o.pose()).all(): rep.append("pose")
    hg, ho = g.hash(), o.hash()
    for f in ("x", "y", "z", "offset", "ptr"):
        if not np.array_equal(hg[f], ho[f]): rep.append(f"hash.{f} ({int((hg[f] != ho[f]).sum())})")
    vg, vo = g.visible_ids(), o.visible_ids()
    if len(vg) != len(vo) or not np.array_equal(vg, vo): rep.append(f"visible ids ({len(vg)}/{len(vo)})")
    bg, bo = g.vba(), o.vba()
    for f in ("sdf", "w"):
        d = bg[f] != bo[f]
        if d.any():
            idx = np.nonzero(d)[0]
            rep.append(f"vba.{f} ({len(idx)}; blocks {sorted(set((idx // 512).tolist()))[:8]})")
    if k > 0 and oko:
        r = ~same_bits(g.range_image(), o.range_image())
        if r.any(): rep.append(f"range ({int(r.sum())})")
    print(f"frame {k}: ok {okg} visible {len(vg)}: " + (", ".join(rep) if rep else "identical"))
