"""k_ed_fill in isolation: a C2 scene after 12 orbit frames, then back-to-back fill launches over
the last frame's visible list (tf_time_stage(TF_STAGE_EXPECTED_DEPTHS)).  GPU box only.
ED_MICRO_FRAMES sets the number of frames (12: ~11k visible entries, 5: ~6k)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from topfusion_amd import TopFu, default_params, synth
W, H = 640, 480
fx, fy, cx, cy = synth.intrinsics(W, H)
g = TopFu(default_params(cols=W, rows=H, fx=fx, fy=fy, cx=cx, cy=cy))
nf = int(os.environ.get("ED_MICRO_FRAMES", "12"))
seq = synth.orbit_sequence(nf, W, H, seed=7)
for k in range(nf):
    ok = g(seq[k])
pose = g.getCameraPose()[:3, :4]
n = g.last_stats["noVisibleEntries"]
ms = [g.time_stage("expected_depths", pose, 500) for _ in range(3)]
print(json.dumps({"lds_max_n": os.environ.get("TFUSION_ED_LDS_MAX_N"), "n": n, "ok": bool(ok),
                  "us_per_launch": [round(m * 1000, 2) for m in ms]}))
