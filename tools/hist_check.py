"""Steady-state history-length histogram of the C3 workload (GPU box diagnostic)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import vxpt  # noqa: E402
from bench import C1_DIR, scene_args  # noqa: E402


class A:
    world = 256
    scene = "c3"


chunks, hs, fd, _, pos = scene_args(A)
r = vxpt.Renderer(1920, 1080, device=0)
r.load_settings()
r.generate_terrain(chunks, height_scale=hs, freq_den=fd, global_y=True)
r.set_camera(pos, C1_DIR, 90.0, prev=(pos, C1_DIR, 90.0))
r.set_sky()
p = vxpt.DenoiseParams.defaults()
for f in range(12):
    r.render_frame(f, 4, p)
    r.sync()
    h = r.read("HIST_LEN").ravel()
    d = r.read("DEPTH").ravel()
    nonsky = d < 5e5
    hh = h[nonsky]
    print("frame %2d  non-sky %d  hist<=4: %.4f  mean %.2f  %s  denoise %.3f ms" % (
        f, nonsky.sum(), (hh <= 4).mean(), hh.mean(), np.percentile(hh, [1, 10, 50]), r.timings()["denoise_ms"]))
