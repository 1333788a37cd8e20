"""Steady-state history-fix workload of the C3 bench scene: after K frames, the pixels the history
fix filters (history length <= 4, in the denoising range) per 16x16 tile -- how many tiles list
pixels, and how the lists are distributed (sparse <= 64 / dense).  Usage: python tools/hf_stats.py"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd"))
import vxpt  # noqa: E402
from bench import C1_DIR, scene_args  # noqa: E402


class A:
    world = 256
    scene = "c3"


chunks, hs, fd, _, pos = scene_args(A)
w, h = 1920, 1080
r = vxpt.Renderer(w, h)
r.load_settings()
r.generate_terrain(chunks, height_scale=hs, freq_den=fd, global_y=True)
r.set_camera(pos, C1_DIR, 90.0, prev=(pos, C1_DIR, 90.0))
r.set_sky()
p = vxpt.DenoiseParams.defaults()
for frames in (8, 18):
    r.render_frames(0 if frames == 8 else 8, 8 if frames == 8 else 10, 4, p)
    hist, depth = r.read("HIST_LEN"), r.read("DEPTH")
    low = (hist <= 4) & (depth < 5e5)
    ty, tx = (h + 15) // 16, (w + 15) // 16
    pad = np.zeros((ty * 16, tx * 16), bool)
    pad[:h, :w] = low
    cnt = pad.reshape(ty, 16, tx, 16).sum(axis=(1, 3)).ravel()
    nz = cnt[cnt > 0]
    print("after %d frames: listed pixels %d (%.2f %%), tiles with a list %d of %d, dense (>64) %d, "
          "max %d, p50/p90/p99 of non-empty %s" % (frames, low.sum(), 100.0 * low.mean(), nz.size, cnt.size,
                                                   (cnt > 64).sum(), cnt.max(),
                                                   np.percentile(nz, [50, 90, 99]).round(1) if nz.size else "-"))
r.close()
