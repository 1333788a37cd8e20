"""Render frames of one band of the C3 frame alone (a single context in band mode, no exchange): the
workload one rank of an N-band partition runs, for kernel traces of the band schedule's fixed costs.
python tools/band_kt.py Y0 Y1 [--frames K] [--width W --height H] [--tune field=value ...] [--rccl]
(--rccl: through a one-rank RCCL communicator on the band, band_frame's schedule)"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd"))
import vxpt  # noqa: E402
from bench import C1_DIR, C1_POS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("y0", type=int)
ap.add_argument("y1", type=int)
ap.add_argument("--frames", type=int, default=6)
ap.add_argument("--warmup", type=int, default=6)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=4)
ap.add_argument("--tune", action="append", default=[])
ap.add_argument("--rccl", action="store_true")
a = ap.parse_args()
pos = tuple(p * 4 for p in C1_POS)
r = vxpt.Renderer(a.width, a.height) if a.rccl else vxpt.Renderer(a.width, a.height, rows=(a.y0, a.y1))
r.load_settings()
if a.tune:
    r.set_tuning(**{k: int(v) for k, v in (t.split("=", 1) for t in a.tune)})
r.generate_terrain((8, 8, 8), height_scale=128.0, freq_den=256.0, global_y=True)
r.set_camera(pos, C1_DIR, 90.0, prev=(pos, C1_DIR, 90.0))
r.set_sky()
if a.rccl:
    r.band_comm_init(vxpt.band_comm_id(), 1, 0)
    r.set_band(a.y0, a.y1)
p = vxpt.DenoiseParams.defaults()
r.render_frames(0, a.warmup, a.spp, p)
r.sync()
t0 = time.perf_counter()
r.render_frames(a.warmup, a.frames, a.spp, p)
r.sync()
t = r.timings()
print("rows %d-%d: %.4f ms per frame (trace %.4f, denoise %.4f)" % (a.y0, a.y1, (time.perf_counter() - t0) / a.frames * 1e3,
                                                                  t["trace_ms"], t["denoise_ms"]))
r.close()
