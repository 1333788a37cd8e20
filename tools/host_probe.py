"""Host enqueue time against GPU frame time (vxpt_timings host_ms / frame_ms) of pipelined runs: the
whole C3 frame in one context, the frame through a one-rank communicator, and bands of the 8-band
partition through a one-rank communicator (bench.band_tuning's schedule).  host_ms close to frame_ms:
the GPU waited for the host.  python tools/host_probe.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from band_proxy import C1_DIR, band_tuning, vxpt  # noqa: E402


def run(rows, comm, frames=12, warmup=6, spp=4, tune=None):
    pos = tuple(p * 4 for p in (35.6184, 11.8733, 42.0387))
    r = vxpt.Renderer(1920, 1080)
    try:
        r.load_settings()
        t = dict(band_tuning(1920, 1080, 8) if rows else {})
        t.update(tune or {})
        if t:
            r.set_tuning(**t)
        r.generate_terrain((8, 8, 8), height_scale=128.0, freq_den=256.0, global_y=True)
        r.set_camera(pos, C1_DIR, 90.0, prev=(pos, C1_DIR, 90.0))
        r.set_sky()
        if comm:
            r.band_comm_init(vxpt.band_comm_id(), 1, 0)
            if rows:
                r.set_band(*rows)
        p = vxpt.DenoiseParams.defaults()
        r.render_frames(0, warmup, spp, p)
        r.sync()
        t0 = time.perf_counter()
        r.render_frames(warmup, frames, spp, p)
        wall = (time.perf_counter() - t0) / frames * 1e3
        tm = r.timings()
        return {"rows": rows, "comm": comm, "tune": tune or {}, "wall_ms": round(wall, 4),
                "frame_ms": round(tm["frame_ms"], 4), "host_ms": round(tm["host_ms"], 4)}
    finally:
        r.close()


if __name__ == "__main__":
    for rows, comm in ((None, False), (None, True), ((416, 536), True), ((832, 1080), True)):
        print(json.dumps(run(rows, comm)), flush=True)
