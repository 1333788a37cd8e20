"""The banded vxpt_render_frames path (a one-rank RCCL communicator: band_frame's schedule, its
exchanges with no neighbour) against a plain context's pipelined loop, C3 scene, optionally on a
band of rows: python tools/band_rccl_probe.py [ROW0 ROW1] -- frame / trace / denoiser ms of each
(VXPT_LIB=... selects the build)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from band_proxy import C1_DIR, band_tuning, vxpt  # noqa: E402


def run(comm, rows, frames=12, warmup=6, spp=4):
    pos = tuple(p * 4 for p in (35.6184, 11.8733, 42.0387))
    r = vxpt.Renderer(1920, 1080, rows=rows) if rows and not comm else vxpt.Renderer(1920, 1080)
    try:
        r.load_settings()
        tune = band_tuning(1920, 1080, 8) if rows else {}
        if tune:
            r.set_tuning(**tune)
        r.generate_terrain((8, 8, 8), height_scale=128.0, freq_den=256.0, global_y=True)
        r.set_camera(pos, C1_DIR, 90.0, prev=(pos, C1_DIR, 90.0))
        r.set_sky()
        if comm:
            r.band_comm_init(vxpt.band_comm_id(), 1, 0)
            if rows:
                r.set_band(*rows)  # one rank: no neighbour, the band's rows only
        p = vxpt.DenoiseParams.defaults()
        r.render_frames(0, warmup, spp, p)
        r.sync()
        t0 = time.perf_counter()
        r.render_frames(warmup, frames, spp, p)
        r.sync()
        wall = (time.perf_counter() - t0) / frames * 1e3
        t = r.timings()
        return {"comm": comm, "rows": rows, "wall_ms": round(wall, 4), "frame_ms": round(t["frame_ms"], 4),
                "trace_ms": round(t["trace_ms"], 4), "denoise_ms": round(t["denoise_ms"], 4)}
    finally:
        r.close()


def main():
    rows = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else None
    for comm in (False, True, False, True):
        print(json.dumps(dict(run(comm, rows), lib=os.path.basename(os.environ.get("VXPT_LIB", "libvxpt.so")))),
              flush=True)


if __name__ == "__main__":
    main()
