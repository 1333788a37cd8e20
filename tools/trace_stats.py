"""Traversal statistics of the C3 workload (experiment tool, GPU box).

Needs the instrumented build: make -C real-time-path-tracing-voxel-blocks_amd libvxpt_stats.so,
then VXPT_LIB=<that .so> python tools/trace_stats.py.  Prints, per ray kind, the
rays traced, mean DDA outer iterations per ray and the mean over waves of the
slowest lane's iterations (SIMD efficiency = mean / mean-of-max).
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import vxpt  # noqa: E402
from bench import C1_DIR, scene_args  # noqa: E402

KINDS = {0: "path rays", 1: "BRDF candidate", 2: "camera", 3: "visibility x4 (ReSTIR)", 4: "visibility (RIS)",
         5: "stragglers (all queues)"}


class A:
    world = int(os.environ.get("WORLD", 256))
    scene = "c3"


def main():
    lib = vxpt.load_library()
    lib.vxpt_debug_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    chunks, hs, fd, _, pos = scene_args(A)
    r = vxpt.Renderer(1920, 1080, device=0)
    r.load_settings()
    r.generate_terrain(chunks, height_scale=hs, freq_den=fd, global_y=True)
    r.set_camera(pos, C1_DIR, 90.0, prev=(pos, C1_DIR, 90.0))
    r.set_sky()
    p = vxpt.DenoiseParams.defaults()
    buf = np.zeros(192, np.uint64)
    for f in range(4):
        r.render_frame(f, 4, p)
    r.sync()
    lib.vxpt_debug_stats(buf.ctypes.data, 1)
    for f in range(4, 8):
        r.render_frame(f, 4, p)
    r.sync()
    lib.vxpt_debug_stats(buf.ctypes.data, 1)
    for k, name in KINDS.items():
        g = [int(v) for v in buf[8 * k:8 * k + 8]]
        rays, waves, mx = g[0], g[1], g[2]
        if waves == 0:
            continue
        lv = g[3:7]
        its = sum(lv)
        print("%-24s rays/pass %9.0f lanes/wave %5.1f iters/ray %6.2f max/wave %6.2f simd-eff %.2f | "
              "per ray: skip64 %.2f skip16 %.2f skip4 %.2f brick %.2f cellsteps %.2f" % (
                  name, rays / 16.0, rays / waves, its / rays, mx / waves, its / (64.0 * mx),
                  lv[0] / rays, lv[1] / rays, lv[2] / rays, lv[3] / rays, g[7] / rays))
    print("per-ray iterations in the launch (bins [0,2) [2,4) [4,8) .. [128,inf)), up = d.y > 0, event = hit/occluded")
    for k, name in KINDS.items():
        g = [int(v) for v in buf[64 + 16 * k:64 + 16 * k + 16]]
        n = sum(g[:8])
        if n == 0:
            continue
        print("%-24s %s up %.3f event %.3f max %d" % (name, " ".join("%.4f" % (v / n) for v in g[:8]), g[8] / n,
                                                       g[9] / n, g[10]))
    print("timings", r.timings())


if __name__ == "__main__":
    main()
