import os, sys
sys.path.insert(0, "."); sys.path.insert(0, "real-time-path-tracing-voxel-blocks_amd"); sys.path.insert(0, "tests")
import numpy as np, vxpt, bench
a = type("A", (), dict(world=256, scene="c3", width=1920, height=1080))()
chunks, hs, fd, _, pos = bench.scene_args(a)
r = vxpt.Renderer(1920, 1080)
r.load_settings(); r.generate_terrain(chunks, height_scale=hs, freq_den=fd, global_y=True)
r.set_camera(pos, bench.C1_DIR, 90.0, prev=(pos, bench.C1_DIR, 90.0)); r.set_sky()
p = vxpt.DenoiseParams.defaults()
for f in range(12):
    r.render_frame(f, 4, p)
h = r.read("HIST_LEN"); d = r.read("DEPTH")
m = d < 1e20
print("non-sky px", m.sum(), "hist<=4:", ((h <= 4) & m).sum(), "hist dist:", np.percentile(h[m], [1, 5, 50, 95]))
