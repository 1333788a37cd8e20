"""C5: 64 frames x 1 spp on the C1 scene, GPU vs oracle, relative RMS of the
denoised output and of the last frame's radiance over non-sky pixels.
python tools/c5_check.py [W H FRAMES]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402
import vxpt  # noqa: E402
from test_gpu_parity import _setup, _inject_sky, _dn_params  # noqa: E402

w, h, frames = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 256, 64)
r, o = _setup(w, h)
_inject_sky(r, o)
p = _dn_params()
t0 = time.time()
for f in range(frames):
    r.trace(f)
    r.denoise(f, f + 1, p)
    o.trace(f)
    o.post_trace()
    o.denoise(f, f + 1)
print("rendered %d frames in %.1f s" % (frames, time.time() - t0))
mask = r.read("DEPTH") < 1e20
for name, which in (("OUTPUT", 21), ("ILLUM", 0)):
    g, c = r.read(name)[..., :3][mask], o.read(which)[..., :3][mask]
    rms = np.sqrt(((g - c) ** 2).mean()) / np.sqrt((c ** 2).mean())
    print("%-7s relative RMS %.3e   max abs %.3e   mean g %.5f c %.5f" % (name, rms, np.abs(g - c).max(), g.mean(), c.mean()))
