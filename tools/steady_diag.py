"""Diagnostic of the C3 steady-state parity test (tests/test_gpu_frames_spp.py): per frame, at the
given pixels, the GPU-vs-oracle difference of the radiance, the clamp's history (PREV_ILLUM /
PREV_FAST), the history length and the output, and the clamp decisions in a window around them.
python tools/steady_diag.py [frames] [y,x ...]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("", "real-time-path-tracing-voxel-blocks_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(REPO, d))
import vxpt  # noqa: E402
from test_gpu_frames_spp import _c3_pair, _clamp_decision_flips  # noqa: E402
from test_gpu_parity import _dn_params, pixel_l2  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 12
pts = [tuple(int(v) for v in a.split(",")) for a in sys.argv[2:]] or [(149, 963), (114, 443)]
r, o = _c3_pair(1920, 1080)
r.debug_clamp_decisions(True)
p = _dn_params()
for f in range(frames):
    r.render_frame(f, 4, p)
    o.render_frame(f, 4)
    e = {n: pixel_l2(r.read(n), o.read(vxpt.BUF[n])) for n in ("ILLUM", "PREV_ILLUM", "PREV_FAST", "OUTPUT")}
    hd = r.read("HIST_LEN") != o.read(19)
    cf = _clamp_decision_flips(r, o)
    g, c = r.read("CLAMP_DECISION").astype(int), o.read(49).astype(int)
    for (y, x) in pts:
        win = (slice(max(0, y - 6), y + 7), slice(max(0, x - 6), x + 7))
        print("f%2d (%d,%d) e illum %.1e prevIllum %.1e prevFast %.1e out %.1e | hist %.2f/%.2f | flips in 13x13 %d "
              "| max e prevIllum in 13x13 %.1e | dec %d/%d" % (
                  f, y, x, e["ILLUM"][y, x], e["PREV_ILLUM"][y, x], e["PREV_FAST"][y, x], e["OUTPUT"][y, x],
                  r.read("HIST_LEN")[y, x], o.read(19)[y, x], int(cf[win].sum()), e["PREV_ILLUM"][win].max(),
                  g[y, x], c[y, x]), flush=True)
    print("f%2d frame: prevIllum e>=1e-3 %d, >=1e-4 %d; clamp flips %d; hist differs %d" % (
        f, int((e["PREV_ILLUM"] >= 1e-3).sum()), int((e["PREV_ILLUM"] >= 1e-4).sum()), int(cf.sum()), int(hd.sum())),
        flush=True)
r.close()
