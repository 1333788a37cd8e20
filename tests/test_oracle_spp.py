"""The oracle's spp > 1 frame (orc_trace_frame_spp, the benchmarked C3 frame of SURVEY §8d /
DESIGN.md §7) equals the same frame composed from the oracle's 1-spp primitives in Python: passes
at iterationIndex f*spp + s, pass s > 0 reusing pass s-1 (its depth / normal / material planes and
the frame's own camera as ReSTIR history), binary32 average r * (1/spp) added in pass order, the
denoiser's history copies and history camera as the previous frame left them, one denoise."""
import numpy as np

import oracle
from golden.make_golden import C1_CAMERA

DN = ([30, 6, 2, 0.5, 0.15, 0.003, 0.01, 0.05, 500000], [1, 1, 1, 1, 1, 1])
W, H, SPP = 48, 32, 3
NR, DEPTH, MAT, PREV_NR, PREV_DEPTH, PREV_MAT = 2, 1, 5, 8, 12, 13


def _make():
    o = oracle.Oracle(W, H)
    o.terrain((2, 1, 2))
    o.set_sky()
    o.set_denoise_params(*DN)
    return o


def _cams():
    pos, d, fov = C1_CAMERA
    moved = (pos[0] + 0.3, pos[1] + 0.05, pos[2] - 0.2)
    return [(pos, d), (pos, d), (moved, (d[0] + 0.03, d[1], d[2]))]


def test_spp_frame_equals_composed_passes():
    a, b = _make(), _make()
    scale = np.float32(1.0) / np.float32(SPP)
    prev = _cams()[0]
    for f, cur in enumerate(_cams()):
        for o in (a, b):
            o.set_camera(*cur, fov=90.0)
            o.set_camera(*prev, fov=90.0, which=1)
        a.render_frame(f, SPP)
        # b: the same frame from 1-spp passes
        hist = {k: b.read(k) for k in (PREV_NR, PREV_DEPTH, PREV_MAT)}
        acc = np.zeros((H, W, 4), np.float32)
        for s in range(SPP):
            if s > 0:
                b.write(PREV_NR, b.read(NR))
                b.write(PREV_DEPTH, b.read(DEPTH))
                b.write(PREV_MAT, b.read(MAT))
                b.set_camera(*cur, fov=90.0, which=1)
            b.trace(f * SPP + s)
            b.post_trace()
            r = b.read(0)
            base = np.zeros_like(acc) if s == 0 else acc
            acc = base.copy()
            acc[..., :3] = base[..., :3] + r[..., :3] * scale
            acc[..., 3] = r[..., 3]
        for k, v in hist.items():
            b.write(k, v)
        b.set_camera(*prev, fov=90.0, which=1)
        b.write(0, acc)
        b.denoise(f, f * SPP + SPP)
        for k in (0, 1, 2, 14, 17, 18, 19, 21):
            np.testing.assert_array_equal(a.read(k).view(np.uint8), b.read(k).view(np.uint8), err_msg="frame %d buf %d" % (f, k))
        prev = cur
    # the average is not any single pass's radiance
    single = _make()
    single.set_camera(*prev, fov=90.0)
    single.set_camera(*prev, fov=90.0, which=1)
    single.trace(0)
    assert not np.array_equal(single.read(0), a.read(0))


def test_spp1_frame_is_the_plain_pass():
    a, b = _make(), _make()
    pos, d, fov = C1_CAMERA
    for o in (a, b):
        o.set_camera(pos, d, fov=fov)
        o.set_camera(pos, d, fov=fov, which=1)
    for f in range(2):
        a.render_frame(f, 1)
        b.trace(f)
        b.post_trace()
        b.denoise(f, f + 1)
        for k in (0, 14, 21):
            np.testing.assert_array_equal(a.read(k).view(np.uint8), b.read(k).view(np.uint8))
