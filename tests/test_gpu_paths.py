"""GPU parity of the hot-path branches the default scenes never reach:

- the specular chain: mirror (roughness 0), dielectric (roughness 0,
  translucency 1), metallic and coloured materials, so path segments 1.. run
  (RayGen.cu:146-173, Bsdf.h:202-245, closesthit.cu:216-305), at the
  reference's bounce limits 3/1 and at 4/4 (every segment diffuse-shaded);
- the C3 world (256^3 voxels, 8x8x8 chunks): DDA probe bit-exact, incl. the
  straggler hand-over state (dda_save / dda_resume), and two frames of trace +
  denoise with the straggler queues asserted non-empty;
- the firefly filter's outlier branch (FireflyFilter.h:131-220) on injected
  outlier reservoirs.

Radiance bars: test_gpu_parity.check_radiance (per-pixel relative L2).
"""
import numpy as np
import pytest

import oracle
import vxpt
from golden.make_golden import C1_CAMERA
from test_gpu_parity import DN_FLOATS, DN_INTS, _dn_params, _inject_frame, _inject_sky, _rel, check_radiance
from test_oracle import _random_rays

pytestmark = pytest.mark.gpu

# block ids of the C1 terrain and the material ids the C1 camera sees: 1 sand (0), 2 soil (1),
# 3 cliff (2) are visible, 7 rocks (6) only to secondary rays
SPECULAR_MATS = [dict(albedo=(0.9, 0.9, 0.9), roughness=0.8, material_id=i) for i in range(12)]
SPECULAR_MATS[0] = dict(albedo=(0.95, 0.9, 0.85), roughness=0.0, material_id=0)                  # mirror
SPECULAR_MATS[2] = dict(albedo=(0.9, 0.95, 1.0), roughness=0.0, translucency=1.0, material_id=2)  # dielectric
SPECULAR_MATS[1] = dict(albedo=(0.8, 0.6, 0.3), roughness=0.3, metallic=1, material_id=1)        # rough metal
SPECULAR_MATS[6] = dict(albedo=(0.3, 0.7, 0.4), roughness=0.5, material_id=6)                    # coloured


def _setup(w, h, bounces, mats=None):
    r = vxpt.Renderer(w, h, bounces=bounces)
    r.load_settings()
    r.generate_terrain((2, 1, 2), height_scale=32.0)
    cam = (C1_CAMERA[0], C1_CAMERA[1], C1_CAMERA[2])
    r.set_camera(*cam[:2], fov=cam[2], prev=cam)
    r.set_sky(0.25, 45.0, 0.0, 1.0)
    o = oracle.Oracle(w, h, bounces=bounces)
    o.terrain((2, 1, 2))
    o.set_camera(*cam[:2], fov=cam[2])
    o.set_camera(*cam[:2], fov=cam[2], which=1)
    o.set_denoise_params(DN_FLOATS, DN_INTS)
    if mats is not None:
        r.upload_materials(mats)
        o.set_materials(mats)
    _inject_sky(r, o)
    return r, o


@pytest.mark.parametrize("bounces", [(3, 1), (4, 4)])
def test_specular_chain_matches_oracle(bounces):
    r, o = _setup(128, 96, bounces, SPECULAR_MATS)
    p = _dn_params()
    for f in range(4):
        r.trace(f)
        cnt = r.trace_counters()
        r.denoise(f, f + 1, p)
        o.trace(f)
        o.post_trace()
        o.denoise(f, f + 1)
        check_radiance(r.read("ILLUM"), o.read(0), "bounces %s frame%d illum" % (bounces, f))
        check_radiance(r.read("OUTPUT"), o.read(21), "bounces %s frame%d output" % (bounces, f))
        for name in ("DEPTH", "MATERIAL", "NORMAL_ROUGH", "ALBEDO", "MAT_PARAM"):
            np.testing.assert_allclose(r.read(name), o.read(vxpt.BUF[name]), rtol=1e-6, atol=1e-7, err_msg=name)
        # segment 1 ran: BRDF-candidate and NEE rays queued from second-segment hits
        assert cnt[5, 0] > 0 and cnt[6, 0] > 0, cnt[:12]
        if bounces == (4, 4):
            assert cnt[9, 0] > 0 and cnt[13, 0] > 0, cnt  # segments 2 and 3
    # the primary G-buffer sees the mirror, metal and dielectric blocks
    mat = r.read("MATERIAL")
    assert (mat == 0).any() and (mat == 1).any() and (mat == 2).any()
    r.close()


def test_dielectric_branch_refracts():
    """A pure dielectric world: primary hits sample reflection or refraction by
    the Fresnel term (Bsdf.h:218-245); the refracted rays re-enter the cell
    they face and are shaded as diffuse (the path's roughness regularisation)."""
    mats = [dict(albedo=(1.0, 1.0, 1.0), roughness=0.0, translucency=1.0, material_id=i) for i in range(12)]
    r, o = _setup(96, 64, (3, 1), mats)
    for f in range(2):
        r.trace(f)
        o.trace(f)
        check_radiance(r.read("ILLUM"), o.read(0), "dielectric frame%d" % f)
    r.close()


C3_CHUNKS = (8, 8, 8)


@pytest.fixture(scope="module")
def c3():
    w, h = 256, 144
    pos = tuple(p * 4 for p in C1_CAMERA[0])
    r = vxpt.Renderer(w, h)
    r.load_settings()
    r.generate_terrain(C3_CHUNKS, height_scale=128.0, freq_den=256.0, global_y=True)
    r.set_camera(pos, C1_CAMERA[1], fov=90.0, prev=(pos, C1_CAMERA[1], 90.0))
    r.set_sky(0.25, 45.0, 0.0, 1.0)
    o = oracle.Oracle(w, h)
    o.terrain(C3_CHUNKS, height_scale=128.0, freq_den=256.0, global_y=True)
    o.set_camera(pos, C1_CAMERA[1], fov=90.0)
    o.set_camera(pos, C1_CAMERA[1], fov=90.0, which=1)
    o.set_denoise_params(DN_FLOATS, DN_INTS)
    _inject_sky(r, o)
    yield r, o, pos
    r.close()


def test_c3_voxels_bit_exact(c3):
    r, o, _ = c3
    v = r.read("VOXELS")
    np.testing.assert_array_equal(v, o.voxels())
    assert v.size == 256 ** 3 and 0.05 < (v != 0).mean() < 0.95


@pytest.mark.parametrize("outside", [False, True])
def test_c3_dda_probe_bit_exact(c3, outside):
    """Long walks over the 256^3 world: the octant empty-cube tables and the
    chunk-boundary faces of 512 chunks; closest hits through dda_closest and
    through the straggler hand-over (save/resume after every iteration)."""
    r, o, pos = c3
    rays = _random_rays(30000, 41 + outside, world=(256, 256, 256), outside=outside)
    # a quarter of the rays from the camera position, as the camera and its BRDF rays see the world
    rays[: len(rays) // 4, 0:3] = np.float32(pos)
    c, tc = o.rays(rays, 0)
    for mode in (0, 4):
        g, tg = r.probe_rays(rays, mode)
        np.testing.assert_array_equal(g, c, err_msg="mode %d" % mode)
        np.testing.assert_array_equal(tg.view(np.uint32), tc.view(np.uint32), err_msg="mode %d" % mode)
    assert c[:, 0].mean() > 0.2
    rays[:, 6] = 1e-3
    rays[:, 7] = np.random.default_rng(5).uniform(1.0, 300.0, len(rays)).astype(np.float32)
    c, _ = o.rays(rays, 2)
    for mode in (2, 6):
        g, _ = r.probe_rays(rays, mode)
        np.testing.assert_array_equal(g[:, 0], c[:, 0], err_msg="mode %d" % mode)


def test_c3_frames_with_stragglers(c3):
    """Two frames of trace + denoise on the C3 world; the walks that exceed the
    iteration cap go through k_queue -> straggler queue -> k_resume."""
    r, o, _ = c3
    p = _dn_params()
    for f in range(2):
        r.trace(f)
        cnt = r.trace_counters()
        r.denoise(f, f + 1, p)
        o.trace(f)
        o.post_trace()
        o.denoise(f, f + 1)
        for name in ("DEPTH", "MATERIAL", "NORMAL_ROUGH"):
            np.testing.assert_allclose(r.read(name), o.read(vxpt.BUF[name]), rtol=1e-6, atol=1e-7, err_msg=name)
        check_radiance(r.read("ILLUM"), o.read(0), "c3 frame%d illum" % f)
        check_radiance(r.read("OUTPUT"), o.read(21), "c3 frame%d output" % f)
        print("queues (rays, level-1, level-2 stragglers):", cnt[:4].tolist())
        # BRDF-candidate and NEE queues sent walks through the straggler hand-over; the
        # ReSTIR queue has rays once there is a previous pass to reuse
        assert (cnt[1:3, 0] > 0).all() and (cnt[1:3, 1] > 0).all(), cnt[:4]
        if f > 0:
            assert cnt[3, 0] > 0 and cnt[3, 1] > 0, cnt[:4]


def test_firefly_outlier_branch_fires():
    """Injected outlier reservoirs (weightSum x1e4 on isolated pixels) are
    detected and filtered (colour from the 3x3 edge-stopping filter, reservoir
    replaced by a neighbour's or clamped) exactly as the oracle does."""
    r, o = _setup(64, 48, (3, 1))
    r.trace(0)
    p = _dn_params()
    rng = np.random.default_rng(17)
    for f in range(3):
        r.trace(f)
        o.trace(f)
        o.post_trace()
        # reservoirs: two W*H halves, the pass of iterationIndex f wrote half f % 2
        res = o.read(vxpt.BUF["RESERVOIRS"])
        half = res.size // 2
        cur = res[(f % 2) * half:(f % 2 + 1) * half]
        depth = o.read(vxpt.BUF["DEPTH"]).reshape(-1)
        cand = np.nonzero((cur["lightData"] != 0) & (cur["weightSum"] > 0) & (depth < 5e5))[0]
        pick = np.sort(rng.choice(cand, size=min(200, len(cand)), replace=False))
        # at most one outlier per 8x4 detection tile (FireflyFilter.h:51-65 averages the tile)
        tile = (pick % 64) // 8 + 8 * ((pick // 64) // 4)
        pick, tile = pick[np.unique(tile, return_index=True)[1]][:40], np.unique(tile)[:40]
        # 1e4 x the largest weight in the tile: an outlier whatever the tile's other samples
        ws = cur["weightSum"].reshape(48 // 4, 4, 64 // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 32)
        cur["weightSum"][pick] = np.maximum(ws[tile].max(1) * 1e4, 10.0).astype(np.float32)
        illum = o.read(0)
        illum.reshape(-1, 4)[pick, :3] *= 50.0
        o.write(vxpt.BUF["RESERVOIRS"], res)
        o.write(0, illum)
        _inject_frame(r, o)
        before = cur["weightSum"][pick].copy()
        r.denoise(f, f + 1, p)
        o.denoise(f, f + 1)
        gres = r.read("RESERVOIRS")
        ores = o.read(vxpt.BUF["RESERVOIRS"])
        for fld in ("lightData", "uvData", "weightSum", "targetPdf", "M"):
            np.testing.assert_array_equal(gres[fld], ores[fld], err_msg=fld)
        assert (ores["weightSum"][(f % 2) * half + pick] < before).all()
        gcur = gres[(f % 2) * half:(f % 2 + 1) * half]
        fired = (gcur["weightSum"][pick] < before).mean()
        assert fired == 1.0, fired
        for name in ("OUTPUT", "PREV_ILLUM"):
            rel = _rel(r.read(name), o.read(vxpt.BUF[name]))
            assert rel.max() < 1e-4, (f, name, rel.max())
        # the filtered radiance written back to the plane
        rel = _rel(r.read("ILLUM"), o.read(0))
        assert rel.max() < 1e-5, (f, "ILLUM", rel.max())
    r.close()
