"""Textured shading: TextureManager's mip chains
(TextureManager.cu:58-117, 216-414) and the closest-hit texture path
(closesthit.cu:167-254: world-grid uv, ray-cone lod, albedo / roughness /
metallic / normal maps).

The reference compresses to BC7/BC5/BC4 with NVTT, which is not reproducible
here: the texels are the uncompressed RGBA8 ones (documented deviation), so
parity is pinned against the oracle restatement on synthetic textures written
by this test (gray, gray+alpha, RGB and RGBA PNGs; the real asset PNGs are
not shipped to the GPU box).  CPU: the PNG decoder against the encoder below.
GPU: the loaded mip chains equal a numpy restatement bit for bit; G-buffers and
radiance of textured frames match the oracle given the same texels.
"""
import os
import shutil
import struct
import zlib

import numpy as np
import pytest

import oracle
import vxpt
from golden.make_golden import C1_CAMERA
from test_gpu_parity import E_MAX_TEXTURED, _compare_radiance, _inject_sky, DN_FLOATS, DN_INTS

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(REPO, "data")


def write_png8(path, img):
    """Minimal PNG encoder: 8-bit gray (H,W), gray+alpha (H,W,2), RGB (H,W,3) or RGBA (H,W,4);
    rows alternate filter types 0 and 1 (None, Sub)."""
    img = np.asarray(img, np.uint8)
    if img.ndim == 2:
        img = img[..., None]
    h, w, ch = img.shape
    ct = {1: 0, 2: 4, 3: 2, 4: 6}[ch]
    raw = bytearray()
    for y in range(h):
        row = img[y].reshape(-1).astype(np.int32)
        if y % 2 == 0:
            raw += b"\x00" + bytes(row.astype(np.uint8))
        else:
            sub = row.copy()
            sub[ch:] = (row[ch:] - row[:-ch]) & 255
            raw += b"\x01" + bytes(sub.astype(np.uint8))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ct, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(bytes(raw))) + chunk(b"IEND", b"")
    open(path, "wb").write(png)


def rgba0(img):
    """Level 0 as the loader expands it: 1ch -> (v,0,0,255), 2ch -> (v,a,0,255), 3ch -> (r,g,b,255)."""
    img = np.asarray(img, np.uint8)
    if img.ndim == 2:
        img = img[..., None]
    h, w, ch = img.shape
    out = np.zeros((h, w, 4), np.uint8)
    out[..., 3] = 255
    if ch == 1:
        out[..., 0] = img[..., 0]
    elif ch == 2:
        out[..., 0], out[..., 1] = img[..., 0], img[..., 1]
    else:
        out[..., :ch] = img
    return out


def mip_chain(img):
    """fillFirstMipmapKernel + fillMipmapKernel (TextureManager.cu:58-117): 2x2 averages, truncated."""
    lv = [rgba0(img)]
    size = lv[0].shape[0]
    max_lod = int(np.log2(size)) - 2
    for _ in range(max_lod):
        p = lv[-1].astype(np.int32)
        q = (p[0::2, 0::2] + p[0::2, 1::2] + p[1::2, 0::2] + p[1::2, 1::2]).astype(np.float32) / np.float32(4.0)
        lv.append(np.minimum(q, 255.0).astype(np.uint8))
    return lv


def _synthetic(rng, n, ch, smooth=True):
    yy, xx = np.mgrid[0:n, 0:n].astype(np.float32)
    base = []
    for c in range(ch):
        f = 0.5 + 0.45 * np.sin(2 * np.pi * (xx * (c + 1) / n + yy * (2 - c % 2) / n) + c)
        base.append(f * 255 + rng.uniform(-30, 30, (n, n)) * (not smooth))
    img = np.clip(np.stack(base, -1), 0, 255).astype(np.uint8)
    return img[..., 0] if ch == 1 else img


# block -> (material, {kind: (file, size, channels)})
TEX = {
    1: ("sand", {"albedo": ("sand_a.png", 64, 3), "normal": ("sand_n.png", 64, 3), "roughness": ("sand_r.png", 64, 1)}),
    2: ("soil", {"albedo": ("soil_a.png", 32, 4), "roughness": ("soil_r.png", 32, 2)}),
    3: ("cliff", {"albedo": ("cliff_a.png", 128, 3), "normal": ("cliff_n.png", 128, 3), "metallic": ("cliff_m.png", 16, 1)}),
    7: ("rocks", {"normal": ("rocks_n.png", 16, 3)}),
}
KINDS = ("albedo", "normal", "roughness", "metallic")


def make_data_dir(root):
    """A data directory whose materials name synthetic textures (everything else the repo's)."""
    rng = np.random.default_rng(11)
    os.makedirs(os.path.join(root, "assets"))
    os.makedirs(os.path.join(root, "textures"))
    for d in ("settings", "tables", "scene"):
        shutil.copytree(os.path.join(DATA, d), os.path.join(root, d))
    shutil.copy(os.path.join(DATA, "assets", "blocks.yaml"), os.path.join(root, "assets"))
    images = {}
    lines = []
    for ln in open(os.path.join(DATA, "assets", "materials.yaml")):
        if ln.strip().startswith("textures:"):
            continue
        lines.append(ln.rstrip("\n"))
        if ln.strip().startswith("- id:"):
            mid = ln.strip()[5:].strip()
            for b, (name, kinds) in TEX.items():
                if name == mid:
                    parts = []
                    for k, (fn, n, ch) in kinds.items():
                        img = _synthetic(rng, n, ch, smooth=(k != "albedo"))
                        write_png8(os.path.join(root, "textures", fn), img)
                        images["textures/" + fn] = img
                        parts.append("%s: textures/%s" % (k, fn))
                    lines.append("    textures: {" + ", ".join(parts) + "}")
    open(os.path.join(root, "assets", "materials.yaml"), "w").write("\n".join(lines) + "\n")
    return images


def test_png_decoder_channel_types(tmp_path):
    rng = np.random.default_rng(2)
    for ch in (1, 2, 3, 4):
        img = rng.integers(0, 256, (24, 40, ch) if ch > 1 else (24, 40), dtype=np.uint8)
        p = str(tmp_path / ("t%d.png" % ch))
        write_png8(p, img)
        got = vxpt.read_png(p)
        np.testing.assert_array_equal(got.reshape(img.shape), img)


def test_mip_chain_restatement():
    img = _synthetic(np.random.default_rng(0), 16, 3)
    lv = mip_chain(img)
    assert [l.shape[0] for l in lv] == [16, 8, 4]
    assert (lv[1][0, 0] == ((rgba0(img)[:2, :2].astype(int).sum((0, 1))) // 4)).all()


@pytest.fixture(scope="module")
def textured(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("texdata"))
    images = make_data_dir(root)
    w, h = 128, 96
    r = vxpt.Renderer(w, h, data_dir=root)
    r.load_settings()
    r.generate_terrain((2, 1, 2), height_scale=32.0)
    cam = (C1_CAMERA[0], C1_CAMERA[1], C1_CAMERA[2])
    r.set_camera(*cam[:2], fov=cam[2], prev=cam)
    r.set_sky(0.25, 45.0, 0.0, 1.0)
    n = r.load_textures()
    yield r, images, n, cam
    r.close()


@pytest.mark.gpu
def test_texture_mip_chains_bit_exact(textured):
    r, images, n, _ = textured
    paths = sorted(images)
    assert n == len(paths)
    table, total = r.texture_table()
    texels = r.read("TEXELS")
    for i, pth in enumerate(paths):
        size, max_lod, offs = table[i]
        exp = mip_chain(images[pth])
        assert size == exp[0].shape[0] and max_lod == len(exp) - 1, pth
        for l, lv in enumerate(exp):
            got = texels[offs[l]:offs[l] + lv.shape[0] * lv.shape[1]].reshape(lv.shape)
            np.testing.assert_array_equal(got, lv, err_msg="%s level %d" % (pth, l))


@pytest.mark.gpu
def test_textured_frames_match_oracle(textured):
    r, images, _, cam = textured
    w, h = r.W, r.H
    o = oracle.Oracle(w, h)
    o.terrain((2, 1, 2))
    o.set_camera(*cam[:2], fov=cam[2])
    o.set_camera(*cam[:2], fov=cam[2], which=1)
    o.set_denoise_params(DN_FLOATS, DN_INTS)
    paths = sorted(images)
    o.set_textures([mip_chain(images[p]) for p in paths])
    for b, (_, kinds) in TEX.items():
        ids = [paths.index("textures/" + kinds[k][0]) if k in kinds else -1 for k in KINDS]
        o.set_material_textures(b, *ids, uv_scale=2.5, world_grid=True)
    _inject_sky(r, o)
    r.trace(0)
    o.trace(0)
    # G-buffer: textured albedo, perturbed normals, texture roughness / metallic
    for name in ("DEPTH", "NORMAL_ROUGH", "ALBEDO", "MAT_PARAM", "GEO_NORMAL_THIN"):
        g, c = r.read(name), o.read(vxpt.BUF[name])
        bad = ~np.isclose(g, c, rtol=2e-4, atol=2e-4)
        assert bad.mean() < 1e-3, (name, bad.mean(), np.argwhere(bad)[:5])
    alb = r.read("ALBEDO")[..., :3]
    assert alb.std() > 0.05  # the textures really modulate the albedo
    _compare_radiance(r.read("ILLUM"), o.read(0), "textured frame0", E_MAX_TEXTURED)
    p = vxpt.DenoiseParams(*DN_FLOATS, *DN_INTS)
    r.denoise(0, 1, p)
    o.post_trace()
    o.denoise(0, 1)
    for f in range(1, 3):
        r.trace(f)
        r.denoise(f, f + 1, p)
        o.trace(f)
        o.post_trace()
        o.denoise(f, f + 1)
        _compare_radiance(r.read("ILLUM"), o.read(0), "textured frame%d" % f, E_MAX_TEXTURED)
        _compare_radiance(r.read("OUTPUT"), o.read(21), "textured output %d" % f, E_MAX_TEXTURED)
    # textures off again: the untextured path
    r.enable_textures(False)
    r.trace(3)
    assert np.allclose(r.read("ALBEDO")[..., :3][r.read("DEPTH") < 1e20], 1.0)
    r.enable_textures(True)
