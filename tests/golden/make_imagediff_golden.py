"""Generate tests/golden/imagediff/*.png and imagediff_ref.json: image pairs and the
verdicts of the reference's OWN ImageDiff (renderer/util/ImageDiff.cpp:94-372, with its
vendored stb), compiled in place by `make -C oracle ref` into oracle/_ref/libref_imagediff.so.
Run in the build container (where /root/reference exists); the fixtures travel, the
reference does not.  The reference's diff images are stored as diff_<case>.png.

Cases cover the canonical gate's three verdicts (identical / very close / close /
different), RGB against RGBA and grey images (channels = min of the two), odd sizes and a
size mismatch (the reference returns an empty result)."""
import ctypes
import json
import os
import struct
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "imagediff")


def write_png(path, img):
    """Minimal PNG encoder (8-bit grey / RGB / RGBA, filter 0) for the fixture inputs."""
    img = np.asarray(img, np.uint8)
    if img.ndim == 2:
        img = img[..., None]
    h, w, c = img.shape
    ctype = {1: 0, 3: 2, 4: 6}[c]
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0)) +
                chunk(b"IDAT", zlib.compress(raw, 9)) + chunk(b"IEND", b""))


def cases():
    rng = np.random.default_rng(2024)
    h, w = 48, 64
    yy, xx = np.mgrid[0:h, 0:w]
    base = np.stack([xx * 4 % 256, yy * 5 % 256, (xx + yy) * 3 % 256], -1).astype(np.uint8)

    def noisy(a, s, frac=1.0):
        n = rng.normal(0.0, s, a.shape) * (rng.random(a.shape[:2] + (1,)) < frac)
        return np.clip(a.astype(np.float64) + n, 0, 255).astype(np.uint8)
    yield "identical", base, base.copy()
    yield "one_pixel", base, np.where((yy == 7) & (xx == 9), 255 - base[..., 0], base[..., 0])[..., None] * \
        np.array([1, 0, 0], np.uint8) + base * np.array([0, 1, 1], np.uint8)
    yield "lsb_noise", base, noisy(base, 0.6, 0.3)
    yield "very_close", base, noisy(base, 1.0, 0.5)
    yield "close", base, noisy(base, 4.0)
    yield "different", base, noisy(base, 30.0)
    yield "shifted", base, np.roll(base, 3, axis=1)
    odd = rng.integers(0, 256, (29, 37, 3)).astype(np.uint8)
    yield "odd_size", odd, noisy(odd, 2.0)
    rgba = np.concatenate([base, rng.integers(0, 256, (h, w, 1)).astype(np.uint8)], -1)
    yield "rgb_vs_rgba", base, rgba
    grey = base[..., 1].copy()
    yield "grey_vs_rgb", grey, base
    yield "size_mismatch", base, base[:40]


def main():
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref_imagediff.so"))
    lib.ref_image_diff.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.ref_image_diff_png.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
    os.makedirs(OUT, exist_ok=True)
    res = {}
    for name, a, b in cases():
        pa, pb = os.path.join(OUT, name + "_a.png"), os.path.join(OUT, name + "_b.png")
        write_png(pa, a)
        write_png(pb, b)
        i5 = np.zeros(5, np.int32)
        f3 = np.zeros(3, np.float32)
        lib.ref_image_diff(pa.encode(), pb.encode(), i5.ctypes.data, f3.ctypes.data)
        pd = os.path.join(OUT, "diff_" + name + ".png")
        ok = lib.ref_image_diff_png(pa.encode(), pb.encode(), pd.encode()) == 0
        res[name] = dict(different_pixels=int(i5[0]), total_pixels=int(i5[1]), is_identical=int(i5[2]),
                         is_very_close=int(i5[3]), is_close=int(i5[4]),
                         pixel_difference_ratio=float(f3[0]), rmse=float(f3[1]), ssim=float(f3[2]),
                         diff_png=("diff_" + name + ".png") if ok else None)
    with open(os.path.join(HERE, "imagediff_ref.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k, v in res.items():
        print(k, v)


if __name__ == "__main__":
    main()
