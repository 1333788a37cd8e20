"""Generate the golden fixtures under tests/golden/ (run in the build container,
where /root/reference exists; the fixtures travel, the reference does not).

noise_ref.npz  -- outputs of the reference's OWN terrain noise generator
                  (voxelengine/Noise.cpp + ext/PerlinNoise.hpp, compiled in
                  place by `make -C oracle ref` into oracle/_ref/libref_noise.so)
                  at every column the C1 (2x1x2 chunks, freq 1/64) and C3
                  (8x8x8 chunks, freq 1/256) terrains sample
                  (VoxelSceneGen.cu:361-381), plus the two SURVEY §8c KAT points.
oracle_c1.npz  -- the oracle's own C1 render at 64x48 (regression pin of the
                  restatement itself; NOT reference-derived).
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def noise_points(n, freq_den):
    g = np.arange(n, dtype=np.float32)
    freq = np.float32(1.0) / np.float32(freq_den)
    gx, gz = np.meshgrid(g * freq, g * freq)  # row = z, col = x
    return np.stack([gx.ravel(), gz.ravel()], 1).astype(np.float32)


POINTS = {"c1": (64, 64.0), "c3": (256, 256.0)}
KAT_XY = np.array([[0.0, 0.0], [10.0 / 64.0, 5.0 / 64.0]], np.float32)

C1_CAMERA = ([35.6184, 11.8733, 42.0387], [-0.321564, -0.0129988, -0.946799], 90.0)
DENOISE_DEFAULT = ([30, 6, 2, 0.5, 0.15, 0.003, 0.01, 0.05, 500000], [1, 1, 1, 1, 1, 1])


def make_noise():
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref_noise.so"))
    lib.ref_noise.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    out = {}
    for k, (n, fd) in list(POINTS.items()) + [("kat", (0, None))]:
        xy = KAT_XY if fd is None else noise_points(n, fd)
        r = np.zeros(len(xy), np.float32)
        lib.ref_noise(4, 124, len(xy), xy.ctypes.data, r.ctypes.data)
        out[k] = r
    np.savez_compressed(os.path.join(HERE, "noise_ref.npz"), **out)


def make_oracle_c1():
    import oracle
    o = oracle.Oracle(64, 48)
    o.terrain((2, 1, 2))
    o.set_camera(*C1_CAMERA[:2], fov=C1_CAMERA[2])
    o.set_camera(*C1_CAMERA[:2], fov=C1_CAMERA[2], which=1)
    o.set_sky()
    o.set_denoise_params(*DENOISE_DEFAULT)
    outs = {}
    for f in range(2):
        o.trace(f)
        if f == 0:
            outs["depth"] = o.read(1)
            outs["normal_rough"] = o.read(2)
            outs["illum0"] = o.read(0)
        o.post_trace()
        o.denoise(f, f + 1)
    outs["output1"] = o.read(21)
    outs["hist1"] = o.read(19)
    np.savez_compressed(os.path.join(HERE, "oracle_c1.npz"), **outs)


if __name__ == "__main__":
    make_noise()
    make_oracle_c1()
    print("wrote", os.listdir(HERE))
