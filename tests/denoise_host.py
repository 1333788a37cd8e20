"""Test helper (CPU): the library's temporal accumulation and history clamping (denoise.hip, run on the host
by tests/native/denoise_driver.hip) against the oracle's passes on the oracle's own inputs, frame by
frame, through the lantern-edit scenario of tests/test_gpu_meshes.py.
Usage: python tests/denoise_host.py DRIVER [firefly 0/1]"""
import os, shutil, sys, subprocess, tempfile
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(R, d) for d in ("tests", "oracle", "real-time-path-tracing-voxel-blocks_amd")]
import numpy as np
import oracle
import test_gpu_meshes as T
from test_lights import _base_obj, _prism_obj, _random_mesh_obj
from golden.make_golden import C1_CAMERA


def dump(o, path, mode, fl, ints):
    with open(path, "wb") as f:
        f.write(np.array([o.W, o.H, mode], np.int32).tobytes())
        f.write(np.asarray(o.camera_info(0), np.float32)[:32].tobytes())
        f.write(np.asarray(o.camera_info(1), np.float32)[:32].tobytes())
        f.write(np.asarray(fl, np.float32).tobytes())
        f.write(np.asarray(ints, np.int32).tobytes())
        for k in (0, 2, 7, 8, 17, 18, 15, 16):
            f.write(np.ascontiguousarray(o.read(k), np.float32).tobytes())
        for k in (1, 5, 12, 19, 20):
            f.write(np.ascontiguousarray(o.read(k), np.float32).tobytes())


def rel(a, b):
    return np.abs(a - b) / np.maximum(np.maximum(np.abs(a), np.abs(b)), 1e-6)


class Scene:
    """The lantern scene of tests/test_gpu_meshes.py on the oracle (128x96, C1 camera) and its edit
    schedule: remove the last lantern at frame 2, the first at 4, re-add the last at 6."""

    def __init__(self, ff):
        self.dir = d = tempfile.mkdtemp(); os.makedirs(d + "/models")
        _prism_obj(d + "/models/lanternLight.obj"); _base_obj(d + "/models/lanternBase.obj")
        _random_mesh_obj(d + "/models/leavesCube4.obj", n=120)
        self.o = o = oracle.Oracle(128, 96)
        o.terrain(T.CH)
        self.ids = o.voxels()
        placed = T.place_meshes(self.ids)
        o.set_voxels(self.ids, T.CH)
        cam = (C1_CAMERA[0], C1_CAMERA[1], C1_CAMERA[2])
        o.set_camera(*cam[:2], fov=cam[2]); o.set_camera(*cam[:2], fov=cam[2], which=1)
        o.set_sky(0.25, 45.0, 0.0, 1.0)
        self.ints = list(T.DN_INTS)
        self.ints[4] = ff
        o.set_denoise_params(T.DN_FLOATS, self.ints)
        self.defs, params = T.asset_tables()
        for b, p in params.items():
            o.set_material(b, **p)
        self.models = {b: oracle.parse_obj(d + "/models/" + f) for b, f in
                       ((T.LIGHT, "lanternLight.obj"), (T.BASE, "lanternBase.obj"), (T.LEAVES, "leavesCube4.obj"))}
        o.set_meshes(self.models, self.defs)
        self.first, self.width = min(self.defs), T.CH[0] * 32
        lanterns = sorted((p for p in placed if p[3] == T.LIGHT),
                          key=lambda p: oracle.instance_id(self.first, self.width, T.LIGHT - 1, *p[:3]))
        self.edits = {2: (lanterns[-1], 0), 4: (lanterns[0], 0), 6: (lanterns[-1], T.LIGHT)}

    def trace(self, f, edits=True):
        """The frame's edit (if any), trace and post-trace copies."""
        o = self.o
        if edits and f in self.edits:
            (x, y, z, _), b = self.edits[f]
            self.ids[T._idx(x, y, z)] = b
            o.set_voxels(self.ids, T.CH)
            o.set_prev_scene_empty(True)
            o.light_edit(oracle.instance_id(self.first, self.width, T.LIGHT - 1, x, y, z), removed=b == 0)
            o.set_meshes(self.models, self.defs, light_update="update")
        o.trace(f); o.set_prev_scene_empty(False); o.post_trace()

    def close(self):
        shutil.rmtree(self.dir, ignore_errors=True)


def run(driver, ff):
    """Per frame (from 1): max relative differences (temporal ping, pong, history length; clamped
    history, fast history, history length) of the library's code vs the oracle's."""
    sc = Scene(ff)
    o, d, ints, W, H = sc.o, sc.dir, sc.ints, 128, 96
    worst, stats = 0.0, []
    for f in range(8):
        sc.trace(f)
        if f > 0:
            snap = {k: o.read(k).copy() for k in (0, 14, 15, 16, 17, 18, 19, 20, 21)}
            it = f + 1
            if ff:
                o.run_pass(0, (it - 1) & 1, 0)
            o.run_pass(1)
            st, out = os.path.join(d, "s.bin"), os.path.join(d, "o.bin")
            dump(o, st, 0, T.DN_FLOATS, ints)
            subprocess.run([driver, st, out], check=True)
            n = W * H
            g = np.fromfile(out, np.float32)
            gp, gq, gh = g[:4 * n].reshape(H, W, 4), g[4 * n:8 * n].reshape(H, W, 4), g[8 * n:].reshape(H, W)
            o.run_pass(2)
            rt = [rel(gp, o.read(15)).max(), rel(gq, o.read(16)).max(), rel(gh, o.read(19)).max()]
            o.run_pass(3)
            dump(o, st, 1, T.DN_FLOATS, ints)
            subprocess.run([driver, st, out], check=True)
            g = np.fromfile(out, np.float32)
            hi, hf, hh = g[:4 * n].reshape(H, W, 4), g[4 * n:8 * n].reshape(H, W, 4), g[8 * n:].reshape(H, W)
            o.run_pass(4)
            e = rel(hi[..., :3], o.read(17)[..., :3]).max(-1)
            rc = [e.max(), rel(hf, o.read(18)).max(), rel(hh, o.read(20)).max()]
            bad = np.argwhere(e > 1e-4)
            print("frame %d temporal max rel ping %.2e pong %.2e hist %.2e | clamp prevIllum %.2e prevFast %.2e hist %.2e"
                  " | clamp pixels > 1e-4: %d %s" % (f, *rt, *rc, len(bad), [tuple(v[::-1]) for v in bad[:6]]), flush=True)
            worst = max(worst, max(rt + rc))
            stats.append((f, rt, rc))
            for k, v in snap.items():
                o.write(k, v)
        o.denoise(f, f + 1)
    print("worst", worst)
    sc.close()
    return stats


def chained_divergence(eps, frames=7, edits=True, seed=1):
    """The oracle's denoised frames with and without a relative perturbation `eps` of every frame's
    radiance (the size of the GPU's rounding differences): per frame, the largest per-pixel L2 of
    the clamped history and the fraction of output pixels within 1e-4."""
    from test_gpu_parity import pixel_l2
    runs = []
    for e in (0.0, eps):
        rng = np.random.default_rng(seed)
        sc = Scene(1)
        out = []
        for f in range(frames):
            sc.trace(f, edits)
            if e:
                il = sc.o.read(0).copy()
                il[..., :3] *= (1 + e * rng.standard_normal(il[..., :3].shape)).astype(np.float32)
                sc.o.write(0, il)
            sc.o.denoise(f, f + 1)
            out.append((sc.o.read(17).copy(), sc.o.read(21).copy()))
        sc.close()
        runs.append(out)
    return [(float(pixel_l2(b[0], a[0]).max()), float((pixel_l2(b[1], a[1]) < 1e-4).mean()))
            for a, b in zip(*runs)]


if __name__ == "__main__":
    run(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
