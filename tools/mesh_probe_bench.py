"""Throughput of the instanced-mesh BVH query (meshes.hip k_mesh_probe) on a leaves-heavy world:
synthetic 600-triangle meshes on N random cells of the C1 world, 1080p-many random rays.
Run under rocprofv3 --kernel-trace --stats for the kernel's own time.
python tools/mesh_probe_bench.py [instances] [rays]"""
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "real-time-path-tracing-voxel-blocks_amd"))
import vxpt  # noqa: E402


def _random_mesh_obj(path, n=600, seed=4):  # the synthetic leaves mesh of tests/test_lights.py
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        for t in range(n):
            c = rng.uniform(-0.05, 1.07, 3)
            for k in range(3):
                v = np.clip(c + rng.normal(0, 0.02 if t % 3 else 0.3, 3), -0.05, 1.07)
                f.write("v %.7f %.7f %.7f\n" % tuple(v))
        for t in range(n):
            f.write("f %d %d %d\n" % (3 * t + 1, 3 * t + 2, 3 * t + 3))


n_inst = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
n_rays = int(sys.argv[2]) if len(sys.argv) > 2 else 1920 * 1080
root = tempfile.mkdtemp()
os.makedirs(os.path.join(root, "models"))
_random_mesh_obj(os.path.join(root, "models", "leavesCube4.obj"))
r = vxpt.Renderer(64, 64)
r.load_settings()
r.generate_terrain((2, 1, 2))
r.load_models(root)
rng = np.random.default_rng(1)
cells = set()
while len(cells) < n_inst:
    cells.add((int(rng.integers(0, 64)), int(rng.integers(0, 32)), int(rng.integers(0, 64))))
for c in sorted(cells):
    r.set_block(*c, 14)
o = rng.uniform([0, 0, 0], [64, 32, 64], (n_rays, 3))
d = rng.normal(size=(n_rays, 3))
d /= np.linalg.norm(d, axis=1, keepdims=True)
rays = np.zeros((n_rays, 8), np.float32)
rays[:, 0:3], rays[:, 4:7], rays[:, 7] = o, d, 1e27
for cull in (0, 1, 1):
    t0 = time.time()
    out, ids = r.mesh_probe(rays, cull)
    dt = time.time() - t0
print("instances %d (%d triangles each), rays %d: hit fraction %.3f, call %.1f ms incl. copies"
      % (len(r.instances()), 600, n_rays, out[:, 3].mean(), dt * 1e3))
for _ in range(2):  # visibility form (k_mesh_occluded): any hit, both faces
    t0 = time.time()
    occ = r.mesh_occluded(rays)
    dt = time.time() - t0
closest, _ = r.mesh_probe(rays, 0)
assert (occ == closest[:, 3].astype(np.uint8)).all(), "any-hit and closest-hit disagree"
print("occluded: fraction %.3f, call %.1f ms incl. copies" % (occ.mean(), dt * 1e3))
