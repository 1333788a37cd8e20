"""Instanced block meshes and their emissive-triangle lights (first slice):
the OBJ reader (ObjUtils.cpp:13-120), the instance set of a world (BlockManager +
VoxelEngine::collectInstanceTransforms, VoxelEngine.cu:323-384), the light records
(generateLightInfosKernel + TriangleLight::Store, VoxelEngine.cu:53-116, Light.h:124-137) and
their alias table (buildAliasTable / AliasTable::update, VoxelEngine.cu:150-192,
AliasTable.cu:58-131).

The reference's OBJ assets are not shipped here: the meshes are synthetic OBJ files written by
the tests (a lantern-like emissive prism and a base), so the light table is pinned by the
oracle restatement (oracle/orc_lights.cpp, oracle.collect_instances / alias_table) and by
known answers (IEEE f16 rounding against numpy, octahedral encodings of the axes).
Bit-exact: instance rows, light records, weights and alias bins.
"""
import os
import shutil

import numpy as np
import pytest

import oracle
import vxpt

CH = (2, 1, 2)
LIGHT, BASE = 16, 15
BLOCKS = {b: dict(instanced=True, light_base=(BASE if b == LIGHT else 0)) for b in range(13, 30)}


def _idx(x, y, z, chunks=CH):
    cx, cy, cz = chunks
    return ((x >> 5) + cx * ((z >> 5) + cz * (y >> 5))) * 32768 + (x & 31) + 32 * ((z & 31) + 32 * (y & 31))


def _prism_obj(path, lo=0.28, hi=0.72, y0=0.07, y1=0.62):
    """An open four-sided prism (8 triangles, like the lantern's light) with texcoords."""
    v = [(lo, y0, lo), (hi, y0, lo), (hi, y0, hi), (lo, y0, hi), (lo, y1, lo), (hi, y1, lo), (hi, y1, hi), (lo, y1, hi)]
    faces = []
    for a, b in ((0, 1), (1, 2), (2, 3), (3, 0)):
        faces += [(a, b, b + 4), (a, b + 4, a + 4)]
    with open(path, "w") as f:
        f.write("# synthetic emissive prism\n")
        for p in v:
            f.write("v %.6f %.6f %.6f\n" % p)
        f.write("vt 0.375 0.5\nvt 0.625 0.5\n")
        for k, (a, b, c) in enumerate(faces):
            f.write("f %d/1 %d/2 %d/%d\n" % (a + 1, b + 1, c + 1, 1 + k % 2))


def _random_mesh_obj(path, n=600, seed=4):
    """n random triangles inside the leaves' overhanging box (-0.05 .. 1.07), some tiny, some large."""
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        for t in range(n):
            c = rng.uniform(-0.05, 1.07, 3)
            for k in range(3):
                v = np.clip(c + rng.normal(0, 0.02 if t % 3 else 0.3, 3), -0.05, 1.07)
                f.write("v %.7f %.7f %.7f\n" % tuple(v))
        for t in range(n):
            f.write("f %d %d %d\n" % (3 * t + 1, 3 * t + 2, 3 * t + 3))


def _deep_mesh_triangles(n=3000, ratio=1.012, size=0.3):
    """n triangles in the y-z plane at geometrically spaced x in (0, 1] (x_i = ratio^(i - n + 1)):
    binned SAH peels a few per level, so the BLAS builds to the depth limit (40)."""
    x = ratio ** np.arange(n, dtype=np.float64)
    x /= x[-1]
    s = size * x
    return np.stack([np.stack([x, 0.5 - s, 0.5 - s], 1), np.stack([x, 0.5 + s, 0.5 - s], 1),
                     np.stack([x, 0.5 + 0 * s, 0.5 + s], 1)], 1).astype(np.float32)


def _deep_mesh_obj(path):
    t = _deep_mesh_triangles()
    with open(path, "w") as f:
        for tri in t:
            for v in tri:
                f.write("v %.9g %.9g %.9g\n" % tuple(v))
        for k in range(len(t)):
            f.write("f %d %d %d\n" % (3 * k + 1, 3 * k + 2, 3 * k + 3))


def _base_obj(path):
    """A flat quad (2 triangles) with `v//n` corners."""
    with open(path, "w") as f:
        f.write("v 0 0 0\nv 1 0 0\nv 1 0 1\nv 0 0 1\nvn 0 1 0\nf 1//1 3//1 2//1\nf 1//1 4//1 3//1\n")


@pytest.fixture
def model_root(tmp_path):
    os.makedirs(tmp_path / "models")
    _prism_obj(str(tmp_path / "models" / "lanternLight.obj"))
    _base_obj(str(tmp_path / "models" / "lanternBase.obj"))
    _random_mesh_obj(str(tmp_path / "models" / "leavesCube4.obj"))
    return tmp_path


@pytest.fixture
def deep_model_root(tmp_path):
    """The leaves' mesh replaced by _deep_mesh_triangles: a BLAS at the builder's depth limit."""
    os.makedirs(tmp_path / "models")
    _prism_obj(str(tmp_path / "models" / "lanternLight.obj"))
    _base_obj(str(tmp_path / "models" / "lanternBase.obj"))
    _deep_mesh_obj(str(tmp_path / "models" / "leavesCube4.obj"))
    return tmp_path


# ---------------------------------------------------------------- CPU
def test_f16_rounding_matches_ieee():
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.standard_normal(20000).astype(np.float32) * np.float32(300),
                        rng.random(20000).astype(np.float32) * np.float32(1e-4),
                        np.array([65504, 65519, 65520, 2.0 ** -25, 2.0 ** -24, 3 * 2.0 ** -26, -0.0, np.inf], np.float32)])
    L = oracle.lib()
    got = np.array([L.orc_f32_to_f16(float(v)) for v in x], np.uint32)
    with np.errstate(over="ignore"):
        want = x.astype(np.float16).view(np.uint16).astype(np.uint32)
    assert np.array_equal(got, want)
    back = np.array([L.orc_f16_to_f32(int(h)) for h in want], np.float32)
    assert np.array_equal(back.view(np.uint32), want.astype(np.uint16).view(np.float16).astype(np.float32).view(np.uint32))


def test_octahedral_known_answers_and_round_trip():
    L = oracle.lib()
    enc = lambda n: L.orc_oct_encode(oracle._p(np.array(n, np.float32)))  # noqa: E731
    assert enc([0, 0, 1]) == 32767 | (32767 << 16)
    assert enc([1, 0, 0]) == 65534 | (32767 << 16)
    assert enc([0, -1, 0]) == 32767
    rng = np.random.default_rng(9)
    out = np.zeros(3, np.float32)
    for _ in range(2000):
        n = rng.standard_normal(3).astype(np.float32)
        n /= np.float32(np.linalg.norm(n))
        L.orc_oct_decode(enc(n), oracle._p(out))
        assert np.abs(out - n).max() < 2e-4  # 16-bit octahedral quantisation


def test_obj_reader_matches_oracle(tmp_path):
    p = str(tmp_path / "m.obj")
    with open(p, "w") as f:
        f.write("v 0.1 0.2 0.3\nv 1.0000001 -2.5e-3 7\nv 0.333333343 0.5 0.25\nv 9 9 9\nvt 0.25 0.75\nvt 1 0\n"
                "f 1/1 2/2 3/1\nf 1//3 2//1 3//2\nf 1 2 3 4\nf 2/2/1 3/1/1 4/5/1\nf -1/1 0/0 7/2\n")
    a, b = vxpt.read_obj(p), oracle.parse_obj(p)
    assert a[0].shape == (5, 3, 3)
    for x, y in zip(a, b):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))
    _prism_obj(str(tmp_path / "prism.obj"))
    a, b = vxpt.read_obj(str(tmp_path / "prism.obj")), oracle.parse_obj(str(tmp_path / "prism.obj"))
    assert a[0].shape == (8, 3, 3) and np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    with open(p, "w") as f:
        f.write("v 0 0 0\nf x/1 1 1\n")
    with pytest.raises(IOError):
        vxpt.read_obj(p)


def test_instance_collection_known_answer():
    ids = np.zeros(int(np.prod(CH)) * 32768, np.uint8)
    ids[_idx(3, 4, 5)] = LIGHT   # a lantern: its light and its base
    ids[_idx(40, 2, 7)] = BASE   # a bare base: its base and (quirk) a light instance
    ids[_idx(10, 9, 60)] = 14    # leaves
    rows = oracle.collect_instances(ids, CH, BLOCKS)
    W = 64
    iid = lambda obj, x, y, z: 13 + obj * W ** 3 + x + W * (z + W * y)  # noqa: E731
    want = sorted([(13, iid(13, 10, 9, 60), 10, 9, 60),
                   (14, iid(14, 3, 4, 5), 3, 4, 5), (14, iid(14, 40, 2, 7), 40, 2, 7),
                   (15, iid(15, 3, 4, 5), 3, 4, 5), (15, iid(15, 40, 2, 7), 40, 2, 7)])
    assert [tuple(r) for r in rows] == want


def test_alias_table_reproduces_the_distribution():
    w = np.random.default_rng(3).random(37).astype(np.float32) * np.float32(5)
    q, p, alias, s = oracle.alias_table(w)
    n = len(w)
    got = q.astype(np.float64) / n
    for j in range(n):
        if alias[j] >= 0:
            got[alias[j]] += (1.0 - q[j]) / n
    assert np.allclose(got, w / w.sum(), atol=1e-6)


# ---------------------------------------------------------------- GPU
def _expected(r, root):
    """The oracle's instance rows, light records, weights and alias bins for r's world."""
    ids = r.read("VOXELS")
    rows = oracle.collect_instances(ids, CH, BLOCKS)
    tri, _ = oracle.parse_obj(str(root / "models" / "lanternLight.obj"))
    cells = rows[rows[:, 0] == LIGHT - 1][:, 2:5]
    recs, w = oracle.tri_lights(tri, cells, [3.737, 2.718, 1.189])
    return rows, recs, w


@pytest.mark.gpu
def test_light_table_matches_oracle(model_root):
    r = vxpt.Renderer(64, 64)
    r.load_settings()
    r.generate_terrain(CH, height_scale=32.0)
    assert r.load_models(str(model_root)) == 3  # the prism, the base, the leaves; the rest are missing
    assert np.array_equal(r.model(LIGHT)[0], oracle.parse_obj(str(model_root / "models" / "lanternLight.obj"))[0])
    mp, recs, bins, lum = r.lights()
    assert len(r.instances()) == 0 and len(recs) == 0 and lum == 0.0
    cells = [(3, 20, 5), (40, 18, 7), (63, 31, 63), (0, 25, 0), (17, 22, 41)]
    for c in cells:
        r.set_block(*c, LIGHT)
    r.set_block(30, 21, 30, BASE)
    rows, want, w = _expected(r, model_root)
    assert np.array_equal(r.instances(), rows)
    mp, recs, bins, lum = r.lights()
    nl = len(cells) + 1  # the bare base carries a light instance too (collectInstanceTransforms)
    assert len(recs) == 8 * nl and len(mp) == nl
    light_rows = rows[rows[:, 0] == LIGHT - 1]
    assert np.array_equal(mp, np.stack([light_rows[:, 1], np.arange(nl) * 8, np.full(nl, 8)], 1).astype(np.uint32))
    assert np.array_equal(recs.view(np.uint32).reshape(-1, 8), want)
    q, p, alias, s = oracle.alias_table(w)
    assert np.array_equal(bins["q"].view(np.uint32), q.view(np.uint32))
    assert np.array_equal(bins["p"].view(np.uint32), p.view(np.uint32))
    assert np.array_equal(bins["alias"], alias)
    assert np.float32(lum).view(np.uint32) == s.view(np.uint32)
    # removing every lantern empties the table; a later world upload rebuilds it
    for c in cells:
        r.set_block(*c, 0)
    r.set_block(30, 21, 30, 0)
    assert len(r.instances()) == 0 and len(r.lights()[1]) == 0
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cull", [0, 1])
def test_mesh_probe_matches_brute_force(model_root, cull):
    """The two-level BVH walk (meshes.hip) equals the oracle's brute-force loop over every
    instance and triangle bit for bit: t, barycentrics, instance row and triangle.  The any-hit
    walk of visibility rays (vxpt_mesh_occluded) reports exactly the rays the brute-force loop
    finds any triangle for, both faces (closesthit.cu:616-625 traces them without culling)."""
    _probe_vs_brute_force(model_root, cull, 0.2)


def _probe_vs_brute_force(model_root, cull, min_hit):
    r = vxpt.Renderer(64, 64)
    r.load_settings()
    r.generate_terrain(CH, height_scale=32.0)
    r.load_models(str(model_root))
    rng = np.random.default_rng(11 + cull)
    cells = set()
    while len(cells) < 90:
        cells.add((int(rng.integers(0, 64)), int(rng.integers(0, 32)), int(rng.integers(0, 64))))
    for k, c in enumerate(sorted(cells)):
        r.set_block(*c, (14, 14, 14, 14, 16, 15)[k % 6])
    rows = r.instances()
    models = {b: oracle.parse_obj(str(model_root / "models" / f))[0]
              for b, f in ((14, "leavesCube4.obj"), (15, "lanternBase.obj"), (16, "lanternLight.obj"))}
    n = 6000
    o = rng.uniform([0, 0, 0], [64, 32, 64], (n, 3))
    d = rng.normal(size=(n, 3))
    aim = rows[rng.integers(0, len(rows), n // 2), 2:5] + rng.uniform(-0.05, 1.07, (n // 2, 3))
    d[: n // 2] = aim - o[: n // 2]  # half the rays aim into an instance's cell
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[::97, 1] = 0.0  # axis-parallel components
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3], rays[:, 4:7] = o, d
    rays[:, 3] = np.where(np.arange(n) % 5 == 0, 0.5, 0.0)
    rays[:, 7] = np.where(np.arange(n) % 7 == 0, 20.0, 1e27)
    got, gid = r.mesh_probe(rays, cull)
    want, wid = oracle.mesh_probe(models, rows, rays, cull)
    assert min_hit < want[:, 3].mean() < 0.95
    np.testing.assert_array_equal(gid, wid)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    if not cull:
        occ = r.mesh_occluded(rays)
        assert occ.dtype == np.uint8 and 0 < occ.sum() < len(occ)
        np.testing.assert_array_equal(occ, want[:, 3].astype(np.uint8))
    r.close()


def test_light_id_remap_known_answers():
    """The oracle's restatement of buildLightIdMapping / buildIncrementalLightMapping
    (VoxelEngine.cu:503-633) on a hand-derived edit sequence: the full build maps nothing, the
    first incremental update neither (m_instanceToLightRange still empty), later ones keep a
    light's position within its instance's run, removed / changed instances map to -1, and a
    full reload resets the update type without refreshing the instance ranges."""
    o = oracle.Oracle(8, 8)
    A, B, C = 101, 202, 303
    o._light_update({A: (0, 4), B: (4, 4)}, 8, True)
    assert o._lights_prev == 0
    o.light_edit(C, removed=False)
    o._light_update({A: (0, 4), B: (4, 4), C: (8, 4)}, 12, False)
    assert o._lights_prev == 8 and (o._remap_keep[:8] == -1).all()
    o.light_edit(A, removed=True)
    o._light_update({B: (0, 4), C: (4, 4)}, 8, False)
    assert o._remap_keep.tolist() == [-1] * 4 + [0, 1, 2, 3] + [4, 5, 6, 7]
    o._light_update({B: (0, 4), C: (4, 4)}, 8, True)  # reload
    assert (o._remap_keep == -1).all() and not o._lights["incremental"]
    o.light_edit(B, removed=True)
    o._light_update({C: (0, 4)}, 4, False)
    assert o._remap_keep.tolist() == [-1] * 4 + [0, 1, 2, 3]
    # a changed instance (re-placed lantern) loses its lights too
    o.light_edit(C, removed=False)
    o._light_update({C: (0, 4)}, 4, False)
    assert o._remap_keep.tolist() == [-1] * 4


def test_bvh_builder_keeps_the_depth_limit():
    """The mesh BVH builder (vxpt_bvh_depth, no GPU) on degenerate inputs: SAH splits only while a
    child of n - 1 primitives could still reach its leaves by median splits, so the deepest leaf
    stays <= 40 (the walk's 84-entry stack holds a TLAS and a BLAS path) -- geometrically spaced
    boxes reach exactly the limit; identical, huge-range and non-finite boxes build too."""
    t = _deep_mesh_triangles()
    boxes = np.concatenate([t.min(1), t.max(1)], 1)
    for leaf in (1, 2, 4):
        d, nodes = vxpt.bvh_depth(boxes, leaf)
        assert d <= 40 and nodes >= 2 * (len(boxes) // leaf) - 1
    assert vxpt.bvh_depth(boxes, 4)[0] == 40  # the budget rule is what bounds it
    same = np.tile(np.array([[0.4, 0.4, 0.4, 0.6, 0.6, 0.6]], np.float32), (5000, 1))
    assert vxpt.bvh_depth(same, 4)[0] == 11  # identical centroids: balanced median splits
    x = (2.0 ** np.arange(120)).astype(np.float32)
    huge = np.stack([x - 0.01, 0 * x, 0 * x, x + 0.01, 0 * x + 1, 0 * x + 1], 1)
    assert vxpt.bvh_depth(huge, 2)[0] <= 40
    bad = huge.copy()
    bad[::7, 0] = np.inf
    bad[3::7, 3] = np.nan
    assert vxpt.bvh_depth(bad, 2) is not None
    rng = np.random.default_rng(1)
    c = rng.random((20000, 3)).astype(np.float32)
    assert vxpt.bvh_depth(np.concatenate([c - 0.01, c + 0.01], 1), 4)[0] <= 20


@pytest.mark.gpu
@pytest.mark.parametrize("cull", [0, 1])
def test_deep_bvh_walk_matches_brute_force(deep_model_root, cull):
    """A BLAS at the depth limit (40) under a TLAS of 90 instances: the walk's shared stack holds
    both levels and the closest / any hits still equal the brute-force loop bit for bit."""
    _probe_vs_brute_force(deep_model_root, cull, 0.05)


def test_library_light_remap_matches_oracle_on_random_edits(tmp_path):
    """The library's light-id remap (csrc/light_map.hpp, compiled here into a CPU driver) equals the
    oracle's restatement of buildLightIdMapping / buildIncrementalLightMapping over random sequences
    of lantern placements / removals and occasional full reloads (incl. emptying the light table)."""
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "light_map_driver")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", os.path.join(repo, "real-time-path-tracing-voxel-blocks_amd", "csrc"),
                           os.path.join(repo, "tests", "native", "light_map_driver.cpp"), "-o", exe])
    rng = np.random.default_rng(7)
    for trial in range(6):
        o = oracle.Oracle(8, 8)
        live = {}  # instance id -> light count
        script, expect = [], []

        def update(full):
            m = sorted(live.items())
            ranges, first = {}, 0
            for iid, cnt in m:
                ranges[iid] = (first, cnt)
                first += cnt
            prev = o._lights["num"]
            o._light_update(ranges, first, full)
            expect.append(o._remap_keep[:prev].tolist())
            trip = " ".join("%d %d %d" % (iid, f, c) for iid, (f, c) in sorted(ranges.items()))
            script.append("update %d %d %d %d %s" % (int(full), prev, first, len(m), trip))

        update(True)
        for step in range(40):
            r = rng.random()
            if r < 0.08:
                update(True)  # reload
                continue
            for _ in range(int(rng.integers(1, 4))):
                if live and rng.random() < 0.5:
                    iid = int(rng.choice(sorted(live)))
                    del live[iid]
                    o.light_edit(iid, removed=True)
                    script.append("edit %d 1" % iid)
                else:
                    iid = int(rng.integers(13, 13 + 300))
                    live[iid] = 8 if trial % 2 == 0 else int(rng.integers(1, 9))
                    o.light_edit(iid, removed=False)
                    script.append("edit %d 0" % iid)
            if rng.random() < 0.1:
                for iid in list(live):
                    del live[iid]
                    o.light_edit(iid, removed=True)
                    script.append("edit %d 1" % iid)
            update(False)
        out = subprocess.run([exe], input="\n".join(script) + "\n", capture_output=True, text=True, check=True).stdout
        got = [[int(v) for v in ln.split()[1:]] for ln in out.splitlines()]
        assert got == expect, trial
        assert any(any(v >= 0 for v in e) for e in expect)  # some lights were carried over


@pytest.fixture(scope="module")
def mesh_walk_driver(tmp_path_factory):
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path_factory.mktemp("mw") / "mesh_walk_driver")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                           "-I", os.path.join(repo, "real-time-path-tracing-voxel-blocks_amd", "csrc"), "-x", "hip",
                           os.path.join(repo, "tests", "native", "mesh_walk_driver.hip"), "-o", exe])
    return exe


@pytest.mark.parametrize("meshes", ["synthetic", "deep", "reference"])
def test_library_mesh_walk_on_host_equals_brute_force(mesh_walk_driver, tmp_path, meshes):
    """The library's two-level BVH (bvh_build.hpp) and its walk (vx_mesh.hpp: (node, entry distance)
    stack entries, one stack for both levels), run on the host by a driver, equal the oracle's
    brute-force loop over every instance and triangle bit for bit: closest hits with and without
    back-face culling (t, barycentrics, instance row, triangle) and the any-hit answer -- with the
    synthetic meshes, with a BLAS at the builder's depth limit, and with the reference's own meshes
    (tests/golden/models: lanternLight 8, lanternBase 100, leavesCube4 1,960 triangles overhanging
    the cell)."""
    deep = meshes == "deep"
    import subprocess
    o = oracle.Oracle(8, 8)
    o.terrain(CH, 32.0)
    ids = o.voxels()
    rng = np.random.default_rng(17 + deep)
    cells = set()
    while len(cells) < 90:
        cells.add((int(rng.integers(0, 64)), int(rng.integers(0, 32)), int(rng.integers(0, 64))))
    for k, c in enumerate(sorted(cells)):
        ids[_idx(*c)] = (14, 14, 14, 14, 16, 15)[k % 6]
    rows = oracle.collect_instances(ids, CH, BLOCKS)
    leaves = _deep_mesh_triangles() if deep else None
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "models")
    if meshes == "reference":
        for src, dst in (("leavesCube4.obj", "leaves.obj"), ("lanternLight.obj", "light.obj"),
                         ("lanternBase.obj", "base.obj")):
            shutil.copy(os.path.join(golden, src), tmp_path / dst)
        leaves = oracle.parse_obj(str(tmp_path / "leaves.obj"))[0]
    elif not deep:
        _random_mesh_obj(str(tmp_path / "leaves.obj"))
        leaves = oracle.parse_obj(str(tmp_path / "leaves.obj"))[0]
    if meshes != "reference":
        _prism_obj(str(tmp_path / "light.obj"))
        _base_obj(str(tmp_path / "base.obj"))
    models = {14: np.asarray(leaves, np.float32).reshape(-1, 3, 3),
              15: oracle.parse_obj(str(tmp_path / "base.obj"))[0], 16: oracle.parse_obj(str(tmp_path / "light.obj"))[0]}
    with open(tmp_path / "meshes.bin", "wb") as f:
        for b in range(32):
            t = np.asarray(models.get(b, np.zeros((0, 3, 3))), np.float32).reshape(-1, 9)
            f.write(np.int32(len(t)).tobytes())
            f.write(t.tobytes())
        f.write(np.int32(len(rows)).tobytes())
        f.write(np.ascontiguousarray(rows, np.int32).tobytes())
    n = 6000
    org = rng.uniform([0, 0, 0], [64, 32, 64], (n, 3))
    d = rng.normal(size=(n, 3))
    aim = rows[rng.integers(0, len(rows), n // 2), 2:5] + rng.uniform(-0.05, 1.07, (n // 2, 3))
    d[: n // 2] = aim - org[: n // 2]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[::97, 1] = 0.0
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3], rays[:, 4:7] = org, d
    rays[:, 3] = np.where(np.arange(n) % 5 == 0, 0.5, 0.0)
    rays[:, 7] = np.where(np.arange(n) % 7 == 0, 20.0, 1e27)
    rays.tofile(tmp_path / "rays.bin")
    res = subprocess.run([mesh_walk_driver, str(tmp_path / "meshes.bin"), str(tmp_path / "rays.bin"),
                          str(tmp_path / "out.bin")], capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr
    if deep:
        assert "deepest blas 40" in res.stderr, res.stderr
    got = np.fromfile(tmp_path / "out.bin", np.int32).reshape(-1, 13)
    for cull in (0, 1):
        want, wid = oracle.mesh_probe(models, rows, rays, cull)
        g = got[:, 6 * cull:6 * cull + 6]
        assert 0.03 < want[:, 3].mean() < 0.95
        np.testing.assert_array_equal(g[:, 4:6], wid, err_msg="cull %d ids" % cull)
        np.testing.assert_array_equal(g[:, 0:3], want[:, 0:3].view(np.int32), err_msg="cull %d t/u/v" % cull)
        np.testing.assert_array_equal(g[:, 3], want[:, 3].astype(np.int32))
        if cull == 0:
            np.testing.assert_array_equal(got[:, 12], want[:, 3].astype(np.int32), err_msg="occluded")
