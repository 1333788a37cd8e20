"""Instanced meshes in the path tracer (the rendering half), GPU vs oracle.

The C1 world with lanterns (emissive light mesh + its base, blocks 16 / 15) and leaves (thin-film
mesh, block 14) placed on the terrain in front of the C1 camera.  Two mesh sets: the reference's own
meshes (data/models/lanternLight.obj 8 faces, lanternBase.obj 100, leavesCube4.obj 1,960 with
bounds -0.05..1.07 overhanging its cell; committed as data fixtures under tests/golden/models) and
the synthetic OBJ files of test_lights.  The materials are the repo's data/assets materials.yaml
entries, read here independently of the library (MaterialManager.cpp:150-190: materialId = the
material's index, an emissive material's albedo is its radiance).

Covered against oracle/orc_mesh.cpp + orc_trace.cpp over 4 frames of trace + denoise:
  closest hit = min(voxel DDA, mesh BVH walk) with back faces culled, ties to the voxel face;
  mesh-hit shading with the general self-intersection-safe spawn (SelfHit.h:539-656);
  emissive hits before the first diffuse bounce (closesthit.cu:107-122);
  thin-film normal flip and front / back spawn choice (closesthit.cu:124-133, 288, 457, 614);
  8 local-light NEE candidates from the light alias table (closesthit.cu:350-378);
  BRDF-candidate rays that hit an emissive triangle (closesthit.cu:518-551, 854-900);
  visibility rays against voxels and meshes, local lights traced to 0.01 short;
  ReSTIR temporal reuse of local-light reservoirs (Restir.h:383-415);
  the light-id remap across lantern edits (VoxelEngine.cu:503-633, 1192-1284; Restir.h:48-79).
"""
import os
import shutil

import numpy as np
import pytest
import yaml

import oracle
import vxpt
from golden.make_golden import C1_CAMERA
from test_gpu_parity import (DN_FLOATS, DN_INTS, RTOL_DN, _dn_params, _inject_frame, _inject_sky, _rel,
                              check_radiance)
from test_lights import _base_obj, _prism_obj, _random_mesh_obj

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CH = (2, 1, 2)
LIGHT, BASE, LEAVES = 16, 15, 14


def _idx(x, y, z):
    return ((x >> 5) + CH[0] * ((z >> 5) + CH[2] * (y >> 5))) * 32768 + (x & 31) + 32 * ((z & 31) + 32 * (y & 31))


def asset_tables():
    """blocks.yaml + materials.yaml of the repo data: block defs for the instance / light collection and
    the MaterialParameter of each instanced block."""
    with open(os.path.join(REPO, "data", "assets", "blocks.yaml")) as f:
        blocks = {b["id"]: b for b in yaml.safe_load(f)["blocks"]}
    with open(os.path.join(REPO, "data", "assets", "materials.yaml")) as f:
        mats = yaml.safe_load(f)["materials"]
    index = {m["id"]: i for i, m in enumerate(mats)}
    props = {m["id"]: m.get("properties", {}) for m in mats}
    defs, params = {}, {}
    for b, d in blocks.items():
        if not d.get("instanced"):
            continue
        p = props.get(d.get("material"), {})
        emissive = bool(d.get("emissive")) or bool(p.get("is_emissive"))
        rad = tuple(p.get("emissive_radiance", (0.0, 0.0, 0.0))) if p.get("is_emissive") else (0.0, 0.0, 0.0)
        defs[b] = dict(instanced=True, light_base=d.get("light_base", 0), emissive=emissive, radiance=rad)
        params[b] = dict(albedo=rad if p.get("is_emissive") else tuple(p.get("albedo", (1.0, 1.0, 1.0))),
                         roughness=p.get("roughness", 0.5), metallic=int(p.get("metallic", 0.0) != 0),
                         translucency=p.get("translucency", 0.0), material_id=index.get(d.get("material"), 0),
                         emissive=bool(p.get("is_emissive")), thin=bool(p.get("is_thinfilm")),
                         world_grid=bool(p.get("use_world_grid_uv")), uv_scale=p.get("uv_scale", 1.0))
    return defs, params


def place_meshes(ids):
    """Lanterns and leaves on top of the terrain along the C1 camera's view direction."""
    pos, d = np.array(C1_CAMERA[0]), np.array(C1_CAMERA[1], np.float64)
    d /= np.linalg.norm(d)
    placed = []
    for k, dist in enumerate([6, 8, 10, 12, 14, 16, 18, 21]):
        p = pos + d * dist
        x, z = int(p[0]) + (k % 3) - 1, int(p[2])
        col = [y for y in range(32) if 1 <= ids[_idx(x, y, z)] <= 12]
        if not col or max(col) + 1 >= 32:
            continue
        y = max(col) + 1
        ids[_idx(x, y, z)] = LEAVES if k % 2 else LIGHT
        placed.append((x, y, z, int(ids[_idx(x, y, z)])))
    return placed


GOLDEN_MODELS = os.path.join(REPO, "tests", "golden", "models")


@pytest.fixture(params=["reference", "synthetic"])
def mesh_scene(tmp_path, request):
    os.makedirs(tmp_path / "models")
    if request.param == "reference":  # ModelManager.cpp:172-226 loads these from data/models
        for f in ("lanternLight.obj", "lanternBase.obj", "leavesCube4.obj"):
            shutil.copy(os.path.join(GOLDEN_MODELS, f), tmp_path / "models" / f)
    else:
        _prism_obj(str(tmp_path / "models" / "lanternLight.obj"))
        _base_obj(str(tmp_path / "models" / "lanternBase.obj"))
        _random_mesh_obj(str(tmp_path / "models" / "leavesCube4.obj"), n=120)
    w, h = 128, 96
    r = vxpt.Renderer(w, h)
    r.load_settings()
    o = oracle.Oracle(w, h)
    o.terrain(CH)
    ids = o.voxels()
    placed = place_meshes(ids)
    assert sum(1 for p in placed if p[3] == LIGHT) >= 2 and sum(1 for p in placed if p[3] == LEAVES) >= 2, placed
    o.set_voxels(ids, CH)
    r.upload_voxels(ids, CH)
    assert r.load_models(tmp_path) >= 3
    cam = (C1_CAMERA[0], C1_CAMERA[1], C1_CAMERA[2])
    r.set_camera(*cam[:2], fov=cam[2], prev=cam)
    r.set_sky(0.25, 45.0, 0.0, 1.0)
    o.set_camera(*cam[:2], fov=cam[2])
    o.set_camera(*cam[:2], fov=cam[2], which=1)
    o.set_denoise_params(DN_FLOATS, DN_INTS)
    defs, params = asset_tables()
    for b, p in params.items():
        o.set_material(b, **p)
    models = {b: oracle.parse_obj(str(tmp_path / "models" / f)) for b, f in
              ((LIGHT, "lanternLight.obj"), (BASE, "lanternBase.obj"), (LEAVES, "leavesCube4.obj"))}
    rows = o.set_meshes(models, defs)
    _inject_sky(r, o)
    yield r, o, rows, placed, dict(models=models, defs=defs)
    r.close()


def test_mesh_scene_matches_oracle(mesh_scene):
    r, o, rows, placed, _ = mesh_scene
    inst = r.instances()
    # the library's instance rows are the oracle's (object, id, x, y, z); rows here are (block, x, y, z, light)
    np.testing.assert_array_equal(inst[:, 0] + 1, rows[:, 0])
    np.testing.assert_array_equal(inst[:, 2:5], rows[:, 1:4])
    mapping, recs, _, _ = r.lights()
    assert len(recs) == int((rows[:, 4] >= 0).sum()) * 8 and len(recs) > 0
    p = _dn_params()
    for f in range(4):
        r.trace(f)
        r.denoise(f, f + 1, p)
        o.trace(f)
        o.post_trace()
        o.denoise(f, f + 1)
        for name in ("DEPTH", "MATERIAL", "NORMAL_ROUGH", "GEO_NORMAL_THIN", "ALBEDO", "MAT_PARAM"):
            np.testing.assert_allclose(r.read(name), o.read(vxpt.BUF[name]), rtol=1e-6, atol=1e-7,
                                       err_msg="frame %d %s" % (f, name))
        check_radiance(r.read("ILLUM"), o.read(0), "meshes frame%d illum" % f)
        check_radiance(r.read("OUTPUT"), o.read(21), "meshes frame%d output" % f)
        res_g, res_o = r.read("RESERVOIRS"), o.read(vxpt.BUF["RESERVOIRS"])
        np.testing.assert_array_equal(res_g["lightData"], res_o["lightData"], err_msg="frame %d lightData" % f)
    depth, mat, geo = r.read("DEPTH"), r.read("MATERIAL"), r.read("GEO_NORMAL_THIN")
    # the primary rays see emissive lantern lights (material 0xFFFF at a finite depth) and the thin leaves
    assert ((mat == 0xFFFF) & (depth < 1e26)).sum() > 0
    assert (geo[..., 3] == 1.0).sum() > 0
    # local lights were selected by the reservoirs (light index < number of lights)
    res = r.read("RESERVOIRS")
    li = res["lightData"] & 0x7FFFFFFF
    assert ((res["lightData"] != 0) & (li < len(recs))).sum() > 0


def _frame(r, o, f, p, tag, output):
    """Trace parity every frame.  With `output`, the denoiser then runs on both sides from the same
    inputs (the oracle's planes injected, test_gpu_parity._inject_frame) and its outputs are
    compared: chained from each side's own history the reference's clamp is chaotic from the fifth
    frame of history on (tests/test_denoise_host.py), so a chained comparison measures rounding,
    not parity."""
    r.trace(f)
    o.trace(f)
    o.set_prev_scene_empty(False)
    o.post_trace()
    res_g, res_o = r.read("RESERVOIRS"), o.read(vxpt.BUF["RESERVOIRS"])
    np.testing.assert_array_equal(res_g["lightData"], res_o["lightData"], err_msg=tag + " lightData")
    np.testing.assert_array_equal(res_g["M"], res_o["M"], err_msg=tag + " M")
    check_radiance(r.read("ILLUM"), o.read(0), tag + " illum")
    if output:
        _inject_frame(r, o)
    r.denoise(f, f + 1, p)
    o.denoise(f, f + 1)
    if output:
        for name in ("OUTPUT", "PREV_ILLUM", "PREV_FAST"):
            rel = _rel(r.read(name), o.read(vxpt.BUF[name]))
            assert rel.max() < RTOL_DN, (tag, name, rel.max(), np.unravel_index(rel.argmax(), rel.shape))
        np.testing.assert_allclose(r.read("HIST_LEN"), o.read(19), rtol=1e-6, err_msg=tag + " histLen")
    return res_g


def _lantern_edits(mesh_scene, output):
    """Remove the last lantern, then the first one (the rest shift down), then re-add the last, two
    frames after each edit; trace parity every frame, the denoised output too when `output`."""
    r, o, rows, placed, ex = mesh_scene
    models, defs = ex["models"], ex["defs"]
    first, width = min(defs), CH[0] * 32
    lanterns = sorted((p for p in placed if p[3] == LIGHT),
                      key=lambda p: oracle.instance_id(first, width, LIGHT - 1, *p[:3]))
    assert len(lanterns) >= 2
    p = _dn_params()
    f = 0
    for _ in range(2):
        _frame(r, o, f, p, "pre frame%d" % f, output)
        f += 1
    edits = [(lanterns[-1], 0), (lanterns[0], 0), (lanterns[-1], LIGHT)]
    mapped = 0
    for k, ((x, y, z, _), block) in enumerate(edits):
        r.set_block(x, y, z, block)
        ids = r.read("VOXELS")
        o.set_voxels(ids, CH)
        o.set_prev_scene_empty(True)
        o.light_edit(oracle.instance_id(first, width, LIGHT - 1, x, y, z), removed=block == 0)
        o.set_meshes(models, defs, light_update="update")
        remap, pending = r.light_remap()
        exp = o._remap_keep[:len(remap)]
        assert pending and len(remap) == o._lights_prev, (k, len(remap))
        np.testing.assert_array_equal(remap, exp, err_msg="edit %d remap" % k)
        if k == 0:
            assert (remap == -1).all()  # the first incremental update after the full build
        else:
            assert (remap == -1).any() or block != 0
        mapped += int((remap >= 0).sum())
        for _ in range(2):
            res = _frame(r, o, f, p, "edit%d frame%d" % (k, f), output)
            f += 1
        assert not r.light_remap()[1]
    assert mapped > 0
    # local-light reservoirs survive the remaps
    li = res["lightData"] & 0x7FFFFFFF
    assert ((res["lightData"] != 0) & (li < len(r.lights()[1]))).sum() > 0


def test_lantern_edits_remap_reservoirs(mesh_scene):
    """Remove / re-add lanterns between frames: each edit is an incremental light update whose
    previous -> current light table (the first one after the scene's full build maps nothing,
    m_instanceToLightRange being empty until then) is applied to the previous reservoirs in the
    one pass after it.  The library's table equals the oracle's restatement, and the traced
    frames -- reservoirs bit for bit, radiance per pixel -- equal the oracle's."""
    _lantern_edits(mesh_scene, output=False)


def test_denoised_frames_across_lantern_edits(mesh_scene):
    """The same edits with the denoiser compared every frame on identical inputs: the frames after
    each edit (histories reset where a lantern vanished or reappeared, the light-id remap applied)
    denoise as the oracle does."""
    _lantern_edits(mesh_scene, output=True)


def test_base_only_edits_follow_the_grid(mesh_scene):
    """A lantern base placed and removed on its own (defined deviation): the library's
    instance set is always collectInstanceTransforms of the edited grid (VoxelEngine.cu:323-384), so a
    bare base cell carries its light's instance as at load, and its edit is that light's incremental
    light update (the reference's incremental addInstancedBlock of a bare base registers no light,
    VoxelEngine.cu:1278-1284, and deleting one leaves a stale light instance).  The oracle restates
    the same rule (collect_instances + light_edit of the light instance): the instance rows, the
    light remap of each update and the traced frames agree."""
    r, o, rows, placed, ex = mesh_scene
    models, defs = ex["models"], ex["defs"]
    first, width = min(defs), CH[0] * 32
    leaves = [p for p in placed if p[3] == LEAVES]
    x, y, z = leaves[0][0], leaves[0][1] + 1, leaves[0][2]
    assert r.read("VOXELS")[_idx(x, y, z)] == 0
    p = _dn_params()
    f = 0
    for _ in range(2):
        _frame(r, o, f, p, "pre frame%d" % f, False)
        f += 1
    light_iid = oracle.instance_id(first, width, LIGHT - 1, x, y, z)
    for k, block in enumerate((BASE, 0)):
        r.set_block(x, y, z, block)
        o.set_voxels(r.read("VOXELS"), CH)
        o.set_prev_scene_empty(True)
        o.light_edit(light_iid, removed=block == 0)
        got_rows = o.set_meshes(models, defs, light_update="update")
        inst = r.instances()
        np.testing.assert_array_equal(inst[:, 0] + 1, got_rows[:, 0])
        np.testing.assert_array_equal(inst[:, 2:5], got_rows[:, 1:4])
        # the bare base carries a light instance (and its own base instance) while it stands
        at = [tuple(int(v) for v in row) for row in inst if (row[2], row[3], row[4]) == (x, y, z)]
        assert (len(at) == 2) == (block == BASE), at
        remap, pending = r.light_remap()
        assert pending and len(remap) == o._lights_prev, (k, len(remap))
        np.testing.assert_array_equal(remap, o._remap_keep[:len(remap)], err_msg="base edit %d remap" % k)
        for _ in range(2):
            _frame(r, o, f, p, "base edit%d frame%d" % (k, f), False)
            f += 1
