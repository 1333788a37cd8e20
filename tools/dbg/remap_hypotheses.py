"""Debug (CPU): which stale input would make the oracle's frame-5 history at (40, 12) equal the GPU's?"""
import os, sys, tempfile
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(R, d) for d in ("tests", "oracle", "real-time-path-tracing-voxel-blocks_amd")]
import numpy as np
import oracle
import test_gpu_meshes as T
from test_lights import _base_obj, _prism_obj, _random_mesh_obj
from golden.make_golden import C1_CAMERA

GPU = np.array([0.06207283, 0.08113439, 0.11520769])
PX = [(40, 12), (35, 17), (38, 27), (76, 30), (50, 71)]


def run(hyp):
    d = tempfile.mkdtemp(); os.makedirs(d + "/models")
    _prism_obj(d + "/models/lanternLight.obj"); _base_obj(d + "/models/lanternBase.obj")
    _random_mesh_obj(d + "/models/leavesCube4.obj", n=120)
    o = oracle.Oracle(128, 96)
    o.terrain(T.CH)
    ids = o.voxels()
    placed = T.place_meshes(ids)
    o.set_voxels(ids, T.CH)
    cam = (C1_CAMERA[0], C1_CAMERA[1], C1_CAMERA[2])
    o.set_camera(*cam[:2], fov=cam[2]); o.set_camera(*cam[:2], fov=cam[2], which=1)
    o.set_sky(0.25, 45.0, 0.0, 1.0)
    o.set_denoise_params(T.DN_FLOATS, T.DN_INTS)
    defs, params = T.asset_tables()
    for b, p in params.items():
        o.set_material(b, **p)
    models = {b: oracle.parse_obj(d + "/models/" + f) for b, f in
              ((T.LIGHT, "lanternLight.obj"), (T.BASE, "lanternBase.obj"), (T.LEAVES, "leavesCube4.obj"))}
    o.set_meshes(models, defs)
    first, width = min(defs), T.CH[0] * 32
    lanterns = sorted((p for p in placed if p[3] == T.LIGHT),
                      key=lambda p: oracle.instance_id(first, width, T.LIGHT - 1, *p[:3]))
    edits = {2: (lanterns[-1], 0), 4: (lanterns[0], 0)}
    saved = {}
    for f in range(6):
        if f in edits:
            (x, y, z, _), b = edits[f]
            ids[T._idx(x, y, z)] = b
            o.set_voxels(ids, T.CH)
            o.set_prev_scene_empty(True)
            o.light_edit(oracle.instance_id(first, width, T.LIGHT - 1, x, y, z), removed=b == 0)
            o.set_meshes(models, defs, light_update="update")
        o.trace(f); o.set_prev_scene_empty(False); o.post_trace()
        if f == 5 and hyp in saved:
            for k, v in saved[hyp].items():
                o.write(k, v)
        o.denoise(f, f + 1)
        if f == 3:
            saved["H1_prev_gbuffer_of_frame3"] = {12: o.read(12).copy(), 8: o.read(8).copy(), 13: o.read(13).copy()}
            saved["H2_histories_of_frame3"] = {17: o.read(17).copy(), 18: o.read(18).copy(), 20: o.read(20).copy()}
    return o.read(17)


base = run("none")
for hyp in ["H1_prev_gbuffer_of_frame3", "H2_histories_of_frame3"]:
    v = run(hyp)
    diff = np.abs(v[..., :3] - base[..., :3]).max(-1) > 1e-4 * (1 + np.abs(base[..., :3]).max(-1))
    ys, xs = np.nonzero(diff)
    print(hyp, "pixels changed", int(diff.sum()), "at (40,12):", v[12, 40, :3], "gpu", GPU,
          "| changed among the GPU's 5:", sum(1 for (x, y) in PX if diff[y, x]))
