"""ORACLE (test infrastructure only) -- ctypes binding of liboracle.so, the CPU
restatement of the reference's offline hot path (see oracle/*.cpp headers for
the reference file:line each function follows).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline; the product never does.

Pinning: Perlin noise KATs from the reference's PerlinNoise.hpp (SURVEY.md
§8c: octave2D_01(0,0,4)=0.890182078, (10/64,5/64)=0.961326897, 64x64 map
min/max/mean) and the reference camera KATs (renderer/test/camera/test.cpp:
145-257) are checked in tests/test_oracle.py; the voxel DDA is pinned against a
brute-force culled-triangle caster over the face mesh the reference builds.
Shading and denoising have no reference golden vectors --
their parity is against this restatement only.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
# ORACLE_LIB: another build of the same sources (bench.py's CPU baseline builds one with
# -march=native for the host it runs on)
LIB = os.environ.get("ORACLE_LIB") or os.path.join(HERE, "liboracle.so")
TABLES = os.path.join(REPO, "data", "tables")

RESERVOIR_DTYPE = np.dtype([("lightData", "<u4"), ("uvData", "<u4"), ("weightSum", "<f4"), ("targetPdf", "<f4"),
                            ("M", "<f4")])
FLOAT1 = {1, 5, 12, 13, 19, 20, 49}
# default cube materials (data/assets/materials.yaml order): (block id, roughness, material id)
TERRAIN_ROUGHNESS = [0.8, 0.9, 0.85, 0.9, 0.8, 0.7, 0.85, 0.6, 0.7, 0.65, 0.75, 0.75]

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        sig = {
            "orc_create": (P, [I, I, ctypes.c_char_p]),
            "orc_destroy": (None, [P]),
            "orc_set_bounces": (None, [P, I, I]),
            "orc_terrain": (I, [P, I, I, I, F, F, I, I]),
            "orc_set_voxels": (I, [P, P, I, I, I]),
            "orc_set_prev_scene_empty": (None, [P, I]),
            "orc_set_textures": (None, [P, P, ctypes.c_size_t, P, I]),
            "orc_set_material_textures": (None, [P, I, I, I, I, I, F, I]),
            "orc_get_voxels": (I, [P, P]),
            "orc_set_material": (None, [P, I, F, F, F, F, I, F, I]),
            "orc_set_sky": (I, [P, F, F, F, F]),
            "orc_set_sky_maps": (None, [P, P, P, P]),
            "orc_get_sky": (None, [P, P, P, P, P, P, P]),
            "orc_set_camera": (None, [P, P, P, F, I]),
            "orc_get_camera": (None, [P, I, P]),
            "orc_camera_kat": (None, [I, I, F, F, P, I, P, P]),
            "orc_postprocess": (None, [I, I, P, P, P, P, F, I, I, I, F, F, F, P]),
            "orc_copy_camera_to_prev": (None, [P]),
            "orc_trace": (None, [P, I, I, I, I]),
            "orc_post_trace": (None, [P]),
            "orc_trace_frame_spp": (None, [P, I, I]),
            "orc_set_denoise_params": (None, [P, P, P]),
            "orc_denoise": (None, [P, I, I]),
            "orc_pass": (None, [P, I, I, I]),
            "orc_set_band": (None, [P, I, I]),
            "orc_buffer": (I, [P, I, P, I]),
            "orc_rand": (F, [P, I, I, I, I]),
            "orc_perlin": (F, [F, F, I]),
            "orc_dda": (None, [P, I, P, P, P, I]),
            "orc_f32_to_f16": (ctypes.c_uint32, [F]),
            "orc_f16_to_f32": (F, [ctypes.c_uint32]),
            "orc_oct_encode": (ctypes.c_uint32, [P]),
            "orc_oct_decode": (None, [ctypes.c_uint32, P]),
            "orc_tri_lights": (None, [P, I, P, I, P, P, P]),
            "orc_mesh_probe": (None, [P, P, P, P, I, P, I, I, P, P]),
            "orc_set_material_flags": (None, [P, I, I, I, I, F]),
            "orc_set_meshes": (None, [P, P, P, P, P, I, P, I, P, I, P, P, P]),
            "orc_set_light_remap": (None, [P, P, I, I]),
        }
        for k, (r, a) in sig.items():
            fn = getattr(L, k)
            fn.restype = r
            fn.argtypes = a
        _lib = L
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def perlin(x, y, octaves=4):
    return lib().orc_perlin(x, y, octaves)


def camera_kat(w, h, yaw, pitch, uvs):
    uvs = np.ascontiguousarray(uvs, np.float32).reshape(-1, 2)
    n = uvs.shape[0]
    d, b = np.zeros((n, 3), np.float32), np.zeros((n, 2), np.float32)
    lib().orc_camera_kat(w, h, yaw, pitch, _p(uvs), n, _p(d), _p(b))
    return d, b


class Oracle:
    def __init__(self, width, height, bounces=(3, 1)):
        self.L = lib()
        self.W, self.H = width, height
        self.h = self.L.orc_create(width, height, TABLES.encode())
        if not self.h:
            raise RuntimeError("oracle tables missing under " + TABLES)
        self.L.orc_set_bounces(self.h, bounces[0], bounces[1])
        for b, r in enumerate(TERRAIN_ROUGHNESS, start=1):
            self.L.orc_set_material(self.h, b, 1.0, 1.0, 1.0, r, 0, 0.0, b - 1)
        self.chunks = None
        # Scene's light-update state (Scene.h:91-115): light count, update type, the edit sets and
        # m_instanceToLightRange (only an incremental update refreshes it)
        self._lights = dict(num=0, incremental=False, changed=set(), removed=set(), range={})
        self._lights_dirty = False

    def set_materials(self, mats):
        """Same list as vxpt.Renderer.upload_materials (block ids 1..len)."""
        for b, m in enumerate(mats, start=1):
            al = m.get("albedo", (1.0, 1.0, 1.0))
            self.L.orc_set_material(self.h, b, al[0], al[1], al[2], m.get("roughness", 0.8),
                                    int(m.get("metallic", 0)), m.get("translucency", 0.0), m.get("material_id", b - 1))

    def set_material(self, block, albedo=(1.0, 1.0, 1.0), roughness=0.5, metallic=0, translucency=0.0,
                     material_id=0, emissive=False, thin=False, world_grid=False, uv_scale=1.0):
        """One block's MaterialParameter (any block id < 32; for an emissive block `albedo` is its
        radiance, MaterialManager.cpp:162-167)."""
        self.L.orc_set_material(self.h, block, albedo[0], albedo[1], albedo[2], roughness, int(metallic),
                                translucency, material_id)
        self.L.orc_set_material_flags(self.h, block, int(emissive), int(thin), int(world_grid), float(uv_scale))

    def set_meshes(self, models, blocks, rows=None, light_update="full"):
        """The world's instanced meshes.  models: {block: (pos [T,3,3], uv [T,3,2])};
        blocks: {block: dict(instanced, light_base, emissive, radiance)}; rows: instance rows
        (object, id, x, y, z), collected from this oracle's voxels when None.  The light records
        are generated in the library's order (emissive objects by object id, each instance's
        triangles in a row) and their alias table built as AliasTable::update does.  light_update: the
        light update this is -- "full" (scene init / reload), "update" (after light_edit calls; full
        or incremental as the edits made it), None (an edit of no emissive block: the light table
        is unchanged and no remap follows); after an update the next trace pass remaps the previous
        pass's light indices."""
        if rows is None:
            rows = collect_instances(self.voxels(), self.chunks, blocks)
        rows = np.asarray(rows, np.int32).reshape(-1, 5)
        pos, uv, off, cnt = [], [], np.zeros(32, np.int32), np.zeros(32, np.int32)
        acc = 0
        for b in range(32):
            if b in models and len(models[b][0]):
                p_, u_ = models[b]
                off[b], cnt[b] = acc, len(p_)
                pos.append(np.asarray(p_, np.float32).reshape(-1, 9))
                uv.append(np.asarray(u_, np.float32).reshape(-1, 6))
                acc += len(p_)
        pos = np.ascontiguousarray(np.concatenate(pos) if pos else np.zeros((1, 9), np.float32))
        uv = np.ascontiguousarray(np.concatenate(uv) if uv else np.zeros((1, 6), np.float32))
        inst = np.zeros((len(rows), 5), np.int32)
        recs, ws, nl = [], [], 0
        k = 0
        while k < len(rows):
            obj = int(rows[k, 0])
            e = k
            while e < len(rows) and rows[e, 0] == obj:
                e += 1
            b = obj + 1
            bd = blocks.get(b, {})
            t = cnt[b]
            for i in range(k, e):
                inst[i] = (b, rows[i, 2], rows[i, 3], rows[i, 4], -1)
            if bd.get("emissive") and t > 0:
                r, w = tri_lights(models[b][0], rows[k:e, 2:5], bd.get("radiance", (0.0, 0.0, 0.0)))
                for i in range(k, e):
                    inst[i, 4] = nl + (i - k) * t
                recs.append(r)
                ws.append(w)
                nl += t * (e - k)
            k = e
        lights = np.ascontiguousarray(np.concatenate(recs) if recs else np.zeros((1, 8), np.uint32))
        if nl:
            q, pr, al, _ = alias_table(np.concatenate(ws))
        else:
            q, pr, al = np.zeros(1, np.float32), np.zeros(1, np.float32), np.zeros(1, np.int32)
        q, pr, al = (np.ascontiguousarray(q, np.float32), np.ascontiguousarray(pr, np.float32),
                     np.ascontiguousarray(al, np.int32))
        inst = np.ascontiguousarray(inst)
        self.L.orc_set_meshes(self.h, _p(pos), _p(uv), _p(off), _p(cnt), acc, _p(inst), len(inst), _p(lights), nl,
                              _p(q), _p(pr), _p(al))
        self._mesh_keep = (pos, uv, off, cnt, inst, lights, q, pr, al)
        ranges = {int(rows[i, 1]): (int(inst[i, 4]), int(cnt[inst[i, 0]])) for i in range(len(rows)) if inst[i, 4] >= 0}
        if light_update is not None:
            self._light_update(ranges, int(nl), light_update == "full")
        return inst

    def light_edit(self, instance, removed):
        """deleteInstancedBlock / addInstancedBlock of an emissive block (VoxelEngine.cu:1206-1212,
        1278-1284): the next light update is incremental, with `instance` removed or changed."""
        st = self._lights
        st["incremental"] = True
        (st["removed"] if removed else st["changed"]).add(int(instance))

    def _light_update(self, cur, total, full):
        """VoxelEngine::updateLight (VoxelEngine.cu:658-709) with buildLightIdMapping (:503-539) and
        buildIncrementalLightMapping (:541-633): the previous light index -> current index table of
        the next pass (Restir.h:48-79).  cur: {instance id: (first light, count)} of the new table."""
        st = self._lights
        if full:
            st["incremental"] = False
        prev_n = st["num"]
        remap = np.full(max(prev_n, 1), -1, np.int32)
        if prev_n > 0:
            if st["incremental"]:
                owner = [None] * prev_n
                for iid, (off, cnt) in st["range"].items():
                    for i in range(cnt):
                        if off + i < prev_n:
                            owner[off + i] = iid
                for p in range(prev_n):
                    iid = owner[p]
                    if iid is None or iid in st["removed"] or iid in st["changed"] or iid not in cur:
                        continue
                    (po, pc), (co, cc) = st["range"][iid], cur[iid]
                    rel = p - po
                    if rel < pc and rel < cc and co + rel < total:
                        remap[p] = co + rel
                st["range"] = dict(cur)
            st["changed"].clear()
            st["removed"].clear()
        st["num"] = total
        self._lights_prev = prev_n
        self._remap_keep = remap
        self.L.orc_set_light_remap(self.h, _p(remap), prev_n, 1)
        self._lights_dirty = True

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_destroy(self.h)
            self.h = None

    def terrain(self, chunks=(2, 1, 2), height_scale=32.0, freq_den=None, use_fma=True, keep_balls=False,
                global_y=False):
        if freq_den is None:
            freq_den = 32.0 * chunks[0]
        self.L.orc_terrain(self.h, chunks[0], chunks[1], chunks[2], height_scale, freq_den, int(use_fma),
                           (1 if keep_balls else 0) | (2 if global_y else 0))
        self.chunks = tuple(chunks)

    def voxels(self):
        cx, cy, cz = self.chunks
        out = np.zeros(cx * cy * cz * 32768, np.uint8)
        self.L.orc_get_voxels(self.h, _p(out))
        return out

    def set_voxels(self, ids, chunks):
        ids = np.ascontiguousarray(ids, np.uint8)
        self.L.orc_set_voxels(self.h, _p(ids), *chunks)
        self.chunks = tuple(chunks)

    def set_sky(self, tod=0.25, axis=45.0, rot=0.0, bright=1.0):
        self.L.orc_set_sky(self.h, tod, axis, rot, bright)

    def set_sky_maps(self, sky, sun, sun_dir):
        sky = np.ascontiguousarray(sky, np.float32)
        sun = np.ascontiguousarray(sun, np.float32)
        sd = np.ascontiguousarray(sun_dir, np.float32)
        self.L.orc_set_sky_maps(self.h, _p(sky), _p(sun), _p(sd))

    def sky(self):
        sky, sun, sd = np.zeros((512, 1024, 4), np.float32), np.zeros((32, 32, 4), np.float32), np.zeros(3, np.float32)
        n = 1024 * 512
        q, p, a = np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.int32)
        self.L.orc_get_sky(self.h, _p(sky), _p(sun), _p(sd), _p(q), _p(p), _p(a))
        return dict(sky=sky, sun=sun, sun_dir=sd, q=q, p=p, alias=a)

    def set_camera(self, pos, direction, fov=90.0, which=0):
        pos = np.asarray(pos, np.float32)
        d = np.asarray(direction, np.float32)
        self.L.orc_set_camera(self.h, _p(pos), _p(d), fov, which)

    def camera_info(self, which=0):
        out = np.zeros(32, np.float32)
        self.L.orc_get_camera(self.h, which, _p(out))
        return out

    def trace(self, it, y0=0, y1=None, primary_only=False):
        self.L.orc_trace(self.h, it, y0, self.H if y1 is None else y1, int(primary_only))
        # the light remap holds for the one pass after a light update (OptixRenderer.cpp:451-458)
        if self._lights_dirty and (y1 is None or y1 >= self.H):
            self._lights_dirty = False
            self.L.orc_set_light_remap(self.h, _p(self._remap_keep), 0, 0)

    def render_frame(self, frame, spp=1, denoise=True):
        """One OfflineBackend::renderFrame (OfflineBackend.cpp:46-89) at spp samples per pixel, as
        vxpt_render_frame defines it: spp 1-spp passes at iterationIndex
        frame*spp + s, radiance averaged in pass order, the G-buffer and depth of the last pass, one
        denoise (frameNum = frame, iterationIndex = frame*spp + spp).  orc_trace_frame_spp."""
        it0 = frame * spp
        if spp == 1:
            self.trace(it0)
            self.post_trace()
        else:
            self.L.orc_trace_frame_spp(self.h, it0, spp)
            if self._lights_dirty:  # held for the frame's first pass (cleared there by the C side)
                self._lights_dirty = False
                self.L.orc_set_light_remap(self.h, _p(self._remap_keep), 0, 0)
        if denoise:
            self.denoise(frame, it0 + spp)

    def set_textures(self, chains):
        """chains: list of mip-level lists (level l = (S>>l, S>>l, 4) uint8 RGBA)."""
        info, parts, off = [], [], 0
        for levels in chains:
            info += [levels[0].shape[0], len(levels) - 1]
            for lv in levels:
                info.append(off)
                parts.append(np.ascontiguousarray(lv, np.uint8).reshape(-1))
                off += lv.shape[0] * lv.shape[1]
        self._texels = np.concatenate(parts) if parts else np.zeros(4, np.uint8)
        self._texinfo = np.array(info, np.int32)
        self.L.orc_set_textures(self.h, _p(self._texels), off, _p(self._texinfo), len(chains))

    def set_material_textures(self, block_id, albedo=-1, normal=-1, rough=-1, metal=-1, uv_scale=1.0,
                              world_grid=True):
        self.L.orc_set_material_textures(self.h, block_id, albedo, normal, rough, metal, float(uv_scale),
                                         int(world_grid))

    def set_prev_scene_empty(self, on):
        """The next trace's ReSTIR temporal visibility sees no previous scene (after a voxel edit)."""
        self.L.orc_set_prev_scene_empty(self.h, int(on))

    def post_trace(self):
        self.L.orc_post_trace(self.h)

    def set_denoise_params(self, fl, ints):
        fl = np.asarray(fl, np.float32)
        ints = np.asarray(ints, np.int32)
        self.L.orc_set_denoise_params(self.h, _p(fl), _p(ints))

    def denoise(self, frame, it):
        self.L.orc_denoise(self.h, frame, it)

    def run_pass(self, which, arg=0, arg2=0):
        self.L.orc_pass(self.h, which, arg, arg2)

    def set_band(self, y0, y1):
        self.L.orc_set_band(self.h, y0, y1)

    def _alloc(self, which):
        n = self.W * self.H
        if which == 14:
            return np.zeros(2 * n, RESERVOIR_DTYPE)
        if which in FLOAT1:
            return np.zeros((self.H, self.W), np.float32)
        return np.zeros((self.H, self.W, 4), np.float32)

    def read(self, which):
        out = self._alloc(which)
        self.L.orc_buffer(self.h, which, _p(out), 0)
        return out

    def write(self, which, data):
        ref = self._alloc(which)
        data = np.ascontiguousarray(data, dtype=ref.dtype).reshape(ref.shape)
        self.L.orc_buffer(self.h, which, _p(data), 1)

    def rand(self, i, j, s, d):
        return self.L.orc_rand(self.h, i, j, s, d)

    def rays(self, rays, mode=0):
        """mode 0: DDA closest, 1: brute-force mesh caster, 2: DDA occluded."""
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        n = rays.shape[0]
        out = np.zeros((n, 6), np.int32)
        t = np.zeros(n, np.float32)
        self.L.orc_dda(self.h, n, _p(rays), _p(out), _p(t), mode)
        return out, t


def postprocess(frame_in, depth, params, state, dt_ms, sun=None, sun_luminance=1.0):
    """PostProcessor::run restated (orc_post.cpp) on a W x H x 4 float32 denoiser output.
    params: a ctypes struct laid out as vxpt_post_params; state: float32[2] (average
    luminance, exposure), updated in place; sun: (px, py, u, v) when the sun projects
    on screen.  Returns the W x H x 4 frame."""
    L = lib()
    h, w = frame_in.shape[:2]
    src = np.ascontiguousarray(frame_in, dtype=np.float32)
    dep = np.ascontiguousarray(depth, dtype=np.float32)
    out = np.zeros((h, w, 4), np.float32)
    on, px, py, u, v = (0, 0, 0, 0.0, 0.0) if sun is None else (1,) + tuple(sun)
    L.orc_postprocess(w, h, src.ctypes.data, dep.ctypes.data, ctypes.addressof(params), state.ctypes.data,
                      float(dt_ms), int(on), int(px), int(py), float(u), float(v), float(sun_luminance),
                      out.ctypes.data)
    return out


# ---------------------------------------------------------------- instanced meshes + lights
# (restatements of BlockManager, VoxelEngine::collectInstanceTransforms,
# generateInstanceLights and AliasTable::update -- the C part is orc_lights.cpp)
N_BLOCK_TYPES = 30  # BlockTypeNum (generated/voxelengine/BlockType.h:39)


def parse_obj(path):
    """ObjUtils::extractMeshFromOBJ (ObjUtils.cpp:13-120): (pos [T,3,3], uv [T,3,2]) float32, one
    vertex per face corner; the first three corners of a face; 1-based indices clamped at the
    first element, a missing texcoord index reads element 0.  Floats through strtof, as the
    stream extraction does (no double rounding)."""
    libc = ctypes.CDLL(None)
    libc.strtof.restype = ctypes.c_float
    libc.strtof.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p)]

    def f32(tok):
        return libc.strtof(tok.encode(), None)

    def lead_int(s):
        k = 0
        if k < len(s) and s[k] in "+-":
            k += 1
        while k < len(s) and s[k].isdigit():
            k += 1
        digits = s[:k]
        return (int(digits), k) if digits.lstrip("+-") else (None, 0)

    vp, vt, pi, ti = [], [], [], []
    for line in open(path):
        t = line.split()
        if not t:
            continue
        if t[0] == "v":
            vp.append([f32(t[k + 1]) if k + 1 < len(t) else 0.0 for k in range(3)])
        elif t[0] == "vt":
            vt.append([f32(t[k + 1]) if k + 1 < len(t) else 0.0 for k in range(2)])
        elif t[0] == "f":
            for c in t[1:4]:
                v, p = lead_int(c)
                if v is None:
                    raise ValueError("bad face corner " + c)
                if p < len(c) and c[p] == "/":
                    p += 1
                tx = 0
                if p >= len(c) or c[p] != "/":
                    tv, _ = lead_int(c[p:])
                    tx = tv if tv is not None else 0
                pi.append(max(v - 1, 0))
                ti.append(max(tx - 1, 0))
    n = len(pi) - len(pi) % 3
    pos = np.array([vp[i] if i < len(vp) else [0.0] * 3 for i in pi[:n]], np.float32).reshape(-1, 3, 3)
    uv = np.array([vt[i] if i < len(vt) else [0.0] * 2 for i in ti[:n]], np.float32).reshape(-1, 3, 2)
    return pos, uv


def instance_id(first, width, obj, x, y, z):
    """PositionToInstanceId (VoxelMath.h:120-133): first = the first instanced block id, width = the
    world's x extent; every coordinate clamped to width - 1."""
    W = width
    x, y, z = min(x, W - 1), min(y, W - 1), min(z, W - 1)
    return first + obj * W * W * W + (x + W * (z + W * y))


def collect_instances(ids, chunks, blocks):
    """VoxelEngine::collectInstanceTransforms (VoxelEngine.cu:323-384) on a chunk-major id grid.
    blocks: {block id: dict(instanced=bool, light_base=int)}.  Returns int32 [N, 5] rows
    (object, instance id, x, y, z) ordered by object then instance id; for a repeated instance
    id the last cell in x, y, z order wins."""
    cx, cy, cz = chunks
    W, H, D = cx * 32, cy * 32, cz * 32
    g = ids.reshape(cy, cz, cx, 32, 32, 32)  # chunk (y, z, x), then cell (y, z, x)
    grid = g.transpose(2, 5, 0, 3, 1, 4).reshape(W, H, D)  # [x, y, z]
    inst = [b for b in range(N_BLOCK_TYPES) if blocks.get(b, {}).get("instanced")]
    first = inst[0] if inst else N_BLOCK_TYPES
    by_obj = {}

    def iid(obj, x, y, z):
        return instance_id(first, W, obj, x, y, z)

    for obj in range(first - 1, N_BLOCK_TYPES - 1):
        block = obj + 1
        base = blocks.get(block, {}).get("light_base", 0)
        hit = (grid == block) | ((grid == base) if base else False)
        for x, y, z in zip(*np.nonzero(hit)):  # x, y, z lexicographic
            x, y, z = int(x), int(y), int(z)
            by_obj.setdefault(obj, {})[iid(obj, x, y, z)] = (x, y, z)
            if base and grid[x, y, z] == block:
                by_obj.setdefault(base - 1, {})[iid(base - 1, x, y, z)] = (x, y, z)
    rows = [(o, i) + by_obj[o][i] for o in sorted(by_obj) for i in sorted(by_obj[o])]
    return np.array(rows, np.int32).reshape(-1, 5)


def tri_lights(tri, cells, radiance):
    """generateLightInfosKernel + extractRadianceKernel: (records uint32 [I*T, 8], weights f32)."""
    tri = np.ascontiguousarray(tri, np.float32).reshape(-1, 9)
    cells = np.ascontiguousarray(cells, np.int32).reshape(-1, 3)
    rad = np.ascontiguousarray(radiance, np.float32)
    out = np.zeros((len(tri) * len(cells), 8), np.uint32)
    w = np.zeros(len(tri) * len(cells), np.float32)
    if len(out):
        lib().orc_tri_lights(_p(tri), len(tri), _p(cells), len(cells), _p(rad), _p(out), _p(w))
    return out, w


def alias_table(weights):
    """AliasTable::update's CPU build (AliasTable.cu:58-131) in binary32: p = w / sum,
    scaled = p * n, FIFO small/large queues; the sum accumulated in binary64 and rounded once
    (the library's choice for thrust::reduce's unspecified order).  Returns (q, p, alias, sum)."""
    from collections import deque
    w = np.asarray(weights, np.float32)
    n = len(w)
    s = np.float32(np.sum(w.astype(np.float64)))
    prob = (w / s).astype(np.float32)
    scaled = (prob * np.float32(n)).astype(np.float32)
    alias = np.full(n, -1, np.int32)
    small = deque(i for i in range(n) if scaled[i] < np.float32(1.0))
    large = deque(i for i in range(n) if not scaled[i] < np.float32(1.0))
    while small and large:
        si, li = small.popleft(), large.popleft()
        alias[si] = li
        scaled[li] = np.float32(scaled[li] - np.float32(np.float32(1.0) - scaled[si]))
        (small if scaled[li] < np.float32(1.0) else large).append(li)
    for i in list(small) + list(large):
        scaled[i] = np.float32(1.0)
    return scaled, prob, alias, s


def mesh_probe(models, rows, rays, cull):
    """Closest instanced-mesh hit by brute force (orc_mesh_probe).  models: {block: pos [T,3,3]};
    rows: vxpt_get_instances rows (object, id, x, y, z); rays [N, 8].  Returns (out [N,4], ids [N,2])."""
    rows = np.asarray(rows, np.int32).reshape(-1, 5)
    tris, off, cnt = [], [], []
    acc = 0
    for r in rows:
        pos = models.get(int(r[0]) + 1)
        k = 0 if pos is None else len(pos)
        off.append(acc)
        cnt.append(k)
        if k:
            tris.append(np.asarray(pos, np.float32).reshape(-1, 9))
        acc += k
    tris = np.ascontiguousarray(np.concatenate(tris) if tris else np.zeros((1, 9), np.float32), np.float32)
    off, cnt = np.array(off + [0], np.int32), np.array(cnt + [0], np.int32)
    cells = np.ascontiguousarray(rows[:, 2:5].astype(np.float32).reshape(-1) if len(rows) else np.zeros(3, np.float32))
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
    out, ids = np.zeros((len(rays), 4), np.float32), np.zeros((len(rays), 2), np.int32)
    lib().orc_mesh_probe(_p(tris), _p(off), _p(cnt), _p(cells), len(rows), _p(rays), len(rays), int(cull), _p(out),
                         _p(ids))
    return out, ids
