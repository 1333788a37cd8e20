// ORACLE (test infrastructure only): C-ABI over the CPU restatement, loaded by
// tests/ (ctypes), __graft_entry__.smoke() and bench.py's cpu_baseline leg.
#include <cstring>
#include <memory>

#include "orc_trace.h"

using namespace orc;

namespace {
struct Ctx {
    Scene s;
    Frame f;
    DenoiseParams dp;
};
std::vector<F4> *f4_buf(Frame &f, int id) {
    switch (id) {
        case 0: return &f.illum;
        case 2: return &f.normalRough;
        case 3: return &f.geoNormalThin;
        case 4: return &f.albedo;
        case 6: return &f.matParam;
        case 7: return &f.motion;
        case 8: return &f.prevNormalRough;
        case 9: return &f.prevGeoNormalThin;
        case 10: return &f.prevAlbedo;
        case 11: return &f.prevMatParam;
        case 15: return &f.ping;
        case 16: return &f.pong;
        case 17: return &f.prevIllum;
        case 18: return &f.prevFast;
        case 21: return &f.output;
        default: return nullptr;
    }
}
std::vector<float> *f1_buf(Frame &f, int id) {
    switch (id) {
        case 1: return &f.depth;
        case 5: return &f.material;
        case 12: return &f.prevDepth;
        case 13: return &f.prevMaterial;
        case 19: return &f.histLen;
        case 20: return &f.prevHistLen;
        case 49: return &f.clampBits;
        default: return nullptr;
    }
}
}  // namespace

extern "C" {

void *orc_create(int W, int H, const char *tablesDir) {
    auto *c = new Ctx();
    if (!c->s.bn.load(tablesDir) || !c->s.sky.load_tables(tablesDir)) { delete c; return nullptr; }
    c->f.alloc(W, H);
    return c;
}
void orc_destroy(void *p) { delete static_cast<Ctx *>(p); }

void orc_set_bounces(void *p, int total, int diffuse) {
    auto *c = static_cast<Ctx *>(p);
    c->s.totalBounceLimit = total;
    c->s.diffuseBounceLimit = diffuse;
}

// flags: bit0 keep shader balls, bit1 global-y heights (synthetic tall worlds, see orc_scene.cpp)
int orc_terrain(void *p, int cx, int cy, int cz, float heightScale, float freqDen, int useFma, int flags) {
    auto *c = static_cast<Ctx *>(p);
    generate_terrain(c->s.world, cx, cy, cz, heightScale, freqDen, useFma != 0, (flags & 1) != 0, (flags & 2) != 0);
    return 0;
}
int orc_set_voxels(void *p, const uint8_t *ids, int cx, int cy, int cz) {
    auto *c = static_cast<Ctx *>(p);
    c->s.world.cx = cx; c->s.world.cy = cy; c->s.world.cz = cz;
    c->s.world.ids.assign(ids, ids + (size_t)cx * cy * cz * 32768);
    return 0;
}
int orc_get_voxels(void *p, uint8_t *out) {
    auto *c = static_cast<Ctx *>(p);
    std::memcpy(out, c->s.world.ids.data(), c->s.world.ids.size());
    return (int)c->s.world.ids.size();
}
void orc_set_material(void *p, int blockId, float r, float g, float b, float rough, int metallic, float transl,
                      int materialId) {
    auto *c = static_cast<Ctx *>(p);
    Material &m = c->s.mats[blockId];
    m.albedo = F3(r, g, b);
    m.roughness = rough;
    m.metallic = metallic != 0;
    m.translucency = transl;
    m.materialId = materialId;
}
int orc_set_sky(void *p, float tod, float axis, float rot, float bright) {
    static_cast<Ctx *>(p)->s.sky.build(tod, axis, rot, bright);
    return 0;
}
// Inject sky/sun maps produced elsewhere (e.g. the GPU) and rebuild the alias tables.
void orc_set_sky_maps(void *p, const float *sky, const float *sun, const float *sunDir) {
    Sky &k = static_cast<Ctx *>(p)->s.sky;
    k.sky.assign(sky, sky + (size_t)k.skyW * k.skyH * 4);
    k.sun.assign(sun, sun + (size_t)k.sunW * k.sunH * 4);
    k.sunDir = F3(sunDir[0], sunDir[1], sunDir[2]);
    std::vector<float> a((size_t)k.skyW * k.skyH), b((size_t)k.sunW * k.sunH);
    for (size_t i = 0; i < a.size(); ++i) a[i] = luminance(F3(k.sky[4 * i], k.sky[4 * i + 1], k.sky[4 * i + 2]));
    for (size_t i = 0; i < b.size(); ++i) b[i] = luminance(F3(k.sun[4 * i], k.sun[4 * i + 1], k.sun[4 * i + 2]));
    k.skyAlias = build_alias(a, k.skySum);
    k.sunAlias = build_alias(b, k.sunSum);
}
void orc_get_sky(void *p, float *sky, float *sun, float *sunDir, float *alias_q, float *alias_p, int *alias_a) {
    Sky &k = static_cast<Ctx *>(p)->s.sky;
    if (sky) std::memcpy(sky, k.sky.data(), k.sky.size() * 4);
    if (sun) std::memcpy(sun, k.sun.data(), k.sun.size() * 4);
    if (sunDir) { sunDir[0] = k.sunDir.x; sunDir[1] = k.sunDir.y; sunDir[2] = k.sunDir.z; }
    if (alias_q)
        for (size_t i = 0; i < k.skyAlias.size(); ++i) {
            alias_q[i] = k.skyAlias[i].q; alias_p[i] = k.skyAlias[i].p; alias_a[i] = k.skyAlias[i].alias;
        }
}
// which: 0 = current camera, 1 = previous (history) camera
void orc_set_camera(void *p, const float *pos, const float *dir, float fovDeg, int which) {
    auto *c = static_cast<Ctx *>(p);
    Camera cam = make_offline_camera(c->f.W, c->f.H, F3(pos[0], pos[1], pos[2]), F3(dir[0], dir[1], dir[2]), fovDeg);
    (which ? c->s.prevCam : c->s.cam) = cam;
}
// out: pos3 dir3 uvToWorld(9, m00 m10 m20 m01 ...) worldToUv(9) res2 invRes2 tanHalfFov2 yaw pitch = 32 floats
void orc_get_camera(void *p, int which, float *o) {
    auto *c = static_cast<Ctx *>(p);
    const Camera &k = which ? c->s.prevCam : c->s.cam;
    const float v[32] = {k.pos.x, k.pos.y, k.pos.z, k.dir.x, k.dir.y, k.dir.z,
                         k.uvToWorld.m00, k.uvToWorld.m10, k.uvToWorld.m20, k.uvToWorld.m01, k.uvToWorld.m11,
                         k.uvToWorld.m21, k.uvToWorld.m02, k.uvToWorld.m12, k.uvToWorld.m22,
                         k.worldToUv.m00, k.worldToUv.m10, k.worldToUv.m20, k.worldToUv.m01, k.worldToUv.m11,
                         k.worldToUv.m21, k.worldToUv.m02, k.worldToUv.m12, k.worldToUv.m22,
                         k.res.x, k.res.y, k.invRes.x, k.invRes.y, k.tanHalfFov.x, k.tanHalfFov.y, k.yaw, k.pitch};
    std::memcpy(o, v, sizeof(v));
}
// Camera with explicit yaw/pitch (renderer/test/camera KAT set-up: init(w,h), yaw, pitch, update)
void orc_camera_kat(int w, int h, float yaw, float pitch, const float *uv, int n, float *dirs, float *uvBack) {
    Camera c;
    c.init(w, h);
    c.yaw = yaw;
    c.pitch = pitch;
    c.update_matrices();
    for (int i = 0; i < n; ++i) {
        F3 d = c.uv_to_dir(F2(uv[2 * i], uv[2 * i + 1]));
        dirs[3 * i] = d.x; dirs[3 * i + 1] = d.y; dirs[3 * i + 2] = d.z;
        F2 b = c.dir_to_uv(d);
        uvBack[2 * i] = b.x; uvBack[2 * i + 1] = b.y;
    }
}
void orc_copy_camera_to_prev(void *p) {
    auto *c = static_cast<Ctx *>(p);
    c->s.prevCam = c->s.cam;
}

void orc_trace(void *p, int it, int y0, int y1, int primaryOnly) {
    auto *c = static_cast<Ctx *>(p);
    trace_frame(c->s, c->f, it, y0, y1, primaryOnly != 0);
}
void orc_post_trace(void *p) { post_trace_copies(static_cast<Ctx *>(p)->f); }

// The trace passes of one spp > 1 frame (the benchmarked frame): spp
// 1-spp passes (RayGen.cu:102-182 each) at iterationIndex it0 + s, s = 0..spp-1.
// - Pass s > 0 takes pass s-1 as its ReSTIR history (Restir.h:348-381 GetPrevSurface reads the
//   previous pass's depth / normal / material, reservoirs by iterationIndex parity, Restir.h:13,50)
//   and pass s-1's camera, the frame's own: prevCam = cam.  Pass 0 reads the previous frame's last
//   pass through the denoiser's history copies (Denoiser.cu:394-407) and the frame's history camera.
// - Radiance averaged in pass order, acc = acc + r * (1/spp) per channel in binary32 (first pass
//   from 0); .w, depth and every G-buffer plane are the last pass's.
// - The light-id remap and the empty previous scene of an edit hold for the frame's first pass only.
// Leaves the average in illum for denoise_frame(frameNum, it0 + spp) and the denoiser's history
// copies (prevNormalRough / prevDepth / prevMaterial) as the previous frame left them.
void orc_trace_frame_spp(void *p, int it0, int spp) {
    auto *c = static_cast<Ctx *>(p);
    Scene &s = c->s;
    Frame &f = c->f;
    const size_t n = (size_t)f.W * f.H;
    const std::vector<F4> histNr = f.prevNormalRough;
    const std::vector<float> histDepth = f.prevDepth, histMat = f.prevMaterial;
    const Camera histCam = s.prevCam;
    std::vector<F4> acc(n);
    const float scale = 1.0f / (float)spp;
    for (int k = 0; k < spp; ++k) {
        if (k > 0) {
            f.prevNormalRough = f.normalRough;
            f.prevDepth = f.depth;
            f.prevMaterial = f.material;
            s.prevCam = s.cam;
        }
        trace_frame(s, f, it0 + k, 0, f.H, false);
        post_trace_copies(f);
        s.lightsDirty = false;
        s.prevSceneEmpty = false;
        for (size_t i = 0; i < n; ++i) {
            const F4 r = f.illum[i];
            F4 a = k == 0 ? F4(0.0f) : acc[i];
            a.x = a.x + r.x * scale;
            a.y = a.y + r.y * scale;
            a.z = a.z + r.z * scale;
            a.w = r.w;
            acc[i] = a;
        }
    }
    f.prevNormalRough = histNr;
    f.prevDepth = histDepth;
    f.prevMaterial = histMat;
    s.prevCam = histCam;
    f.illum = acc;
}
void orc_set_prev_scene_empty(void *p, int on) { static_cast<Ctx *>(p)->s.prevSceneEmpty = on != 0; }
// the light-id remap of the next pass (dirty = 0: the pass after it, no remap)
void orc_set_light_remap(void *p, const int *remap, int prevNumLights, int dirty) {
    Scene &s = static_cast<Ctx *>(p)->s;
    s.prevNumLights = prevNumLights;
    s.lightRemap.assign(remap, remap + (prevNumLights > 0 ? prevNumLights : 0));
    s.lightsDirty = dirty != 0;
}
// textures: nTex mip chains; info per texture = size, maxLod, then maxLod + 1 level offsets (texels)
void orc_set_textures(void *p, const uint8_t *texels, size_t nTexels, const int *info, int nTex) {
    Scene &s = static_cast<Ctx *>(p)->s;
    s.texels.assign(texels, texels + 4 * nTexels);
    s.textures.clear();
    for (int i = 0; i < nTex; ++i) {
        Texture t;
        t.size = *info++;
        t.maxLod = *info++;
        for (int l = 0; l <= t.maxLod; ++l) t.off.push_back((unsigned)*info++);
        s.textures.push_back(t);
    }
}
void orc_set_material_textures(void *p, int blockId, int albedo, int normal, int rough, int metal, float uvScale,
                               int worldGrid) {
    Material &m = static_cast<Ctx *>(p)->s.mats[blockId];
    m.tex[0] = albedo; m.tex[1] = normal; m.tex[2] = rough; m.tex[3] = metal;
    m.uvScale = uvScale;
    m.worldGridUV = worldGrid != 0;
}
// emissive / thin-film flags and the world-grid uv set-up of a block's material (instanced
// meshes: lantern light, leaves, lantern base); for an emissive block the albedo is its radiance
// (MaterialManager.cpp:162-167)
void orc_set_material_flags(void *p, int blockId, int emissive, int thin, int worldGrid, float uvScale) {
    Material &m = static_cast<Ctx *>(p)->s.mats[blockId];
    m.isEmissive = emissive != 0;
    m.isThinfilm = thin != 0;
    m.worldGridUV = worldGrid != 0;
    m.uvScale = uvScale;
}
// The world's instanced meshes: triangles (9 floats) and texcoords (6 floats) per block type,
// concatenated, with per-block offsets / counts (32 entries); instance rows of 5 ints
// (block, x, y, z, first light or -1); light records (8 u32 each) and their alias table.
void orc_set_meshes(void *p, const float *pos, const float *uv, const int *triOff, const int *triCnt, int nTri,
                    const int *inst, int nInst, const uint32_t *lights, int nLights, const float *aliasQ,
                    const float *aliasP, const int *aliasA) {
    MeshSet &m = static_cast<Ctx *>(p)->s.mesh;
    m.pos.assign(pos, pos + (size_t)nTri * 9);
    m.uv.assign(uv, uv + (size_t)nTri * 6);
    for (int b = 0; b < 32; ++b) { m.triOff[b] = triOff[b]; m.triCnt[b] = triCnt[b]; }
    m.inst.resize(nInst);
    for (int i = 0; i < nInst; ++i) {
        const int *r = inst + (size_t)i * 5;
        m.inst[i].block = r[0];
        m.inst[i].cell = F3((float)r[1], (float)r[2], (float)r[3]);
        m.inst[i].lightBase = r[4];
    }
    m.numLights = nLights;
    m.lights.assign(lights, lights + (size_t)nLights * 8);
    m.lightAlias.resize(nLights);
    for (int i = 0; i < nLights; ++i) m.lightAlias[i] = AliasBin{aliasQ[i], aliasP[i], aliasA[i]};
}
// rows [y0, y1) the denoiser passes compute (multi-GPU band schedule; 0,0 = whole frame)
void orc_set_band(void *p, int y0, int y1) {
    Frame &f = static_cast<Ctx *>(p)->f;
    f.y0 = y0;
    f.y1 = y1;
}
void orc_set_denoise_params(void *p, const float *fl, const int *in) {
    DenoiseParams &d = static_cast<Ctx *>(p)->dp;
    d.maxAccumulatedFrameNum = fl[0]; d.maxFastAccumulatedFrameNum = fl[1]; d.phiLuminance = fl[2];
    d.lobeAngleFraction = fl[3]; d.roughnessFraction = fl[4]; d.depthThreshold = fl[5];
    d.disocclusionThreshold = fl[6]; d.disocclusionThresholdAlternate = fl[7]; d.denoisingRange = fl[8];
    d.enableTemporalAccumulation = in[0]; d.enableHistoryFix = in[1]; d.enableHistoryClamping = in[2];
    d.enableSpatialFiltering = in[3]; d.enableFireflyFilter = in[4]; d.atrousIterationNum = in[5];
}
void orc_denoise(void *p, int frameNum, int it) {
    auto *c = static_cast<Ctx *>(p);
    denoise_frame(c->s, c->f, c->dp, frameNum, it);
}
// Single passes: 0 firefly(arg=parity) 1 copy_sky 2 temporal 3 history_fix 4 history_clamp
// 5 atrous_smem 6 atrous ping->pong (arg=step, arg2=frameIndex) 7 atrous pong->ping 8 copy_nonsky(arg=src buf id)
// 9 history copies
void orc_pass(void *p, int which, int arg, int arg2) {
    auto *c = static_cast<Ctx *>(p);
    Frame &f = c->f;
    switch (which) {
        case 0: pass_firefly(c->s, f, arg, c->dp.phiLuminance); break;
        case 1: pass_copy_sky(f); break;
        case 2: pass_temporal(c->s, f, c->dp); break;
        case 3: pass_history_fix(c->s, f); break;
        case 4: pass_history_clamp(f); break;
        case 5: pass_atrous_smem(c->s, f, c->dp); break;
        case 6: pass_atrous(c->s, f, f.ping, f.pong, c->dp, (unsigned)arg2, (unsigned)arg); break;
        case 7: pass_atrous(c->s, f, f.pong, f.ping, c->dp, (unsigned)arg2, (unsigned)arg); break;
        case 8: { auto *b = f4_buf(f, arg); if (b) pass_copy_nonsky(f, *b); } break;
        case 9: pass_history_copies(f); break;
        case 10: pass_frame0(f); break;
        default: break;
    }
}
// dir 0: read buffer into data; 1: write data into buffer.  id 14 = reservoirs (2*W*H*20 B)
int orc_buffer(void *p, int id, void *data, int dir) {
    Frame &f = static_cast<Ctx *>(p)->f;
    if (id == 14) {
        size_t n = f.reservoir.size() * sizeof(Reservoir);
        if (dir) std::memcpy(f.reservoir.data(), data, n); else std::memcpy(data, f.reservoir.data(), n);
        return (int)n;
    }
    if (auto *b = f4_buf(f, id)) {
        size_t n = b->size() * sizeof(F4);
        if (dir) std::memcpy(b->data(), data, n); else std::memcpy(data, b->data(), n);
        return (int)n;
    }
    if (auto *b = f1_buf(f, id)) {
        size_t n = b->size() * 4;
        if (dir) std::memcpy(b->data(), data, n); else std::memcpy(data, b->data(), n);
        return (int)n;
    }
    return -1;
}

float orc_rand(void *p, int i, int j, int s, int d) { return static_cast<Ctx *>(p)->s.bn.rand(i, j, s, d); }
float orc_perlin(float x, float y, int octaves) {
    static Perlin n(124);
    return n.octave2d_01(x, y, octaves);
}
// rays: n x (o3, d3, tmin, tmax) ; out: n x (hit, x, y, z, face, id) ints + t floats
void orc_dda(void *p, int n, const float *rays, int *out, float *t, int mode) {
    auto *c = static_cast<Ctx *>(p);
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; ++i) {
        const float *r = rays + 8 * i;
        F3 o(r[0], r[1], r[2]), d(r[3], r[4], r[5]);
        if (mode == 2) {
            out[6 * i] = dda_occluded(c->s.world, o, d, r[6], r[7]) ? 1 : 0;
            t[i] = 0;
            continue;
        }
        Hit h = mode == 1 ? mesh_closest(c->s.world, o, d, r[7]) : dda_closest(c->s.world, o, d, r[7]);
        int *q = out + 6 * i;
        q[0] = h.hit; q[1] = h.x; q[2] = h.y; q[3] = h.z; q[4] = h.face; q[5] = h.id;
        t[i] = h.t;
    }
}
}
