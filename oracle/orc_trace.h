// ORACLE (test infrastructure only): frame state + path tracer + denoiser.
#pragma once
#include <cstdint>
#include <vector>
#include "orc_math.h"
#include "orc_scene.h"
#include "orc_sky.h"

namespace orc {

struct Reservoir {  // DIReservoir (RestirCommon.h:6-12)
    uint32_t lightData = 0, uvData = 0;
    float weightSum = 0, targetPdf = 0, M = 0;
};
static_assert(sizeof(Reservoir) == 20, "reservoir is 20 B");

struct Material {  // MaterialParameter subset (SystemParameter.h:11-38)
    F3 albedo{1, 1, 1};
    float roughness = 0.5f;
    bool metallic = false;
    float translucency = 0.0f;
    int materialId = -1;
    bool isEmissive = false, isThinfilm = false;
    int tex[4] = {-1, -1, -1, -1};  // albedo, normal, roughness, metallic texture (-1 = none)
    float uvScale = 1.0f;
    bool worldGridUV = false;
};

// A texture: RGBA8 mip chain (TextureManager.cu:216-259), level l at texels[off[l]], edge size >> l
struct Texture {
    int size = 0, maxLod = 0;
    std::vector<unsigned> off;
};

struct DenoiseParams {  // DenoisingParams (GlobalSettings.h:82-141) with yaml values
    bool enableTemporalAccumulation = true, enableHistoryFix = true, enableHistoryClamping = true;
    bool enableSpatialFiltering = true, enableFireflyFilter = true;
    float maxAccumulatedFrameNum = 30, maxFastAccumulatedFrameNum = 6, phiLuminance = 2;
    float lobeAngleFraction = 0.5f, roughnessFraction = 0.15f, depthThreshold = 0.003f;
    int atrousIterationNum = 1;
    float disocclusionThreshold = 0.01f, disocclusionThresholdAlternate = 0.05f, denoisingRange = 500000.0f;
};

// All per-pixel surfaces of BufferManager.cpp:150-206 that the hot path touches.
struct Frame {
    int W = 0, H = 0;
    // band of rows the denoiser passes compute (multi-GPU schedule; y1 == 0: whole frame)
    int y0 = 0, y1 = 0;
    int by0() const { return y0; }
    int by1() const { return y1 > 0 ? y1 : H; }
    std::vector<F4> illum, normalRough, geoNormalThin, albedo, matParam, motion;
    std::vector<float> depth, material;
    std::vector<F4> prevNormalRough, prevGeoNormalThin, prevAlbedo, prevMatParam;
    std::vector<float> prevDepth, prevMaterial;
    std::vector<Reservoir> reservoir;  // 2*W*H, ping-pong on iterationIndex parity
    std::vector<F4> ping, pong, prevIllum, prevFast, output;
    std::vector<float> histLen, prevHistLen;
    // test diagnostic (buffer 49): the history clamp's decision bits of the last denoise -- 1: the
    // x-only compare cmin.x < centre.x, 2: cmax.x > centre.x, 4: history > 4 (the clamp uses them),
    // 8: the clamp's factor quotient ill-conditioned
    std::vector<float> clampBits;
    void alloc(int w, int h);
};

// Instanced block meshes of a world: object-space triangles per block type,
// the instance rows (vxpt_get_instances order: the cell is the instance's translation), the
// emissive-triangle light records and their alias table.
struct MeshInstance { int block = 0; F3 cell; int lightBase = -1; };  // lightBase: first light, -1 = not emissive
struct MeshSet {
    std::vector<float> pos, uv;           // 9 / 6 floats per triangle, block types concatenated
    int triOff[32] = {}, triCnt[32] = {};  // per block id
    std::vector<MeshInstance> inst;
    std::vector<uint32_t> lights;         // LightInfo records, 8 x u32 each (Light.h:13-23)
    std::vector<AliasBin> lightAlias;
    int numLights = 0;
};

// closest hit of a radiance ray over voxels and meshes; isMesh: row / tri / u / v valid
struct MeshHit { bool hit = false; int row = -1, tri = -1; float t = kRayMax, u = 0, v = 0; };
// brute-force mesh queries (the reference's IAS; meshes.hip walks a BVH to the same answer):
// closest hit with t in [0, tmax], back faces culled, first strictly closer (row, triangle) wins
MeshHit mesh_closest_hit(const MeshSet &m, const F3 &o, const F3 &d, float tmax);
// any triangle, either face, with t in [tmin, tmax]
bool mesh_any_hit(const MeshSet &m, const F3 &o, const F3 &d, float tmin, float tmax);
// the hit's self-intersection-safe front / back spawn points and world normal
// (SelfHit.h:178-193 getTrianglePointAndError, :539-563 getSafeTriangleSpawnOffset,
// :566-656 safeInstancedSpawnOffsetImpl with the instance's translation, :150-164
// offsetSpawnPoint)
void mesh_spawn(const MeshSet &m, const MeshHit &h, F3 &front, F3 &back, F3 &normal);
// texture coordinates at the hit (closesthit.cu:189)
F2 mesh_texcoord(const MeshSet &m, const MeshHit &h);
// TriangleLight::Create (Light.h:85-122) of light record k
struct TriLight { F3 base, edge1, edge2, radiance, normal; float area = 0; };
TriLight tri_light(const MeshSet &m, int k);

struct Scene {
    World world;
    Sky sky;
    BlueNoise bn;
    Material mats[32];   // index = block id (1..12 cubes, 13..29 instanced meshes); 0 unused
    MeshSet mesh;
    Camera cam, prevCam;
    int totalBounceLimit = 3, diffuseBounceLimit = 1;  // RayGen.cu:146-147
    // the pass after a geometry change: prevTopObject = 0 (OptixRenderer.cpp:916-919, 464), so the
    // ReSTIR temporal visibility rays (closesthit.cu:736-755) traverse no scene and see the light
    bool prevSceneEmpty = false;
    // the pass after a light update (VoxelEngine.cu:658-709, OptixRenderer.cpp:447-457): the previous
    // pass's light index i < prevNumLights becomes lightRemap[i] (-1: gone)
    bool lightsDirty = false;
    int prevNumLights = 0;
    std::vector<int> lightRemap;
    std::vector<uint8_t> texels;     // RGBA8 of every texture's mip chain
    std::vector<Texture> textures;    // empty: untextured shading
};

// One 1-spp trace pass (OptixRenderer::render, OptixRenderer.cpp:411-485),
// rows [y0, y1).  primaryOnly: C2 bring-up mode (no shading; G-buffer + sky).
void trace_frame(const Scene &s, Frame &f, int iterationIndex, int y0, int y1, bool primaryOnly);
// Post-trace copies GeoNormal/Albedo/MaterialParameter -> Prev* (OptixRenderer.cpp:476-478)
void post_trace_copies(Frame &f);

// Denoiser::run (Denoiser.cu:24-408); frameNum = OfflineBackend frame counter,
// iterationIndex = value after render() incremented it.
void denoise_frame(const Scene &s, Frame &f, const DenoiseParams &p, int frameNum, int iterationIndex);

// individual passes (exposed for pass-level parity tests)
void pass_firefly(const Scene &s, Frame &f, int reservoirParity, float phiLuminance);
void pass_copy_sky(Frame &f);
void pass_temporal(const Scene &s, Frame &f, const DenoiseParams &p);
void pass_history_fix(const Scene &s, Frame &f);
void pass_history_clamp(Frame &f);
void pass_atrous_smem(const Scene &s, Frame &f, const DenoiseParams &p);
void pass_atrous(const Scene &s, Frame &f, const std::vector<F4> &in, std::vector<F4> &out, const DenoiseParams &p,
                 unsigned frameIndex, unsigned step);
void pass_copy_nonsky(Frame &f, const std::vector<F4> &in);
void pass_history_copies(Frame &f);
void pass_frame0(Frame &f);

}  // namespace orc
