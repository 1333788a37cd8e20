// vxpt -- internal types shared by the host runtime and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>
#include "vx_math.hpp"

namespace vx {

// camera as the kernels see it (shaders/Camera.h:6-150, host-computed matrices)
struct CamDev {
    V3 pos, dir;
    V2 res, invRes, tanHalfFov;
    M3 uvToWorld, worldToUv;
    VX_HD V3 uv_to_dir(V2 uv) const { return normalize(m3_apply(uvToWorld, V3(uv.x, uv.y, 1.0f))); }
    VX_HD V2 dir_to_uv(V3 d) const {
        V3 n = m3_apply(worldToUv, d);
        return {n.x / n.z, n.y / n.z};
    }
};

struct MatDev {  // per block id, MaterialParameter subset (SystemParameter.h:11-38)
    float albedo[3];
    float roughness;
    float translucency;
    int metallic;
    int materialId;
    int thin;
    int tex[4] = {-1, -1, -1, -1};  // albedo, normal, roughness, metallic texture (-1 = none)
    float uvScale = 1.0f;
    int worldGridUV = 0;
    int emissive = 0;  // MaterialParameter.isEmissive: albedo holds the emitted radiance (MaterialManager.cpp:162-167)
};

// One texture's RGBA8 mip chain in the texel buffer (TextureManager.cu:216-259 layout: square,
// power of two, levels 0..maxLod = log2(size) - 2); off[l] = first texel of level l
constexpr int kMaxTexLevels = 14;
struct TexInfo {
    int size, maxLod;
    unsigned off[kMaxTexLevels];
};

struct AliasBin { float q, p; int alias; };

struct Reservoir { uint32_t lightData, uvData; float weightSum, targetPdf, M; };

// Voxel world on the device, laid out for the DDA:
//   macro[m]  one 64-bit occupancy word per 16^3 macro cell (bit = one 4^3 brick,
//             (bx&3) + 4*((bz&3) + 4*(by&3))); m = mx + MX*(mz + MZ*my); 0 = empty macro
//   bricks    u8 block ids, macro-major then brick then cell: a brick is 64
//             contiguous bytes, a macro 4 KiB ((m*64 + brick)*64 + (x&3) + 4*((z&3) + 4*(y&3)))
//   ids       the chunk-major upload layout (x + 32*(z + 32*y) per 32^3 chunk), kept for readback
//   cellMask  one 64-bit word per brick: bit = cell holds a cube block (ids 1..12)
//   top       one bit per 64^3 block (bx + TX*(bz + TZ*by)) when the world has <= 64 of them
struct WorldDev {
    const uint8_t *ids;
    const uint8_t *bricks;
    const uint64_t *macro;
    const uint64_t *cellMask;
    const uint8_t *bdist;     // 8 octant tables of nBricks bytes (brick index as cellMask): edge in bricks
                              // of the largest empty brick cube cornered at the brick and extending into
                              // the octant (0 = occupied, capped at 255); octant = (dx>0) | (dy>0)<<1 | (dz>0)<<2
    const uint32_t *bbox;     // optional (vxpt_tuning.dda_boxes): 8 octant tables of nBricks words, an empty brick
                              // BOX's extents in bricks (x | y << 8 | z << 16; 0 = occupied) grown from the
                              // cube; null: the cube tables alone
    int nBricks;
    int brickSteps;           // cell crossings per brick walk before the walk yields an outer iteration
    int brickStepsCam;        // the same for the camera rays (k_closest, which runs every walk to its end)
                              // (0 = 10: a whole brick); vxpt_tuning.brick_steps
    uint64_t top;
    int topValid;
    const uint16_t *skyTop;   // sky exit (vxpt_tuning.sky_exit; null: off): per x / z direction quadrant q =
                              // (dx > 0) | (dz > 0) << 1 and brick column (bx, bz), 1 + the highest cube cell
                              // row of the columns the quadrant can still reach from it ([q][bz][bx], 0 =
                              // none): a walk not heading down whose cell row is at least that meets no cube
    int cx, cy, cz;       // chunks
    int wx, wy, wz;       // cells
    int mx, my, mz;       // 16^3 macro cells
    int tx, ty, tz;       // 64^3 blocks
};

struct SkyDev {
    const float4 *sky;    // 1024 x 512
    const float4 *sun;    // 32 x 32
    const AliasBin *skyAlias, *sunAlias;
    V3 sunDir;
    int skyW, skyH, sunW, sunH;
    float sunCosMax;
};

struct BlueNoiseDev { const uint8_t *sobol, *scramble, *rank; };

// Per-frame G-buffer planes, SoA, row-major W*H each (BufferManager.cpp:150-186)
struct GBuf {
    float4 *normalRough, *geoNormalThin, *albedo, *matParam;
    float *depth, *material;
    // what a ReSTIR temporal tap reads of this pass's G-buffer (Restir.h:348-381 GetPrevSurface), one
    // 32-byte record per pixel: [2i] = shading normal xyz (the geoNormalThin plane holds the same
    // normal) + roughness with the metallic flag in its sign bit, [2i+1] = albedo xyz + depth.  Written
    // beside the planes by the trace; a tap then reads one 32-byte record instead of five planes.
    float4 *rec;
};

// Per-pixel state of the wavefront trace pass (trace.hip).  One slot per
// pixel in 8x8-tile order (slot = tile*64 + lane, tiles row-major over the
// band), so each 64-lane wave owns one tile in every stage.
// ray queues: 4 per path segment (1 BRDF candidates, 2 RIS visibility, 3 ReSTIR visibility), so at
// most kQueues / 4 segments (vxpt_create bounds total_bounce_limit); straggler queues in kShards shards
constexpr int kQueues = 64;
constexpr int kShards = 8;
constexpr size_t kQueueWords = 2 * kQueues + 4 * kQueues * kShards * 16;
static_assert(kQueueWords % 4 == 0, "k_closest zeroes the counters as uint4");

struct WaveBufs {
    // path state
    float4 *pPos;   // ray origin xyz, primary distance
    float4 *pDir;   // ray direction xyz, BSDF pdf
    float4 *pThr;   // throughput xyz
    float4 *pRad;   // accumulated radiance xyz
    int2 *pMeta;    // x: flags | total segments << 8 | diffuse segments << 16, y: sampler dimension (trace.hip load_meta)
    float4 *pBop;   // BSDF weight of the sampled continuation xyz, terminate flag
    // closest-hit queue (camera / path / BRDF-candidate rays) and its results
    float4 *cRayO, *cRayD;  // o xyz + tmax (< 0: inactive), d xyz
    int4 *cHit;             // cell xyz, face | id << 4 | hit << 12
    float *cT;
    // the diffuse surface being shaded (NEE)
    float4 *sPos;   // front spawn point xyz, hit t
    float4 *sNrm;   // shading normal xyz, roughness
    float4 *sGeo;   // geometric normal xyz, translucency
    float4 *sAlb;   // albedo xyz, metallic
    float4 *sWo;    // wo xyz, skip-albedo flag
    float4 *cSunSky;  // the sun and sky candidates' final weight sum and target pdf (x, y: sun; z, w: sky); a
                      // candidate is selected iff its sample index (nIdx.x / .y) is >= 0 (trace.hip cand_res)
    float4 *rRis;   // the RIS reservoir (lightData, uvData, weightSum, targetPdf; M = 1)
    Reservoir *rRR;
    int4 *nIdx;     // sun light index, sky light index, selected temporal tap, cached-tap mask
    float4 *ls0;    // selected light sample: position / direction xyz, type << 24 | map texel (sun / sky)
    float4 *ls1;    // local lights only: radiance xyz, solid-angle pdf (trace.hip store_ls)
    float4 *tapPsv; // target pdf of the selection at the three temporal taps, first-visibility flag
    float4 *tapM;   // the taps' clamped M
    // instanced meshes: back spawn point of a thin-film surface (xyz, w = thin
    // flag; rays leaving it on the far side start there), the 8 local-light candidates' reservoir
    // and selected sample (position xyz + solid-angle pdf, radiance xyz + type)
    float4 *sBack;
    Reservoir *rLoc;
    float4 *lLoc0, *lLoc1;
    // visibility results: 4 rays per slot (0: RIS/final visibility, 1-3: bias-correction taps)
    uint8_t *oHit;
    // compacted ray queue (trace.hip block_enqueue): o xyz + tmin, d xyz + tmax,
    // result id; one storage reused by the pass's queues, counters 4 per segment
    float4 *qO, *qD;
    int *qId;
    unsigned *qCount;  // kQueueWords: kQueues queue counters, kQueues unused words, then per straggler level (1-4) kQueues queues x kShards shard counters 16 words apart
    // straggler queues (ping-pong by level): walk state of rays stopped at an iteration cap (DdaSaved)
    int4 *sCell[2];
    float4 *sT[2];
    int2 *sFace[2];
};

// Emissive-triangle light record, 32 B (renderer/shaders/Light.h:13-23): centroid, the two
// edge lengths as f16 (lo = edge1), radiance as 4 x f16, the edge directions octahedral
// unorm16x2 encoded
struct LightInfo {
    float center[3];
    uint32_t scalars;
    uint32_t radiance[2];
    uint32_t direction1, direction2;
};
// Instanced-mesh ray queries (the geometry half): two-level BVH -- a TLAS over
// the instances' world boxes, one BLAS per block type's mesh in object space (the instance
// transform is a translation by its cell, VoxelEngine.cu:364-369).  Node boxes are widened at
// build time so that box culling can only drop triangles the exact test would also reject.
// Inner node: count = 0, children left and left + 1; leaf: count primitives from left.
struct BvhNode {
    float lo[3];
    int left;
    float hi[3];
    int count;
};
struct MeshInst {
    float cell[3];
    int block;  // block type -> its BLAS
    int row;    // the instance's row in vxpt_get_instances
};
struct MeshDev {
    const BvhNode *tlas;    // over instances (primitive = MeshInst index)
    const MeshInst *inst;
    const BvhNode *blas;    // every block type's BLAS, concatenated
    const float *tri;       // 9 floats per triangle in BLAS leaf order (object space)
    const int *triId;       // the mesh's own triangle index of each
    const int2 *root;       // per block type: (first BLAS node, first triangle); -1 = no mesh
    int nInst;
};

struct TraceArgs {
    WorldDev world;
    SkyDev sky;
    BlueNoiseDev bn;
    MatDev mats[13];
    CamDev cam, prevCam;
    GBuf cur, prev;
    float4 *illum, *motion;
    Reservoir *resCur;          // written this pass (iterationIndex parity)
    const Reservoir *resPrev;   // read by temporal reuse
    float4 *accum;              // spp accumulation target (nullptr when spp == 1)
    int W, H, y0, y1;
    int iterationIndex;
    int totalBounceLimit, diffuseBounceLimit;
    int segments;               // path segments that can occur (<= totalBounceLimit, see do_trace)
    int primaryOnly;
    float accumScale;           // 1/spp
    int accumFirst;
    WaveBufs wb;
    int tilesX, nSlots;         // 8x8 tiles across the frame width; slots in the band
    int numCU;                  // compute units of the device (traversal grid sizing)
    int iterCap, iterCap2;      // outer DDA iterations before a ray moves to the level-1 / level-2 straggler queue
    int iterCap3, iterCap4;     // > 0: a level-2 (then level-3) resume of that many iterations before the last level
    int prevSceneEmpty;         // the pass after a voxel edit: temporal visibility rays see no previous scene
    const TexInfo *tex;         // texture table (nullptr: no textures loaded)
    const uchar4 *texels;       // every texture's mip chain, RGBA8
    int texEnabled;
    // instanced meshes (mesh.nInst == 0: none, and no mesh kernel runs)
    MeshDev mesh;
    const float *meshUV;        // 6 floats (3 corners' texcoords) per triangle, BLAS leaf order
    const int4 *meshRow;        // per instance row: cell xyz, block id
    const int *meshRowLight;    // per instance row: its first light record, -1 = not emissive
    const MatDev *meshMats;     // materials by block id (0..31)
    const LightInfo *lights;    // emissive-triangle lights (VoxelEngine.cu:53-116)
    const AliasBin *lightAlias;
    int numLights;
    // LoadDIReservoir's remap (Restir.h:48-79): in the pass after a light update (lightsDirty) the
    // previous reservoirs' light index i < prevNumLights becomes lightRemap[i] (-1: empty reservoir)
    const int *lightRemap;
    int prevNumLights;
    int lightsDirty;
    int resumeWgPerCU;  // k_resume workgroups per CU (0: 16)
    int sortMode;       // ray queues grouped by direction class per workgroup (0 off, 1 octant, 2 octant x axis)
    int ldsBricks;      // k_closest reads bricks through a workgroup cache in LDS (trace.hip LdsBricks)
    int resumeSplit;    // straggler walks cut into this many pieces, one lane each (trace.hip k_resume_split)
    int restirWaves;    // k_restir's occupancy bound (0: the compiler's, 4: 4 waves/SIMD)
    int xcdOrder;       // XCD-local workgroup order, bits 1 k_restir, 2 k_closest, 4 k_queue (vxpt_tuning.xcd_order)
    int laterSplit;     // the same for the queues of a path's later segments, after 8 more iterations
    int writeMotion;    // store the (zero) motion vectors: the plane may hold a host upload
    int writePlanes;    // store the G-buffer planes (0: a frame's passes before its last -- only their tap
                        // records are read, by the next pass's temporal reuse)
};

// kernel launchers (defined in the .hip translation units)
hipError_t launch_sky(const float *cfg90, const float *rad10, const float *solar, const float *limb, V3 sunDir,
                      float brightness, float4 *sky, float4 *sun, float *skyPdf, float *sunPdf, int skyW, int skyH,
                      int sunW, int sunH, hipStream_t st);
hipError_t launch_sky_lower(float4 *sky, float *skyPdf, int skyW, int skyH, float sumUpper, hipStream_t st);
// a trace pass in two halves (trace.hip): the first reads nothing of the previous pass; the second
// starts with the temporal reuse.  waitBeforeRestir: event the temporal-reuse kernel waits for (band
// halo exchange), or null
hipError_t launch_trace_front(const TraceArgs &a, hipStream_t st);
hipError_t launch_trace_back(const TraceArgs &a, hipStream_t st, hipEvent_t waitBeforeRestir);
// GBuf::rec of the n pixels from the planes
hipError_t launch_pack_rec(const GBuf &g, size_t n, hipStream_t st);
hipError_t launch_probe_rng(const BlueNoiseDev &bn, int n, const int *q, float *out, hipStream_t st);

struct DenoiseParamsDev {
    float maxAcc, maxFast, phiL, lobeAngleFraction, roughnessFraction, depthThreshold;
    float disocclusionThreshold, disocclusionThresholdAlternate, denoisingRange;
    int enableTA, enableHF, enableHC, enableSpatial, enableFirefly, atrousIterations;
};

struct DenoiseArgs {
    int W, H;
    int y0, y1;                 // band of rows the passes compute (whole frame: 0, H)
    CamDev cam, prevCam;
    DenoiseParamsDev p;
    // inputs of this frame
    float4 *illum;
    const float4 *normalRough, *albedo, *motion;
    const float *depth, *material;
    const float4 *prevNormalRough;
    const float *prevDepth;
    Reservoir *reservoir;       // the pass's reservoirs (parity usedIteration&1)
    // persistent denoiser state
    float4 *ping, *pong, *prevIllum, *prevFast, *output;
    float *histLen, *prevHistLen;
    // world position of every pixel's primary hit (world_pos of depth) + 16-bit material, built
    // once per frame by k_firefly: the stencil passes read it instead of re-deriving a camera
    // ray per tap
    float4 *wpos;
    // history-fix lists (k_temporal -> k_history_fix), per 16x16 tile of the band's
    // grid: up to 256 pixel indices at tile*256, count in hfCount[tile]
    uint32_t *hfList, *hfCount;
    // firefly lists per 16x16 tile of the band: ffCount[tile] entries at tile*256 (local pixel
    // index, filtered radiance, replacement reservoir); the consumer resets the count
    uint32_t *ffCount;
    uint32_t *ffIndex;
    // detected fireflies for k_firefly_filter: {pixel, neighbour weight sum, neighbour count}; the
    // count is reset by the lists' consumer (k_temporal or k_firefly_apply)
    uint4 *ffCand;
    uint32_t *ffCandCount;
    float4 *ffColor;
    Reservoir *ffRes;
    // launch-uniform terms of the temporal pass, computed once on the host with the same IEEE
    // operations (a division per wave each on the device): 1/W, 1/H, the two disocclusion
    // thresholds, the frustum scale tanHalfFov.x / (res.x / 2), 1/(maxAcc+1),
    // 1/(maxFast+1)
    float invW, invH, thrB, thrA, frustumK, invAcc1, invFast1;
    // parity hook (vxpt_debug_clamp_decisions): the history clamp's decision bits per pixel, or null
    float *clampDbg;
    // launch shapes (vxpt_tuning; host side only: read by the launch functions)
    struct {
        int ffFused, taSupertiles, hfSplit, stencilTile;
    } tune;
};

// post-processing (postprocess.hip; ToneMappingParams + PostProcessingPipelineParams, GlobalSettings.h:10-186)
struct PostParamsDev {
    float manualExposure;
    int curve;                      // 0 Narkowicz ACES, 1 Uncharted 2, 2 Reinhard
    float whitePoint, contrast, saturation, lift, gain;
    int enableBloom;
    float bloomThreshold, bloomIntensity, bloomRadius;
    int enableAutoExposure;
    float exposureSpeed, exposureMin, exposureMax, exposureCompensation;
    float histogramMinPercent, histogramMaxPercent, targetLuminance;
    int enableVignette;
    float vignetteStrength, vignetteRadius, vignetteSmoothness;
    int enableLensFlare;
    float lensFlareIntensity, lensFlareGhostSpacing;
    int lensFlareGhostCount;
    float lensFlareHaloRadius, lensFlareSunSize, lensFlareDistortion;
    int crosshair;
};

struct PostArgs {
    int W, H;
    PostParamsDev p;
    const float4 *input;            // the denoiser output (IlluminationOutputBuffer)
    float4 *bloomA, *bloomB;        // bloom extract (wide-radius path) / horizontally blurred bloom
    float4 *frame;                  // result: Float4(sRGB colour, 0) (CopyToInteropBuffer)
    const float *depth;             // lens-flare sun visibility
    unsigned *hist;                 // 256 luminance bins (integer counts, cleared by k_exposure) + the sun flag
    int y0, y1;                     // the rows this context composes (its band; 0, H unbanded)
    float *state;                   // [0] current average luminance, [1] exposure of this frame
    float dtMs;                     // frame time for the exposure adaptation (Timer::getDeltaTime, ms)
    int sunOnScreen, sunPx, sunPy;  // ProjectSunToScreen (PostProcessingPipeline.cu:187-206)
    float sunU, sunV, sunLuminance;
};
hipError_t launch_postprocess(const PostArgs &a, hipStream_t st);
hipError_t launch_post_phase1(const PostArgs &a, hipStream_t st);
hipError_t launch_post_phase2(const PostArgs &a, hipStream_t st);
int post_bloom_half(const PostArgs &a);  // rows of bloomB the compose pass taps above and below
bool decode_png(const std::string &path, int &w, int &h, int &ch, std::vector<uint8_t> &px);
bool load_obj(const std::string &path, std::vector<float> &pos, std::vector<float> &uv);

// closest hit (tie: smaller t, then instance, then triangle) of n rays (o.xyz, tmin, d.xyz, tmax);
// out: t, u, v, hit flag per ray; ids: instance, triangle.  cull = skip back faces (radiance rays)
hipError_t launch_mesh_probe(const MeshDev &m, const float *rays, int n, int cull, float *out, int *ids,
                             hipStream_t st);
// any hit, both faces (visibility rays): occluded 1/0 per ray
hipError_t launch_mesh_occluded(const MeshDev &m, const float *rays, int n, unsigned char *occluded, hipStream_t st);
// One emissive block type's lights: every (instance, triangle) of its mesh, instance-major
// (VoxelEngine.cu:53-116), written from out[0]; weight[k] = luminance(radiance) * area of the
// decoded record (extractRadianceKernel, :139-147).  tri: 9 floats per triangle (object
// space), inst: 3 ints per instance (the cell = the translation of its 3x4 transform).
hipError_t launch_tri_lights(const float *tri, int nTri, const int *inst, int nInst, V3 radiance, LightInfo *out,
                             float *weight, hipStream_t st);

hipError_t launch_firefly(const DenoiseArgs &a, int wy0, int wy1, bool detect, bool apply, hipStream_t st);
hipError_t launch_frame0_init(const DenoiseArgs &a, hipStream_t st);
hipError_t launch_stream_mark(hipStream_t st);
hipError_t launch_temporal(const DenoiseArgs &a, hipStream_t st);
hipError_t launch_history_fix(const DenoiseArgs &a, hipStream_t st);
hipError_t launch_history_clamp(const DenoiseArgs &a, hipStream_t st);
hipError_t launch_atrous_smem(const DenoiseArgs &a, hipStream_t st);
// final: also writes output (sky pixels copy illum, others illum*albedo)
hipError_t launch_atrous(const DenoiseArgs &a, const float4 *in, float4 *out, unsigned step, unsigned frameIndex,
                         bool final, hipStream_t st);
hipError_t launch_copy_output(const DenoiseArgs &a, const float4 *in, hipStream_t st);

}  // namespace vx
