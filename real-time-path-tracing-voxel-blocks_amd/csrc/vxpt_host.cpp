// vxpt -- host runtime behind the C ABI (include/vxpt.h).
//
// Owns the device memory of one GPU (the reference's BufferManager /
// SkyModel / MaterialManager singletons), sets up the camera and the sky the
// way the reference does on its host (mainOffline.cpp:201-251, Sky.cu:355-396,
// AliasTable.cu:66-153), generates the Perlin terrain (VoxelSceneGen.cu:341-388)
// and sequences the kernels of one frame (OfflineBackend.cpp:46-89).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <cfloat>
#include <fstream>
#include <map>
#include <queue>
#include <random>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/vxpt.h"
#include "box_tables.hpp"
#include "bvh_build.hpp"
#include "light_map.hpp"
#include "vx_internal.hpp"

using namespace vx;

namespace {

// ---------------------------------------------------------------- helpers
template <class T>
struct DBuf {
    T *p = nullptr;
    size_t n = 0;
};

struct GSlot {
    float4 *normalRough = nullptr, *geoNormalThin = nullptr, *albedo = nullptr, *matParam = nullptr;
    float *depth = nullptr, *material = nullptr;
    float4 *rec = nullptr;  // ReSTIR tap records (GBuf::rec), 2 float4 per pixel
    bool recStale = false;  // the planes were written from the host since the records were
};

// Perlin noise (siv::BasicPerlinNoise<float>, voxelengine/ext/PerlinNoise.hpp:229-494, 565-568)
struct Perlin {
    uint8_t p[256];
    explicit Perlin(uint32_t seed) {
        for (int i = 0; i < 256; ++i) p[i] = (uint8_t)i;
        std::mt19937 g(seed);
        for (int i = 1; i < 256; ++i) {
            const uint64_t r = (uint64_t)g() % (uint64_t)(i + 1);
            std::swap(p[i], p[r]);
        }
    }
    static float fade(float t) { return t * t * t * (t * (t * 6 - 15) + 10); }
    static float lerp(float a, float b, float t) { return a + (b - a) * t; }
    static float grad(uint8_t hash, float x, float y, float z) {
        const uint8_t h = hash & 15;
        const float u = h < 8 ? x : y;
        const float v = h < 4 ? y : (h == 12 || h == 14 ? x : z);
        return ((h & 1) == 0 ? u : -u) + ((h & 2) == 0 ? v : -v);
    }
    float noise(float x, float y, float z) const {
        const float X = std::floor(x), Y = std::floor(y), Z = std::floor(z);
        const int ix = (int)X & 255, iy = (int)Y & 255, iz = (int)Z & 255;
        const float fx = x - X, fy = y - Y, fz = z - Z;
        const float u = fade(fx), v = fade(fy), w = fade(fz);
        const uint8_t A = (p[ix] + iy) & 255, B = (p[(ix + 1) & 255] + iy) & 255;
        const uint8_t AA = (p[A] + iz) & 255, AB = (p[(A + 1) & 255] + iz) & 255;
        const uint8_t BA = (p[B] + iz) & 255, BB = (p[(B + 1) & 255] + iz) & 255;
        const float q0 = lerp(grad(p[AA], fx, fy, fz), grad(p[BA], fx - 1, fy, fz), u);
        const float q1 = lerp(grad(p[AB], fx, fy - 1, fz), grad(p[BB], fx - 1, fy - 1, fz), u);
        const float q2 = lerp(grad(p[(AA + 1) & 255], fx, fy, fz - 1), grad(p[(BA + 1) & 255], fx - 1, fy, fz - 1), u);
        const float q3 = lerp(grad(p[(AB + 1) & 255], fx, fy - 1, fz - 1), grad(p[(BB + 1) & 255], fx - 1, fy - 1, fz - 1), u);
        return lerp(lerp(q0, q1, v), lerp(q2, q3, v), w);
    }
    float octave01(float x, float y, int oct) const {
        float r = 0, a = 1;
        for (int i = 0; i < oct; ++i) {
            r += noise(x, y, (float)0.34567) * a;
            x *= 2;
            y *= 2;
            a *= 0.5f;
        }
        if (r <= -1.0f) return 0.0f;
        if (1.0f <= r) return 1.0f;
        return r * 0.5f + 0.5f;
    }
};

// minimal YAML reader for the reference's settings / scene / asset files:
// `section:` headers, `key: value` pairs, `- {k: v, ...}` / `properties: {...}` flow maps
std::string trim(const std::string &s) {
    size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
    return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}
std::map<std::string, std::string> parse_flow_map(const std::string &s) {
    std::map<std::string, std::string> m;
    size_t a = s.find('{'), b = s.rfind('}');
    if (a == std::string::npos || b == std::string::npos) return m;
    std::string body = s.substr(a + 1, b - a - 1);
    int depth = 0;
    std::string cur;
    std::vector<std::string> items;
    for (char c : body) {
        if (c == '[') depth++;
        if (c == ']') depth--;
        if (c == ',' && depth == 0) { items.push_back(cur); cur.clear(); continue; }
        cur += c;
    }
    if (!trim(cur).empty()) items.push_back(cur);
    for (auto &it : items) {
        size_t c = it.find(':');
        if (c == std::string::npos) continue;
        m[trim(it.substr(0, c))] = trim(it.substr(c + 1));
    }
    return m;
}
std::vector<float> parse_list(const std::string &s) {
    std::vector<float> v;
    std::string t = s;
    for (char &c : t)
        if (c == '[' || c == ']' || c == ',') c = ' ';
    std::istringstream is(t);
    float f;
    while (is >> f) v.push_back(f);
    return v;
}
bool as_bool(const std::string &s) { return s == "true" || s == "1" || s == "True"; }

}  // namespace

constexpr int kBlockTypes = 30;  // BlockTypeNum (generated/voxelengine/BlockType.h:39)
constexpr int kPostHist = 257;   // 256 luminance bins + the lens flare's sun flag
constexpr int kMaxSets = 3;      // wavefront state sets (vxpt_ctx::nSets; 4 measured slower on bands)

// the measured best schedule; vxpt_set_tuning changes it per context
vxpt_tuning tuning_defaults() {
    vxpt_tuning t{};
    t.dda_boxes = 1;          // empty-box tables: 7.56 -> 7.06 ms of trace per C3 frame (round 3)
    t.box_cap = 32;           // growth limits swept flat (8:8 .. 32:64 within 0.03 ms, round 3); on the round-6 walk
    t.box_cap_up = 32;        // ladder with the direction sort 8:8 -> 32:32 -1.3 % (four runs each)
    t.brick_steps = 3;        // in-brick walks yield after 3 crossings: 6.44 -> 6.26 ms
    t.cam_steps = 10;         // camera rays walk whole bricks
    t.iter_cap = 4;           // caps 4 / 6 / 8 / 12: 7.02 / 6.84 / 7.07 / 7.63 ms (round 2); with the sky exit
                              // (round 6) 5 against 6: 5.439 / 5.438 / 5.440 / 5.463 -> 5.410 / 5.399 / 5.413 / 5.423 ms
    t.iter_cap2 = 6;          // a second level after 6 more iterations (round 2-6: 16, its walks in resume_split
                              // pieces: 5.74 -> 5.66-5.68 ms; one lane per walk at that level: 7.59 ms, round 2)
    t.iter_cap3 = 12;         // round 6: a third level, 12 more iterations, before the pieces: the ladder 4 / 6 / 12
                              // against 5 / 16: 5.46 -> 5.20 ms per C3 frame (four runs each)
    t.resume_wg_per_cu = 24;  // 4 / 8 / 16 / 32: 6.96 / 6.85 / 6.84 / 6.87 ms (round 2); on the round-6 walk ladder
                              // 16 -> 24: 5.195 -> 5.168 ms (four runs each, every run faster)
    t.sort_mode = 2;          // direction-class sort (octant x dominant axis): until round 6 1.5 % faster traversal,
                              // paid back by the producers; on the walk ladder 5.188 -> 5.156 ms (sort 1), with 32-brick
                              // boxes 5.150 -> 5.067 ms (four runs each)
    t.overlap = 1;            // pass halves on two streams: 6.84 -> 6.06 ms
    t.state_sets = 3;         // 3 sets: 5.409 -> 5.394 ms (four interleaved runs each, every run faster; round 5)
    t.firefly_fused = 1;      // -4 us per chain
    t.ta_supertiles = 1;      // temporal pass traffic 351 -> 266 MB per frame
    t.hf_split = 4;           // 16.3 -> 11.8 us history fix (with readlane sums)
    t.stencil_tile = 16;      // 32x32 tiles: 50.0 -> 55.8 / 48.5 -> 52.4 us
    t.lds_bricks = 0;
    t.resume_split = 16;      // (with iter_cap2 0: every straggler in pieces, 5.73 -> 6.7-9.2 ms)
    t.later_split = 16;       // 4/4 bounces: 16.39 -> 15.67 ms per frame (3/1 has no later segments)
    t.restir_waves = 0;       // 4 waves: whole frames slower (Appendix A); see bench.band_tuning for bands
    t.ghost_rows = 1;         // bands: the chain's ordered exchange groups 7 -> 3 per frame
    t.chain_gate = 1;         // the chain alone on the GPU (its roofline); bench.band_tuning: 0 for bands
    t.sky_exit = 1;           // C3 frame 5.443 -> 5.419 ms (two runs each, both faster); one band 1-2 %
    t.xcd_order = 0;
    t.iter_cap4 = 0;          // a fourth level: 4 / 8 / 16 / 6-8-12 ladders 5.26-5.27 ms, no gain
    t.front_streams = 2;      // first halves of consecutive passes side by side: 5.89 -> 5.76 ms per C3
                              // frame; one 136-row band 1.95 -> 1.63 ms (1.56 with 3 state sets)
    return t;
}
bool tuning_valid(const vxpt_tuning &t) {
    auto in = [](int v, int lo, int hi) { return v >= lo && v <= hi; };
    return in(t.dda_boxes, 0, 1) && in(t.box_cap, 1, 255) && in(t.box_cap_up, 1, 255) && in(t.brick_steps, 1, 64) &&
           in(t.cam_steps, 1, 64) && in(t.iter_cap, 1, 1024) && in(t.iter_cap2, 0, 1024) &&
           in(t.resume_wg_per_cu, 1, 64) && in(t.sort_mode, 0, 2) && in(t.overlap, 0, 1) &&
           in(t.state_sets, 2, kMaxSets) && in(t.firefly_fused, 0, 1) && in(t.ta_supertiles, 0, 1) &&
           in(t.hf_split, 1, 16) && (t.stencil_tile == 16 || t.stencil_tile == 32) && in(t.front_streams, 1, kMaxSets) &&
           in(t.lds_bricks, 0, 1) && (t.resume_split == 1 || t.resume_split == 2 || t.resume_split == 4 ||
                                       t.resume_split == 8 || t.resume_split == 16) &&
           (t.later_split == 1 || t.later_split == 2 || t.later_split == 4 || t.later_split == 8 || t.later_split == 16) &&
           (t.restir_waves == 0 || t.restir_waves == 4) && in(t.ghost_rows, 0, 1) &&
           in(t.chain_gate, 0, 1) && in(t.sky_exit, 0, 1) && in(t.xcd_order, 0, 7) && in(t.iter_cap3, 0, 1024) && in(t.iter_cap4, 0, 1024);
}


struct vxpt_ctx {
    int W = 0, H = 0, dev = 0, rowBegin = 0, rowEnd = 0;
    int totalBounce = 3, diffuseBounce = 1;
    std::string dataDir;
    std::string err;
    hipStream_t stream = nullptr;
    hipEvent_t ev[8] = {};
    hipEvent_t runEv[2] = {};  // around a banded vxpt_render_frames run
    vxpt_timing timing{};
    vxpt_tuning tune = tuning_defaults();

    // scene
    int cx = 0, cy = 0, cz = 0;
    DBuf<uint8_t> voxels;
    DBuf<uint8_t> bricks;
    DBuf<uint64_t> macro, cellMask;
    DBuf<uint8_t> bdist;
    // optional empty-box skip tables (vxpt_tuning.dda_boxes; box_tables.hpp)
    bool useBoxes = tune.dda_boxes != 0;
    BrickPrefix brickPrefix;
    int boxCap = tune.box_cap, boxCapUp = tune.box_cap_up;  // box growth limits (box_tables.hpp)
    std::vector<uint32_t> hBox;
    DBuf<uint32_t> bbox;
    int nBricks = 0;
    uint64_t top = 0;
    int topValid = 0;
    // sky exit (WorldDev::skyTop): per brick column 1 + its highest cube cell row (edits raise it, never
    // lower it: a bound), and its suffix maxima per x / z direction quadrant (the device table)
    std::vector<uint16_t> colTop, hSkyTop;
    DBuf<uint16_t> skyTop;
    // host mirrors of the world: picking, incremental edits, chunk files (the device copies are
    // updated from them in place)
    std::vector<uint8_t> hIds, hBricks, hOd;
    std::vector<uint64_t> hMacro, hCell;
    std::vector<int> topCount;  // cube cells per 64^3 block
    std::vector<uint8_t> hNonAir;  // non-air cells (any id, instanced ones too) per 4^3 brick (brick_lin order)
    // how far an instanced block's mesh reaches outside its cell (the largest vertex overhang of the
    // loaded meshes, at least 1): nearest_surface grows every non-air cell by it
    float meshGrow = 1.0f;
    // world edits / uploads so far, and the last nearest-surface search (band halos of a moving
    // camera): a later position p reuses it as nearDist - |p - nearPos| (1-Lipschitz) while the
    // world is unchanged and that keeps >= 3/4 of the searched distance
    unsigned worldVersion = 0, nearVersion = ~0u;
    V3 nearPos{0.0f, 0.0f, 0.0f};
    float nearDist = 0.0f;
    int prevSceneEmpty = 0;     // the next trace pass's temporal visibility sees no previous scene
    MatDev mats[32] = {};  // by block id: 1..12 cubes (kernel arguments), 13..29 instanced meshes (meshMats)
    CamDev cam{}, prevCam{};
    float camYaw = 0, camPitch = 0;

    // sky
    DBuf<float4> sky, sun;
    DBuf<float> skyPdf, sunPdf;
    DBuf<AliasBin> skyAlias, sunAlias;
    std::vector<AliasBin> hSkyAlias;
    V3 sunDir;
    float tabSky[540], tabSkyRad[60];
    DBuf<float> solar, limb;
    bool skyReady = false;

    // textures (materials.yaml `textures`, TextureManager): per block the albedo / normal /
    // roughness / metallic paths, the loaded RGBA8 mip chains and their table
    std::string texPath[13][4];
    DBuf<uchar4> texels;
    DBuf<TexInfo> texTable;
    std::vector<TexInfo> hTex;
    size_t nTexels = 0;
    int texEnabled = 0;

    // instanced block meshes and their emissive-triangle lights
    struct BlockDef {
        std::string model;
        bool instanced = false, baseLight = false, emissive = false;
        int lightBase = 0;
        float emission[3] = {0.f, 0.f, 0.f};
        int triangles = 0;             // of the loaded mesh (0: missing file)
        std::vector<float> pos, uv;    // 9 / 6 floats per triangle, object space
    };
    bool modelsLoaded = false;
    BlockDef blocks[kBlockTypes];
    std::vector<int32_t> instances;    // (objectId, instanceId, x, y, z) by object, then instance id
    std::vector<uint32_t> lightMap;    // (instanceId, first light, triangles) per emissive instance
    DBuf<LightInfo> lights;
    DBuf<AliasBin> lightAlias;
    DBuf<float> lightTri, lightWeight;
    DBuf<int> lightInst;
    unsigned nLights = 0;
    float localLightLum = 0.0f;
    // light-update state (Scene.h:91-115): the update type, the edits' instance sets, the instance ->
    // (first light, count) table of the last incremental update, and the remap the next pass applies
    LightUpdateState lightState;
    unsigned prevNumLights = 0;
    int lightsDirty = 0;
    DBuf<int> lightRemap;
    // two-level BVH of the instanced meshes (meshes.hip): BLAS per block type, TLAS per world
    std::vector<BvhNode> hBlas;
    std::vector<float> hBlasTri;
    std::vector<int> hBlasTriId;
    std::vector<int2> hRoot;  // per block type: (first node, first triangle), -1 = no mesh
    DBuf<BvhNode> blas, tlas;
    DBuf<float> blasTri;
    DBuf<int> blasTriId;
    DBuf<int2> blasRoot;
    DBuf<MeshInst> meshInst;
    int nMeshInst = 0;
    // the path kernels' view of the meshes: texcoords in BLAS leaf order, per instance row its cell +
    // block and first light, materials by block id
    std::vector<float> hBlasUV;
    DBuf<float> blasUV;
    DBuf<int4> meshRow;
    DBuf<int> meshRowLight;
    DBuf<MatDev> meshMats;
    MatDev meshMatsUp[32] = {};  // what meshMats holds (uploaded when the materials change)
    // vxpt_mesh_probe / vxpt_mesh_occluded scratch (grown to the largest call)
    DBuf<float> probeRays, probeOut;
    DBuf<int> probeIds;
    DBuf<unsigned char> probeOcc;

    // blue noise
    DBuf<uint8_t> bnSobol, bnScramble, bnRank;

    // frame buffers
    // G-buffer ring of 3 slots: every trace pass writes a slot that is neither
    // the previous pass's (its ReSTIR history) nor the denoiser's history slot
    // (the previous frame's final G-buffer, Denoiser.cu:394-407), so the frame
    // end hands the last slot to the denoiser by index instead of copying planes.
    // Two more slots let first halves (camera rays .. NEE visibility, which read no previous pass)
    // run ahead while up to two second halves still read their previous passes' slots, and one more
    // keeps the denoiser's previous history slot (histOld) out of the pipelined next frame's reach.
    GSlot gb[6];
    int last = 0;              // slot of the most recent trace output
    int tracePrev = 0;         // slot the most recent trace read as its previous pass
    int tracePrev2 = 0;        // the one before (read by the second half before that)
    int hist = 2;              // denoiser history slot (zero at frame 0)
    int histOld = 2;           // the one before (the history of the most recently enqueued denoiser run)
    float4 *illum = nullptr;   // the most recent pass's radiance (one of illumSet)
    float4 *illumSet[kMaxSets] = {};  // per wavefront state set
    float4 *accum = nullptr, *motion = nullptr;
    float4 *accumBuf[2] = {};  // accum alternates between these per accumulation (first pass picks the other)
    // the motion plane holds only zeros (allocated zeroed; the trace stores zeros, the world is static)
    // until a host write: the trace then skips its zero stores
    bool motionZero = true;
    Reservoir *res = nullptr;  // 2*W*H
    float4 *ping = nullptr, *pong = nullptr, *prevIllum = nullptr, *prevFast = nullptr, *output = nullptr;
    float *clampDbg = nullptr;  // vxpt_debug_clamp_decisions (written while clampDbgOn)
    bool clampDbgOn = false;
    float *histLen = nullptr, *prevHistLen = nullptr;
    float4 *wpos = nullptr;
    uint32_t *ffCount = nullptr, *ffIndex = nullptr, *hfList = nullptr, *hfCount = nullptr, *ffCandCount = nullptr;
    uint4 *ffCand = nullptr;
    float4 *ffColor = nullptr;
    Reservoir *ffRes = nullptr;
    bool denoiseInputIsAccum = false;
    // Wavefront state sets, used round-robin by pass: first halves (k_closest .. the RIS
    // visibility rays) run in order on frontStream, each after the pass that last used its set;
    // second halves (temporal reuse, its rays, k_finish, later segments, the spp accumulation) run
    // in order on the context stream, each after its first half.  With 3 sets a first half may
    // start while the two previous second halves are still running.
    int nSets = 2;
    WaveBufs wb[kMaxSets]{};
    size_t wbSlots[kMaxSets] = {};
    int passCount = 0;         // trace passes so far (set = passCount % nSets)
    int lastSet = 0;           // the set of the most recent pass
    // first halves: on front_streams streams by state set (set % front_streams), so a first half may run
    // beside the previous passes' first halves (it reads nothing a first half writes: the waits on
    // backDone order it behind its set's last user only)
    hipStream_t frontStreams[kMaxSets] = {};
    hipEvent_t frontDone[kMaxSets] = {}, backDone[kMaxSets] = {}, frontGate = nullptr;
    std::vector<hipEvent_t> chainEv;  // vxpt_render_frames: around each frame's denoiser chain
    int numCU = 256;
    std::vector<void *> allocs;

    // post-processing (PostProcessor / PostProcessingPipeline): working, bloom and frame
    // planes, luminance histogram, device exposure state
    vxpt_post_params yamlPost{};
    float4 *bloomA = nullptr, *bloomB = nullptr, *frame = nullptr;
    unsigned *postHist = nullptr;
    float *postState = nullptr;
    float sunLuminance = 1.0f;     // SkyModel::getAccumulatedSunLuminance: the sun map's total pdf

    vxpt_denoise_params yamlDenoise{};
    float skyParams[4] = {0.25f, 45.0f, 0.0f, 1.0f};
    vxpt_material yamlMats[13] = {};

    // band partition (multi-GPU): this context's rank among nranks bands and the
    // transport its halo rows move by -- an RCCL communicator (one process per
    // GPU) or the other contexts of this process (vxpt_band_link)
    int nranks = 1, rank = 0;
    std::vector<int> splits;  // nranks + 1 band boundaries (row_splits, or the equal bands)
    ncclComm_t comm = nullptr;
    std::vector<vxpt_ctx *> linked;
    // the trace-halo exchange runs on its own stream, overlapped with the next
    // pass up to its temporal-reuse kernel (haloDone: recorded after the exchange)
    hipStream_t commStream = nullptr;
    hipEvent_t haloReady = nullptr, haloDone = nullptr;
    // exDone: after the last exchange in stream order; the exchange stream's next group waits for it,
    // and an exchange in stream order waits for an exchange-stream group still pending (haloDone):
    // the communicator's groups run one after another, in the order every rank issues them
    hipEvent_t exDone = nullptr;
    bool exDoneRec = false;
    // vxpt_band_stats collection: timing events from a pool bracketing each exchange group (kind 0 on
    // the context stream, 1 on the exchange stream) and each banded frame's trace (2) and denoiser (3)
    // spans, and the bytes sent to each neighbour.  Completed spans are folded into `ms` and their
    // events reused (stat_fold: at every sync of a banded run, and before a frame once the pool holds
    // kStatPoolFold events), so a long collection keeps a bounded pool.
    struct BandStat {
        bool on = false;
        std::vector<hipEvent_t> pool;
        size_t used = 0;
        struct Span { size_t e0, e1; int kind; };
        std::vector<Span> spans;
        double ms[4] = {};
        int frames = 0, groups = 0, groupsOrdered = 0;
        double up = 0.0, down = 0.0;
    } bst;
    // halo depths the last banded frame exchanged: tap records + reservoirs, histories, G-buffer planes
    int haloTraceRows = 72, haloHistRows = 2, haloPlaneRows = 40;
    bool haloPending = false;
};

namespace {

int fail(vxpt_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}
#define HIPCHK(c, expr)                                                                          \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) return fail((c), VXPT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class T>
int dalloc(vxpt_ctx *c, T *&p, size_t n) {
    void *q = nullptr;
    HIPCHK(c, hipMalloc(&q, n * sizeof(T) + 16));
    HIPCHK(c, hipMemsetAsync(q, 0, n * sizeof(T) + 16, c->stream));  // same stream as every upload
    c->allocs.push_back(q);
    p = (T *)q;
    return 0;
}

bool read_file(const std::string &p, std::vector<uint8_t> &out) {
    std::ifstream f(p, std::ios::binary);
    if (!f) return false;
    out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return true;
}

template <class T>
int grow(vxpt_ctx *c, DBuf<T> &d, size_t n) {
    if (d.n >= n) return 0;
    if (dalloc(c, d.p, n)) return 1;
    d.n = n;
    return 0;
}

template <class T>
int upload_vec(vxpt_ctx *c, DBuf<T> &d, const T *h, size_t n) {
    if (d.n < n) {
        if (dalloc(c, d.p, n)) return VXPT_ERR_HIP;
        d.n = n;
    }
    HIPCHK(c, hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
    return 0;
}

// Camera set-up exactly as mainOffline.cpp:227-246 + Camera::update (Camera.h:44-100)
V3 yaw_pitch_to_dir(float yaw, float pitch) {
    if (std::isnan(yaw) || std::isnan(pitch)) return {0, 0, 1};
    pitch = clampf(pitch, -kPiOver2 + 0.01f, kPiOver2 - 0.01f);
    const float sy = std::sin(yaw), cyw = std::cos(yaw), sp = std::sin(pitch), cp = std::cos(pitch);
    return normalize(V3(sy * cp, sp, cyw * cp));
}
CamDev make_camera_angles(int W, int H, const float pos[3], float yaw, float pitch, float fovDeg) {
    CamDev c{};
    c.res = V2((float)W, (float)H);
    c.invRes = V2(1.0f / c.res.x, 1.0f / c.res.y);
    c.pos = V3(pos[0], pos[1], pos[2]);
    const float fovX = fovDeg * kPiOver180;
    const float fovY = fovX * (c.res.y / c.res.x);
    c.tanHalfFov = V2(std::tan(fovX * 0.5f), std::tan(fovY * 0.5f));
    c.dir = yaw_pitch_to_dir(yaw, pitch);
    const V3 worldUp(0.0f, 1.0f, 0.0f);
    const V3 left = normalize(cross(worldUp, c.dir));
    const V3 up = normalize(cross(c.dir, left));
    const M3 uvToNdc = m3_cols(V3(2.0f, 0.0f, 0.0f), V3(0.0f, 2.0f, 0.0f), V3(-1.0f, -1.0f, 1.0f));
    M3 ndcToView = m3_zero();
    ndcToView.m00 = c.tanHalfFov.x;
    ndcToView.m11 = c.tanHalfFov.y;
    ndcToView.m22 = 1.0f;
    const M3 viewToWorld = m3_cols(-left, up, c.dir);
    c.uvToWorld = m3_mul(m3_mul(viewToWorld, ndcToView), uvToNdc);
    const M3 ndcToUv = m3_cols(V3(0.5f, 0.0f, 0.0f), V3(0.0f, 0.5f, 0.0f), V3(0.5f, 0.5f, 1.0f));
    const M3 worldToView = m3_transpose(viewToWorld);
    M3 viewToNdc = m3_zero();
    viewToNdc.m00 = 1.0f / c.tanHalfFov.x;
    viewToNdc.m11 = 1.0f / c.tanHalfFov.y;
    viewToNdc.m22 = 1.0f;
    c.worldToUv = m3_mul(m3_mul(ndcToUv, viewToNdc), worldToView);
    return c;
}
// the scene's direction -> yaw/pitch (DirToYawPitch) -> Camera::update
CamDev make_camera(int W, int H, const vxpt_camera &in, float *yawOut, float *pitchOut) {
    const V3 d = normalized_c(normalize(V3(in.dir[0], in.dir[1], in.dir[2])));
    const float yaw = std::atan2(d.x, d.z), pitch = std::asin(d.y);
    if (yawOut) *yawOut = yaw;
    if (pitchOut) *pitchOut = pitch;
    return make_camera_angles(W, H, in.pos, yaw, pitch, in.fov_deg);
}

std::vector<AliasBin> build_alias(const std::vector<float> &w, float &sumOut) {
    const unsigned n = (unsigned)w.size();
    double acc = 0.0;
    for (unsigned i = 0; i < n; ++i) acc += (double)w[i];
    const float sum = (float)acc;
    sumOut = sum;
    std::vector<float> prob(n), scaled(n);
    std::vector<int> alias(n, -1);
    for (unsigned i = 0; i < n; ++i) {
        prob[i] = w[i] / sum;
        scaled[i] = prob[i] * n;
    }
    std::queue<int> small, large;
    for (unsigned i = 0; i < n; ++i) (scaled[i] < 1.0f ? small : large).push((int)i);
    while (!small.empty() && !large.empty()) {
        const int s = small.front(); small.pop();
        const int l = large.front(); large.pop();
        alias[s] = l;
        scaled[l] -= (1.0f - scaled[s]);
        (scaled[l] < 1.0f ? small : large).push(l);
    }
    while (!small.empty()) { scaled[small.front()] = 1.0f; small.pop(); }
    while (!large.empty()) { scaled[large.front()] = 1.0f; large.pop(); }
    std::vector<AliasBin> b(n);
    for (unsigned i = 0; i < n; ++i) b[i] = {scaled[i], prob[i], alias[i]};
    return b;
}

float fit6(const float *M, float t, int i, int stride) {  // Sky.cu:19-47
    return (std::pow(1.0f - t, 5.0f) * M[i] + 5.0f * std::pow(1.0f - t, 4.0f) * t * M[i + stride] +
            10.0f * std::pow(1.0f - t, 3.0f) * std::pow(t, 2.0f) * M[i + 2 * stride] +
            10.0f * std::pow(1.0f - t, 2.0f) * std::pow(t, 3.0f) * M[i + 3 * stride] +
            5.0f * (1.0f - t) * std::pow(t, 4.0f) * M[i + 4 * stride] + std::pow(t, 5.0f) * M[i + 5 * stride]);
}

V3 q_rotate3(V3 axis, float angle, V3 v) {  // rotate3f (LinearMath.h:1368)
    const Qt q{normalized_c(axis) * std::sin(angle / 2), std::cos(angle / 2)};
    return q_mul(q_mul(q, {v, 0.f}), q_conj(q)).v;
}

void fill_world(vxpt_ctx *c, WorldDev &w) {
    w.ids = c->voxels.p;
    w.bricks = c->bricks.p;
    w.macro = c->macro.p;
    w.cellMask = c->cellMask.p;
    w.bdist = c->bdist.p;
    w.bbox = c->useBoxes ? c->bbox.p : nullptr;
    w.nBricks = c->nBricks;
    // a brick walk yields its lanes back to the outer loop after brick_steps (3) crossings (fewer lanes
    // idle behind long in-brick walks; C3 trace 6.44 -> 6.26 ms per frame)
    w.brickSteps = c->tune.brick_steps;
    w.brickStepsCam = c->tune.cam_steps;
    w.top = c->top;
    w.topValid = c->topValid;
    w.skyTop = c->tune.sky_exit ? c->skyTop.p : nullptr;
    w.cx = c->cx; w.cy = c->cy; w.cz = c->cz;
    w.wx = c->cx * 32; w.wy = c->cy * 32; w.wz = c->cz * 32;
    w.mx = w.wx / 16; w.my = w.wy / 16; w.mz = w.wz / 16;
    w.tx = (w.wx + 63) / 64; w.ty = (w.wy + 63) / 64; w.tz = (w.wz + 63) / 64;
}

void fill_sky(vxpt_ctx *c, SkyDev &s) {
    s.sky = c->sky.p;
    s.sun = c->sun.p;
    s.skyAlias = c->skyAlias.p;
    s.sunAlias = c->sunAlias.p;
    s.sunDir = c->sunDir;
    s.skyW = 1024; s.skyH = 512; s.sunW = 32; s.sunH = 32;
    s.sunCosMax = std::cos(0.51f * kPi / 180.0f / 2.0f);
}

void fill_denoise(vxpt_ctx *c, const vxpt_denoise_params *p, DenoiseArgs &a, int parity) {
    a.W = c->W; a.H = c->H;
    a.y0 = c->rowBegin; a.y1 = c->rowEnd;
    a.cam = c->cam; a.prevCam = c->prevCam;
    a.p = {p->max_accumulated_frame_num, p->max_fast_accumulated_frame_num, p->phi_luminance,
           p->lobe_angle_fraction, p->roughness_fraction, p->depth_threshold, p->disocclusion_threshold,
           p->disocclusion_threshold_alternate, p->denoising_range, p->enable_temporal_accumulation,
           p->enable_history_fix, p->enable_history_clamping, p->enable_spatial_filtering,
           p->enable_firefly_filter, p->atrous_iteration_num};
    const GSlot &g = c->gb[c->last];
    a.illum = c->denoiseInputIsAccum ? c->accum : c->illum;
    a.normalRough = g.normalRough;
    a.albedo = g.albedo;
    a.motion = c->motion;
    a.depth = g.depth;
    a.material = g.material;
    a.prevNormalRough = c->gb[c->hist].normalRough;
    a.prevDepth = c->gb[c->hist].depth;
    a.reservoir = c->res + (size_t)parity * c->W * c->H;
    a.ping = c->ping; a.pong = c->pong; a.prevIllum = c->prevIllum; a.prevFast = c->prevFast;
    a.output = c->output;
    a.histLen = c->histLen; a.prevHistLen = c->prevHistLen;
    a.ffCount = c->ffCount; a.ffIndex = c->ffIndex; a.ffColor = c->ffColor; a.ffRes = c->ffRes;
    a.ffCand = c->ffCand; a.ffCandCount = c->ffCandCount;
    a.hfList = c->hfList; a.hfCount = c->hfCount;
    a.wpos = c->wpos;
    a.clampDbg = c->clampDbgOn ? c->clampDbg : nullptr;
    a.invW = 1.0f / (float)c->W; a.invH = 1.0f / (float)c->H;
    a.thrB = a.p.disocclusionThreshold + (1.5f / (float)c->H);
    a.thrA = a.p.disocclusionThresholdAlternate + (1.5f / (float)c->H);
    a.frustumK = c->cam.tanHalfFov.x / (c->cam.res.x / 2);
    a.invAcc1 = 1.0f / (a.p.maxAcc + 1.0f);
    a.invFast1 = 1.0f / (a.p.maxFast + 1.0f);
    a.tune.ffFused = c->tune.firefly_fused;
    a.tune.taSupertiles = c->tune.ta_supertiles;
    a.tune.hfSplit = c->tune.hf_split;
    a.tune.stencilTile = c->tune.stencil_tile;
}

// GlobalSettings.h:10-186 defaults (the reference yaml overrides most of them: vxpt_load_settings)
vxpt_post_params default_post() {
    vxpt_post_params p{};
    p.manual_exposure = 10.0f; p.tone_mapping_curve = 0; p.white_point = 10.0f;
    p.contrast = 1.0f; p.saturation = 1.0f; p.lift = 0.0f; p.gain = 1.0f;
    p.enable_bloom = 1; p.bloom_threshold = 1.0f; p.bloom_intensity = 0.15f; p.bloom_radius = 2.0f;
    p.enable_auto_exposure = 1; p.exposure_speed = 1.0f; p.exposure_min = -8.0f; p.exposure_max = 8.0f;
    p.exposure_compensation = 0.0f; p.histogram_min_percent = 40.0f; p.histogram_max_percent = 80.0f;
    p.target_luminance = 0.18f;
    p.enable_vignette = 0; p.vignette_strength = 0.5f; p.vignette_radius = 0.8f; p.vignette_smoothness = 0.5f;
    p.enable_lens_flare = 0; p.lens_flare_intensity = 0.00001f; p.lens_flare_ghost_spacing = 0.15f;
    p.lens_flare_ghost_count = 4; p.lens_flare_halo_radius = 0.1f; p.lens_flare_sun_size = 0.006f;
    p.lens_flare_distortion = 0.015f;
    p.draw_crosshair = 1;
    return p;
}

const vxpt_denoise_params &default_denoise() {
    static vxpt_denoise_params d{30.f, 6.f, 2.f, 0.5f, 0.15f, 0.003f, 0.01f, 0.05f, 500000.f, 1, 1, 1, 1, 1, 1};
    return d;
}

// pointer + byte size of a logical buffer
bool buffer_ptr(vxpt_ctx *c, int which, void *&p, size_t &bytes, bool forWrite, void **mirror) {
    const size_t n = (size_t)c->W * c->H;
    // current = the slot the last trace wrote; PREV_GEO_NORMAL_THIN / ALBEDO /
    // MAT_PARAM = the slot it read as the previous pass (ReSTIR history);
    // PREV_NORMAL_ROUGH / DEPTH / MATERIAL = the denoiser's history slot
    const GSlot &g = c->gb[c->last];
    const GSlot &gp = c->gb[c->tracePrev];
    const GSlot &gh = c->gb[c->hist];
    *mirror = nullptr;
    switch (which) {
        case VXPT_BUF_ILLUM: p = c->denoiseInputIsAccum ? c->accum : c->illum; bytes = n * 16; return true;
        case VXPT_BUF_DEPTH: p = g.depth; bytes = n * 4; return true;
        case VXPT_BUF_NORMAL_ROUGH: p = g.normalRough; bytes = n * 16; return true;
        case VXPT_BUF_GEO_NORMAL_THIN: p = g.geoNormalThin; bytes = n * 16; return true;
        case VXPT_BUF_PREV_GEO_NORMAL_THIN: p = gp.geoNormalThin; bytes = n * 16; return true;
        case VXPT_BUF_ALBEDO: p = g.albedo; bytes = n * 16; return true;
        case VXPT_BUF_PREV_ALBEDO: p = gp.albedo; bytes = n * 16; return true;
        case VXPT_BUF_MATERIAL: p = g.material; bytes = n * 4; return true;
        case VXPT_BUF_MAT_PARAM: p = g.matParam; bytes = n * 16; return true;
        case VXPT_BUF_PREV_MAT_PARAM: p = gp.matParam; bytes = n * 16; return true;
        case VXPT_BUF_MOTION: p = c->motion; bytes = n * 16; return true;
        case VXPT_BUF_PREV_NORMAL_ROUGH: p = gh.normalRough; bytes = n * 16; return true;
        case VXPT_BUF_PREV_DEPTH: p = gh.depth; bytes = n * 4; return true;
        case VXPT_BUF_PREV_MATERIAL: p = gh.material; bytes = n * 4; return true;
        case VXPT_BUF_RESERVOIRS: p = c->res; bytes = 2 * n * sizeof(Reservoir); return true;
        case VXPT_BUF_RES_EVEN: p = c->res; bytes = n * sizeof(Reservoir); return true;
        case VXPT_BUF_RES_ODD: p = c->res + n; bytes = n * sizeof(Reservoir); return true;
        case VXPT_BUF_WPOS: p = c->wpos; bytes = n * 16; return true;
        case VXPT_BUF_FRAME: p = c->frame; bytes = n * 16; return c->frame != nullptr;
        case VXPT_BUF_PING: p = c->ping; bytes = n * 16; return true;
        case VXPT_BUF_PONG: p = c->pong; bytes = n * 16; return true;
        case VXPT_BUF_PREV_ILLUM: p = c->prevIllum; bytes = n * 16; return true;
        case VXPT_BUF_PREV_FAST: p = c->prevFast; bytes = n * 16; return true;
        case VXPT_BUF_HIST_LEN: p = c->histLen; bytes = n * 4; return true;
        case VXPT_BUF_PREV_HIST_LEN: p = c->prevHistLen; bytes = n * 4; return true;
        case VXPT_BUF_OUTPUT: p = c->output; bytes = n * 16; return true;
        case VXPT_BUF_SKY: p = c->sky.p; bytes = 1024 * 512 * 16; return c->sky.p != nullptr;
        case VXPT_BUF_SUN: p = c->sun.p; bytes = 32 * 32 * 16; return c->sun.p != nullptr;
        case VXPT_BUF_VOXELS: p = c->voxels.p; bytes = (size_t)c->cx * c->cy * c->cz * 32768; return c->voxels.p != nullptr;
        case VXPT_BUF_OCTANT_TABLES: p = c->bdist.p; bytes = (size_t)8 * c->nBricks; return !forWrite && c->bdist.p;
        case VXPT_BUF_CELL_MASKS: p = c->cellMask.p; bytes = (size_t)c->nBricks * 8; return !forWrite && c->cellMask.p;
        case VXPT_BUF_BRICK_IDS: p = c->bricks.p; bytes = (size_t)c->nBricks * 64; return !forWrite && c->bricks.p;
        case VXPT_BUF_MACRO_MASKS: p = c->macro.p; bytes = (size_t)c->nBricks / 64 * 8; return !forWrite && c->macro.p;
        case VXPT_BUF_TEXELS: p = c->texels.p; bytes = c->nTexels * 4; return !forWrite && c->texels.p;
        case VXPT_BUF_BLOOM: p = c->bloomB; bytes = n * 16; return c->bloomB != nullptr;
        case VXPT_BUF_LIGHTS: p = c->lights.p; bytes = (size_t)c->nLights * sizeof(LightInfo); return !forWrite && c->nLights;
        case VXPT_BUF_TAP_RECORD: p = g.rec; bytes = n * 32; return !forWrite;
        case VXPT_BUF_CLAMP_DECISION: p = c->clampDbg; bytes = n * 4; return !forWrite && p;
        case VXPT_BUF_BOX_TABLES: p = c->bbox.p; bytes = (size_t)8 * c->nBricks * 4; return !forWrite && c->bbox.p;
        case VXPT_BUF_LIGHT_ALIAS:
            p = c->lightAlias.p; bytes = (size_t)c->nLights * sizeof(AliasBin); return !forWrite && c->nLights;
        default: return false;
    }
}

// brick coordinates (4^3 cells) -> cellMask / octant-table index (16^3 macro cell m, brick lb)
inline size_t brick_lin(const vxpt_ctx *c, int bx, int by, int bz) {
    const size_t m = (size_t)(bx >> 2) + (size_t)(c->cx * 2) * ((bz >> 2) + (size_t)(c->cz * 2) * (by >> 2));
    return m * 64 + (size_t)((bx & 3) + 4 * ((bz & 3) + 4 * (by & 3)));
}
inline bool is_cube(int id) { return id >= 1 && id <= 12; }

// Per-octant empty-box sizes: for every 4^3 brick and each of the 8 ray octants,
// S = the edge (in bricks) of the largest brick-aligned cube with that brick at its
// corner, extending in the octant's directions, that holds no cube cell (0 = the
// brick is occupied; out-of-world counts as empty; capped at 255).  A ray in that
// octant can leave the whole cube in one jump.  3-D "largest empty square"
// recurrence S = 1 + min(S of the 7 forward neighbours), evaluated over the brick box
// [x0,x1] x [y0,y1] x [z0,z1] against the octant's direction; bricks outside the box
// keep their values (an edit recomputes only the bricks behind it).
void octant_fill(vxpt_ctx *c, int oct, int x0, int x1, int y0, int y1, int z0, int z1) {
    const int BX = c->cx * 8, BY = c->cy * 8, BZ = c->cz * 8;
    const size_t nB = (size_t)BX * BY * BZ;
    uint8_t *S = c->hOd.data() + (size_t)oct * nB;
    const int sx = (oct & 1) ? 1 : -1, sy = (oct & 2) ? 1 : -1, sz = (oct & 4) ? 1 : -1;
    auto get = [&](int x, int y, int z) -> int {
        if (x < 0 || y < 0 || z < 0 || x >= BX || y >= BY || z >= BZ) return 255;
        return S[brick_lin(c, x, y, z)];
    };
    for (int iy = 0; iy <= y1 - y0; ++iy)
        for (int iz = 0; iz <= z1 - z0; ++iz)
            for (int ix = 0; ix <= x1 - x0; ++ix) {
                const int x = sx > 0 ? x1 - ix : x0 + ix, y = sy > 0 ? y1 - iy : y0 + iy, z = sz > 0 ? z1 - iz : z0 + iz;
                const size_t b = brick_lin(c, x, y, z);
                int v = 0;
                if (!c->hCell[b]) {
                    int mn = 255;
                    for (int k = 1; k < 8; ++k)
                        mn = std::min(mn, get(x + ((k & 1) ? sx : 0), y + ((k & 2) ? sy : 0), z + ((k & 4) ? sz : 0)));
                    v = std::min(255, 1 + mn);
                }
                S[b] = (uint8_t)v;
            }
}

// the box tables over brick box [x0,x1] x [y0,y1] x [z0,z1] of octant oct, from the cube tables and
// the occupancy prefix counts (both current)
void box_fill(vxpt_ctx *c, int oct, int x0, int x1, int y0, int y1, int z0, int z1) {
    const int boxCap = c->boxCap, boxCapUp = c->boxCapUp;
    const size_t nB = (size_t)c->cx * 8 * c->cy * 8 * c->cz * 8;
    for (int y = y0; y <= y1; ++y)
        for (int z = z0; z <= z1; ++z)
            for (int x = x0; x <= x1; ++x) {
                const size_t b = brick_lin(c, x, y, z);
                c->hBox[oct * nB + b] = grow_box(c->brickPrefix, x, y, z, oct, c->hOd[oct * nB + b], boxCap, boxCapUp);
            }
}
void brick_prefix(vxpt_ctx *c) {
    c->brickPrefix.build(c->cx * 8, c->cy * 8, c->cz * 8,
                         [&](int x, int y, int z) { return c->hCell[brick_lin(c, x, y, z)] != 0; });
}

inline int top_block(const vxpt_ctx *c, int x, int y, int z) {
    const int tx = (c->cx * 32 + 63) / 64, tz = (c->cz * 32 + 63) / 64;
    return (x >> 6) + tx * ((z >> 6) + tz * (y >> 6));
}
void refresh_top(vxpt_ctx *c) {
    c->top = 0;
    for (size_t t = 0; t < c->topCount.size() && t < 64; ++t)
        if (c->topCount[t]) c->top |= 1ull << t;
}

// DDA acceleration layout (WorldDev) from chunk-major ids, built in the host mirrors and uploaded
// the sky exit's table: for each x / z direction quadrant q ((dx > 0) | (dz > 0) << 1) and brick column,
// the highest 1 + cube row over the columns a walk in that quadrant can still reach (x, z not moving
// against the ray: a suffix maximum along each axis), uploaded on the context stream
int upload_sky_top(vxpt_ctx *c) {
    const int nbx = c->cx * 8, nbz = c->cz * 8;
    c->hSkyTop.assign((size_t)4 * nbx * nbz, 0);
    for (int q = 0; q < 4; ++q) {
        const bool px = q & 1, pz = q & 2;
        uint16_t *t = c->hSkyTop.data() + (size_t)q * nbx * nbz;
        for (int kz = 0; kz < nbz; ++kz)
            for (int kx = 0; kx < nbx; ++kx) {
                // walk the columns from the far corner of the quadrant towards its origin
                const int bz = pz ? nbz - 1 - kz : kz, bx = px ? nbx - 1 - kx : kx;
                const int fz = pz ? bz + 1 : bz - 1, fx = px ? bx + 1 : bx - 1;  // the next column along z / x
                uint16_t m = c->colTop[(size_t)bz * nbx + bx];
                if (fz >= 0 && fz < nbz) m = std::max(m, t[(size_t)fz * nbx + bx]);
                if (fx >= 0 && fx < nbx) m = std::max(m, t[(size_t)bz * nbx + fx]);
                t[(size_t)bz * nbx + bx] = m;
            }
    }
    return upload_vec(c, c->skyTop, c->hSkyTop.data(), c->hSkyTop.size());
}

int build_occupancy(vxpt_ctx *c, const uint8_t *ids) {
    const int wx = c->cx * 32, wy = c->cy * 32, wz = c->cz * 32;
    const int mx = wx / 16, my = wy / 16, mz = wz / 16;
    c->hMacro.assign((size_t)mx * my * mz, 0ull);
    c->hBricks.assign((size_t)wx * wy * wz, 0);
    c->hCell.assign((size_t)mx * my * mz * 64, 0ull);
    const int tx = (wx + 63) / 64, ty = (wy + 63) / 64, tz = (wz + 63) / 64;
    c->topCount.assign((size_t)tx * ty * tz, 0);
    c->hNonAir.assign((size_t)mx * my * mz * 64, 0);
    c->colTop.assign((size_t)(wx >> 2) * (wz >> 2), 0);
    for (int y = 0; y < wy; ++y)
        for (int z = 0; z < wz; ++z)
            for (int x = 0; x < wx; ++x) {
                const int ch = (x >> 5) + c->cx * ((z >> 5) + c->cz * (y >> 5));
                const uint8_t id = ids[(size_t)ch * 32768 + (x & 31) + 32 * ((z & 31) + 32 * (y & 31))];
                if (!id) continue;
                const size_t b = brick_lin(c, x >> 2, y >> 2, z >> 2);
                const int lc = (x & 3) + 4 * ((z & 3) + 4 * (y & 3));
                c->hBricks[b * 64 + lc] = id;
                c->hNonAir[b]++;
                // only cube ids (1..12) make a brick visible to the DDA; other ids are empty for it
                if (is_cube(id)) {
                    c->hMacro[b / 64] |= 1ull << (b % 64);
                    c->hCell[b] |= 1ull << lc;
                    c->topCount[top_block(c, x, y, z)]++;
                    uint16_t &ct = c->colTop[(size_t)(z >> 2) * (wx >> 2) + (x >> 2)];
                    ct = std::max<uint16_t>(ct, (uint16_t)(y + 1));
                }
            }
    c->topValid = (tx * ty * tz <= 64) ? 1 : 0;
    refresh_top(c);
    if (int r = upload_sky_top(c)) return r;
    const int BX = wx / 4, BY = wy / 4, BZ = wz / 4;
    const size_t nB = (size_t)BX * BY * BZ;
    c->hOd.assign(8 * nB, 0);
    for (int oct = 0; oct < 8; ++oct) octant_fill(c, oct, 0, BX - 1, 0, BY - 1, 0, BZ - 1);
    c->nBricks = (int)nB;
    if (int r = upload_vec(c, c->bdist, c->hOd.data(), c->hOd.size())) return r;
    if (c->useBoxes) {
        brick_prefix(c);
        c->hBox.assign(8 * nB, 0u);
        for (int oct = 0; oct < 8; ++oct) box_fill(c, oct, 0, BX - 1, 0, BY - 1, 0, BZ - 1);
        if (int r = upload_vec(c, c->bbox, c->hBox.data(), c->hBox.size())) return r;
    }
    if (int r = upload_vec(c, c->bricks, c->hBricks.data(), c->hBricks.size())) return r;
    if (int r = upload_vec(c, c->macro, c->hMacro.data(), c->hMacro.size())) return r;
    if (int r = upload_vec(c, c->cellMask, c->hCell.data(), c->hCell.size())) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

// One voxel edit (VoxelEngine::setVoxelAtGlobal, VoxelEngine.cu:265-276, and the uninstanced
// face-mesh update updateSingleVoxelGlobal, VoxelSceneGen.cu:643-786, whose DDA equivalent is
// this): the id in both layouts, the brick's cube mask, and -- when the brick turns occupied or
// empty -- its macro bit, the 64^3 block bit and the octant tables of the bricks behind it.
int set_block(vxpt_ctx *c, int x, int y, int z, int id) {
    const int wx = c->cx * 32, wy = c->cy * 32, wz = c->cz * 32;
    if (x < 0 || y < 0 || z < 0 || x >= wx || y >= wy || z >= wz || id < 0 || id > 255)
        return fail(c, VXPT_ERR_ARG, "block position or id out of range");
    const size_t ci = (size_t)((x >> 5) + c->cx * ((z >> 5) + c->cz * (y >> 5))) * 32768 + (x & 31) +
                      32 * ((z & 31) + 32 * (y & 31));
    const int old = c->hIds[ci];
    if (old == id) return 0;
    hipStream_t st = c->stream;
    c->hIds[ci] = (uint8_t)id;
    ++c->worldVersion;
    HIPCHK(c, hipMemcpyAsync(c->voxels.p + ci, &c->hIds[ci], 1, hipMemcpyHostToDevice, st));
    const size_t b = brick_lin(c, x >> 2, y >> 2, z >> 2);
    const int lc = (x & 3) + 4 * ((z & 3) + 4 * (y & 3));
    c->hBricks[b * 64 + lc] = (uint8_t)id;
    c->hNonAir[b] += (id != 0 ? 1 : 0) - (old != 0 ? 1 : 0);
    HIPCHK(c, hipMemcpyAsync(c->bricks.p + b * 64 + lc, &c->hBricks[b * 64 + lc], 1, hipMemcpyHostToDevice, st));
    if (is_cube(old) != is_cube(id)) {
        const uint64_t before = c->hCell[b];
        c->hCell[b] = is_cube(id) ? (before | (1ull << lc)) : (before & ~(1ull << lc));
        HIPCHK(c, hipMemcpyAsync(c->cellMask.p + b, &c->hCell[b], 8, hipMemcpyHostToDevice, st));
        c->topCount[top_block(c, x, y, z)] += is_cube(id) ? 1 : -1;
        refresh_top(c);
        if (is_cube(id) && c->colTop[(size_t)(z >> 2) * (wx >> 2) + (x >> 2)] < y + 1) {
            c->colTop[(size_t)(z >> 2) * (wx >> 2) + (x >> 2)] = (uint16_t)(y + 1);
            if (int r = upload_sky_top(c)) return r;
        }
        if ((before != 0) != (c->hCell[b] != 0)) {
            const size_t m = b / 64;
            c->hMacro[m] = c->hCell[b] ? (c->hMacro[m] | (1ull << (b % 64))) : (c->hMacro[m] & ~(1ull << (b % 64)));
            HIPCHK(c, hipMemcpyAsync(c->macro.p + m, &c->hMacro[m], 8, hipMemcpyHostToDevice, st));
            const int bx = x >> 2, by = y >> 2, bz = z >> 2, BX = c->cx * 8, BY = c->cy * 8, BZ = c->cz * 8;
            for (int oct = 0; oct < 8; ++oct)
                octant_fill(c, oct, (oct & 1) ? 0 : bx, (oct & 1) ? bx : BX - 1, (oct & 2) ? 0 : by,
                            (oct & 2) ? by : BY - 1, (oct & 4) ? 0 : bz, (oct & 4) ? bz : BZ - 1);
            HIPCHK(c, hipMemcpyAsync(c->bdist.p, c->hOd.data(), c->hOd.size(), hipMemcpyHostToDevice, st));
            if (c->useBoxes) {  // the boxes that could reach the brick: the same bricks behind it
                brick_prefix(c);
                for (int oct = 0; oct < 8; ++oct)
                    box_fill(c, oct, (oct & 1) ? 0 : bx, (oct & 1) ? bx : BX - 1, (oct & 2) ? 0 : by,
                             (oct & 2) ? by : BY - 1, (oct & 4) ? 0 : bz, (oct & 4) ? bz : BZ - 1);
                HIPCHK(c, hipMemcpyAsync(c->bbox.p, c->hBox.data(), c->hBox.size() * 4, hipMemcpyHostToDevice, st));
            }
        }
    }
    // the mirrors are the copies' sources: let them land before the host edits them again
    HIPCHK(c, hipStreamSynchronize(st));
    // OptixRenderer::update (:916-919): after a geometry change the previous frame's scene is
    // gone, so the next pass's ReSTIR temporal visibility rays (closesthit.cu:736-755) miss
    c->prevSceneEmpty = 1;
    return 0;
}

}  // namespace
static MeshDev mesh_dev(const vxpt_ctx *c);
namespace {

// wavefront trace state of one set for ns slots (8x8 tiles of the band), 4 visibility rays per slot;
// allocated at the first pass that needs it (a band context holds its band's slots only).  The
// allocation's zero fill is enqueued on the context stream: `fresh` tells the caller
int ensure_wave(vxpt_ctx *c, int set, size_t ns, bool &fresh) {
    fresh = false;
    if (c->wbSlots[set] >= ns) return 0;
    fresh = true;
    WaveBufs &w = c->wb[set];
    w = WaveBufs{};  // a smaller earlier set stays allocated (freed with the context)
    if (dalloc(c, w.pPos, ns) || dalloc(c, w.pDir, ns) || dalloc(c, w.pThr, ns) || dalloc(c, w.pRad, ns) ||
        dalloc(c, w.pMeta, ns) || dalloc(c, w.pBop, ns) || dalloc(c, w.cRayO, ns) || dalloc(c, w.cRayD, ns) ||
        dalloc(c, w.cHit, ns) || dalloc(c, w.cT, ns) || dalloc(c, w.sPos, ns) || dalloc(c, w.sNrm, ns) ||
        dalloc(c, w.sGeo, ns) || dalloc(c, w.sAlb, ns) || dalloc(c, w.sWo, ns) || dalloc(c, w.cSunSky, ns) ||
        dalloc(c, w.rRis, ns) || dalloc(c, w.rRR, ns) || dalloc(c, w.nIdx, ns) ||
        dalloc(c, w.ls0, ns) || dalloc(c, w.ls1, ns) || dalloc(c, w.tapPsv, ns) || dalloc(c, w.tapM, ns) ||
        dalloc(c, w.oHit, 4 * ns) ||
        dalloc(c, w.qO, 4 * ns) || dalloc(c, w.qD, 4 * ns) ||
        dalloc(c, w.qId, 4 * ns) || dalloc(c, w.qCount, kQueueWords) ||
        dalloc(c, w.sCell[0], 4 * ns + 2048) || dalloc(c, w.sT[0], 4 * ns + 2048) ||
        dalloc(c, w.sFace[0], 4 * ns + 2048) || dalloc(c, w.sCell[1], 4 * ns + 2048) ||
        dalloc(c, w.sT[1], 4 * ns + 2048) || dalloc(c, w.sFace[1], 4 * ns + 2048) ||
        dalloc(c, w.sBack, ns) || dalloc(c, w.rLoc, ns) || dalloc(c, w.lLoc0, ns) || dalloc(c, w.lLoc1, ns))
        return VXPT_ERR_HIP;
    c->wbSlots[set] = ns;
    return 0;
}

// A pass whose first half is enqueued (trace_front) and whose second half is not yet (trace_back).
struct PassPlan {
    TraceArgs a;
    int next = 0, set = 0;
};

// One 1-spp pass, first half.  overlap: the first half may run beside the previous pass's second
// half (it then waits only for the pass before that to release its state set).  Otherwise it starts
// after everything enqueued on the context stream.  A primary-only pass runs whole on the context
// stream here.
hipStream_t front_stream(const vxpt_ctx *c, int set) { return c->frontStreams[set % c->tune.front_streams]; }

// planes = false: a frame's pass before its last, which writes its tap records but not the G-buffer
// planes (the frame's planes are its last pass's; nothing reads an earlier pass's)
int trace_front(vxpt_ctx *c, int32_t it, uint32_t flags, bool accumulate, bool accumFirst, float accumScale,
                bool overlap, PassPlan &pl, bool planes = true) {
    if (!c->voxels.p) return fail(c, VXPT_ERR_STATE, "no voxels uploaded");
    if (!c->skyReady) return fail(c, VXPT_ERR_STATE, "sky not set");
    TraceArgs a{};
    fill_world(c, a.world);
    fill_sky(c, a.sky);
    a.bn = {c->bnSobol.p, c->bnScramble.p, c->bnRank.p};
    for (int i = 0; i < 13; ++i) a.mats[i] = c->mats[i];
    if (c->nMeshInst > 0) {
        if (!c->meshMats.p || std::memcmp(c->meshMatsUp, c->mats, sizeof(c->mats)) != 0) {
            if (int r = upload_vec(c, c->meshMats, c->mats, 32)) return r;
            std::memcpy(c->meshMatsUp, c->mats, sizeof(c->mats));
            overlap = false;  // the first half reads them: after the upload
        }
        a.mesh = mesh_dev(c);
        a.meshUV = c->blasUV.p;
        a.meshRow = c->meshRow.p;
        a.meshRowLight = c->meshRowLight.p;
        a.meshMats = c->meshMats.p;
        a.lights = c->lights.p;
        a.lightAlias = c->lightAlias.p;
        a.numLights = (int)c->nLights;
    }
    a.cam = c->cam;
    // the temporal taps reproject into the previous pass's view: the frame's history camera for its
    // first pass, the frame's own camera for the later passes of an accumulation
    a.prevCam = (accumulate && !accumFirst) ? c->cam : c->prevCam;
    // the slot this pass writes: not the previous pass's (its temporal taps), not the denoiser's
    // history, and not the one the previous pass's second half may still be reading
    int next = 0;
    while (next == c->last || next == c->hist || next == c->histOld || next == c->tracePrev || next == c->tracePrev2)
        ++next;
    const GSlot &cur = c->gb[next], &prev = c->gb[c->last];
    a.cur = {cur.normalRough, cur.geoNormalThin, cur.albedo, cur.matParam, cur.depth, cur.material, cur.rec};
    a.prev = {prev.normalRough, prev.geoNormalThin, prev.albedo, prev.matParam, prev.depth, prev.material, prev.rec};
    if (prev.recStale) {  // planes uploaded or copied in from the host: rebuild the taps' records
        HIPCHK(c, launch_pack_rec(a.prev, (size_t)c->W * c->H, c->stream));
        c->gb[c->last].recStale = false;
    }
    c->gb[next].recStale = false;  // this pass writes the records (and the planes unless !planes)
    const int set = c->passCount % c->nSets;
    a.illum = c->illumSet[set];
    a.motion = c->motion;
    a.writeMotion = c->motionZero ? 0 : 1;
    a.writePlanes = (planes || (flags & VXPT_TRACE_PRIMARY_ONLY)) ? 1 : 0;
    const size_t n = (size_t)c->W * c->H;
    a.resCur = c->res + (size_t)(((it % 2) + 2) % 2) * n;
    a.resPrev = c->res + (size_t)((((it + 1) % 2) + 2) % 2) * n;
    // the first pass of an accumulation writes the other buffer (the previous accumulation, the
    // pipelined denoiser's input, stays intact); trace_back makes it current
    a.accum = accumulate ? (accumFirst ? (c->accum == c->accumBuf[0] ? c->accumBuf[1] : c->accumBuf[0]) : c->accum)
                         : nullptr;
    a.accumScale = accumScale;
    a.accumFirst = accumFirst ? 1 : 0;
    a.W = c->W; a.H = c->H;
    a.y0 = c->rowBegin; a.y1 = c->rowEnd;
    a.iterationIndex = it;
    a.totalBounceLimit = c->totalBounce;
    a.diffuseBounceLimit = c->diffuseBounce;
    // A path outlives its first segment only through a specular hit (roughness
    // <= 1e-5, closesthit.cu:224) or a diffuse limit above 1 (RayGen.cu:146-173);
    // otherwise the later segments' kernels would find no live path.
    bool anySpecular = false;
    for (int b = 1; b <= 12; ++b) anySpecular |= !(c->mats[b].roughness > 0.00001f);
    if (c->nMeshInst > 0)  // instanced meshes in the world: their materials count too
        for (int b = 13; b < kBlockTypes; ++b)
            anySpecular |= c->blocks[b].triangles > 0 && !c->mats[b].emissive && !(c->mats[b].roughness > 0.00001f);
    a.segments = (c->diffuseBounce == 1 && !anySpecular) ? 1 : c->totalBounce;
    a.primaryOnly = (flags & VXPT_TRACE_PRIMARY_ONLY) ? 1 : 0;
    a.tilesX = (c->W + 7) / 8;
    a.nSlots = a.tilesX * ((a.y1 - a.y0 + 7) / 8) * 64;
    // tuning overlap = 0 (diagnostics): every first half after the previous pass, kernels one at a time
    if (!c->tune.overlap) overlap = false;
    bool fresh;
    if (int r = ensure_wave(c, set, (size_t)a.nSlots, fresh)) return r;
    if (fresh) overlap = false;  // the first half must follow the new buffers' zero fill
    a.wb = c->wb[set];
    a.numCU = c->numCU;
    a.iterCap = c->tune.iter_cap;
    a.iterCap2 = c->tune.iter_cap2;
    a.iterCap3 = c->tune.iter_cap3;
    a.iterCap4 = c->tune.iter_cap4;
    a.resumeWgPerCU = c->tune.resume_wg_per_cu;
    a.sortMode = c->tune.sort_mode;
    a.ldsBricks = c->tune.lds_bricks;
    a.resumeSplit = c->tune.resume_split;
    a.laterSplit = c->tune.later_split;
    a.restirWaves = c->tune.restir_waves;
    // whole 4-tile workgroups per tile row for the panels
    a.xcdOrder = c->tune.xcd_order & (a.tilesX % 4 == 0 ? 7 : 4);
    a.prevSceneEmpty = c->prevSceneEmpty;
    // the one pass after a light update remaps the previous pass's light indices (OptixRenderer.cpp:447-457)
    a.lightsDirty = (c->lightsDirty && c->prevNumLights > 0) ? 1 : 0;
    a.prevNumLights = (int)c->prevNumLights;
    a.lightRemap = c->lightRemap.p;
    // a primary-only pass runs no temporal reuse: the remap waits for the next full pass
    if (!(flags & VXPT_TRACE_PRIMARY_ONLY)) c->lightsDirty = 0;
    a.tex = c->texTable.p;
    a.texels = c->texels.p;
    a.texEnabled = (c->texEnabled && c->texTable.p) ? 1 : 0;
    c->prevSceneEmpty = 0;
    if (a.primaryOnly) {
        HIPCHK(c, launch_trace_front(a, c->stream));
    } else {
        // first half on its front stream: after the pass that last used this state set (overlap), or
        // after everything on the context stream
        hipStream_t fs = front_stream(c, set);
        if (overlap) {
            HIPCHK(c, hipStreamWaitEvent(fs, c->backDone[set], 0));
        } else {
            HIPCHK(c, hipEventRecord(c->frontGate, c->stream));
            HIPCHK(c, hipStreamWaitEvent(fs, c->frontGate, 0));
        }
        HIPCHK(c, launch_trace_front(a, fs));
        HIPCHK(c, hipEventRecord(c->frontDone[set], fs));
    }
    pl.a = a;
    pl.next = next;
    pl.set = set;
    return 0;
}

// Pipelined frames: whether a frame's later first halves wait (on the host) for the previous frame's
// denoiser chain.  Nothing requires it when spp >= 2 and the motion plane is the static world's: a
// first half writes a G-buffer slot that excludes the two the chain reads (hist, histOld), its own state
// set and radiance plane (the chain reads the spp average), and the motion plane only after an upload
// of it.  Otherwise (tuning chain_gate, the default) the gate keeps the chain alone on the GPU.
bool chain_gate(const vxpt_ctx *c, int spp) { return c->tune.chain_gate || spp < 2 || !c->motionZero; }

// The second half of the planned pass, on the context stream, and the ring bookkeeping.
// mark: record ev[1] behind the pass (vxpt_trace's timing; the frame loops keep their own events --
// every marker is one more packet between two kernels of the stream)
int trace_back(vxpt_ctx *c, const PassPlan &pl, bool mark = true) {
    const int set = pl.set;
    if (!pl.a.primaryOnly) {
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->frontDone[set], 0));
        HIPCHK(c, launch_trace_back(pl.a, c->stream, c->haloPending ? c->haloDone : nullptr));
        HIPCHK(c, hipEventRecord(c->backDone[set], c->stream));
    }
    c->haloPending = false;
    if (mark) HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
    c->tracePrev2 = c->tracePrev;
    c->tracePrev = c->last;
    c->last = pl.next;
    c->illum = c->illumSet[set];
    if (pl.a.accum) c->accum = pl.a.accum;
    c->lastSet = set;
    ++c->passCount;
    return 0;
}

int do_trace(vxpt_ctx *c, int32_t it, uint32_t flags, bool accumulate, bool accumFirst, float accumScale,
             bool overlap = false, bool mark = true, bool planes = true) {
    if (mark) HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
    PassPlan pl;
    if (int r = trace_front(c, it, flags, accumulate, accumFirst, accumScale, overlap, pl, planes)) return r;
    return trace_back(c, pl, mark);
}

// history hand-over NormalRough/Depth/Material -> Prev (Denoiser.cu:394-407):
// the slot the frame's last trace wrote becomes the denoiser's history slot
// (whole planes, so the rows a band received from its neighbours come along)
hipError_t history_copies(vxpt_ctx *c) {
    c->histOld = c->hist;
    c->hist = c->last;
    return hipSuccess;
}

// world positions for the band and kWposHalo rows either side (the widest
// stencil, HistoryFix at 2 x 17 rows, reads them there), in the firefly pass's
// launch (`detect`: the filter over the band; `apply`: write the filtered pixels
// back in this launch rather than in the next k_temporal)
constexpr int kWposHalo = 40;
constexpr int kDenoiseRows = kWposHalo;  // the deepest read of the current G-buffer planes by the denoiser
hipError_t firefly_band(const DenoiseArgs &a, bool detect, bool apply, hipStream_t st) {
    return launch_firefly(a, std::max(0, a.y0 - kWposHalo), std::min(a.H, a.y1 + kWposHalo), detect, apply, st);
}

// Denoiser::run (Denoiser.cu:24-408) on the context stream.  (Running all of it but the firefly
// stage on a third stream beside the next frame's first pass was measured and removed)
int do_denoise(vxpt_ctx *c, const vxpt_denoise_params *p, int frameNum, int it) {
    if (!p) p = &c->yamlDenoise;
    const int used = it > 0 ? it - 1 : 0;
    DenoiseArgs a{};
    fill_denoise(c, p, a, used & 1);
    HIPCHK(c, hipEventRecord(c->ev[2], c->stream));
    // the temporal pass applies the firefly lists when it runs
    const bool ffFold = p->enable_temporal_accumulation && frameNum > 0;
    HIPCHK(c, firefly_band(a, p->enable_firefly_filter, !ffFold, c->stream));
    hipStream_t st = c->stream;
    if (frameNum == 0) HIPCHK(c, launch_frame0_init(a, st));
    int fin = 0;  // 0 illum, 1 ping, 2 pong, 3 prevIllum
    if (p->enable_temporal_accumulation && frameNum > 0) {
        HIPCHK(c, launch_temporal(a, st));
        fin = 1;
        if (p->enable_history_fix) { HIPCHK(c, launch_history_fix(a, st)); fin = 2; }
        if (p->enable_history_clamping) { HIPCHK(c, launch_history_clamp(a, st)); fin = 3; }
    }
    bool outputDone = false;
    if (p->enable_spatial_filtering) {
        HIPCHK(c, launch_atrous_smem(a, st));
        fin = 1;
        if (p->atrous_iteration_num > 0) {
            int idx = 1;
            unsigned step = 1u << idx;
            const int maxIt = p->atrous_iteration_num * 2;
            while (idx < maxIt) {
                HIPCHK(c, launch_atrous(a, a.ping, a.pong, step, (unsigned)it, false, st));
                ++idx; step = 1u << idx;
                HIPCHK(c, launch_atrous(a, a.pong, a.ping, step, (unsigned)it, false, st));
                ++idx; step = 1u << idx;
            }
            HIPCHK(c, launch_atrous(a, a.ping, a.pong, step, (unsigned)it, true, st));
            fin = 2;
            outputDone = true;
        }
    }
    if (!outputDone) {
        const float4 *src = fin == 1 ? a.ping : (fin == 2 ? a.pong : (fin == 3 ? a.prevIllum : a.illum));
        HIPCHK(c, launch_copy_output(a, src, st));
    }
    HIPCHK(c, history_copies(c));
    HIPCHK(c, hipEventRecord(c->ev[3], st));
    return 0;
}

// one denoiser pass on the context's band, enqueued on its stream (vxpt_denoise_pass ids)
// margin (banded chains, band_frame's ghost rows): the pass also computes `margin` rows either side of
// the context's rows (8-aligned, clipped to the frame) -- the rows a later pass of the chain reads there,
// computed here from the same inputs as the neighbour computes them instead of received from it
int run_pass(vxpt_ctx *c, const vxpt_denoise_params *p, int pass, int arg, int arg2, int margin = 0) {
    DenoiseArgs a{};
    fill_denoise(c, p, a, pass == 0 ? (arg & 1) : 0);
    a.y0 = std::max(0, a.y0 - margin);
    a.y1 = std::min(a.H, a.y1 + margin);
    switch (pass) {
        case 0: HIPCHK(c, firefly_band(a, true, true, c->stream)); break;  // + world positions
        case 2: HIPCHK(c, launch_temporal(a, c->stream)); break;
        case 3: HIPCHK(c, launch_history_fix(a, c->stream)); break;
        case 4: HIPCHK(c, launch_history_clamp(a, c->stream)); break;
        case 5: HIPCHK(c, launch_atrous_smem(a, c->stream)); break;
        case 6: HIPCHK(c, launch_atrous(a, a.ping, a.pong, (unsigned)arg, (unsigned)arg2, false, c->stream)); break;
        case 7: HIPCHK(c, launch_atrous(a, a.pong, a.ping, (unsigned)arg, (unsigned)arg2, false, c->stream)); break;
        case 10: HIPCHK(c, launch_atrous(a, a.ping, a.pong, (unsigned)arg, (unsigned)arg2, true, c->stream)); break;
        case 11: HIPCHK(c, firefly_band(a, false, false, c->stream)); break;
        case 12: HIPCHK(c, launch_frame0_init(a, c->stream)); break;
        case 13: {
            const float4 *src = arg == 1 ? a.ping : (arg == 2 ? a.pong : (arg == 3 ? a.prevIllum : a.illum));
            HIPCHK(c, launch_copy_output(a, src, c->stream));
        } break;
        case 14: HIPCHK(c, history_copies(c)); break;
        default: return fail(c, VXPT_ERR_ARG, "unknown pass");
    }
    return VXPT_OK;
}

// ---------------------------------------------------------------- band partition
// The multi-GPU schedule of one frame (bands.py restates it for
// the CPU tests): every rank traces and denoises its 8-row-aligned band into
// full-frame buffers, and every pass that reads a neighbourhood is preceded by
// an exchange of exactly the rows it reads outside the band, with the band
// neighbours r +/- 1.  Rows are contiguous in every plane, so a halo is one
// ncclSend / ncclRecv per plane and neighbour, grouped, enqueued on the
// context stream behind the kernels that produced the rows -- no packing, no
// host synchronisation.
constexpr int kTraceHalo = 72;  // ReSTIR temporal taps: 64-pixel disk + reprojection (Restir.h:348-381)
// The next pass's temporal taps read only the previous pass's tap records (GBuf::rec) and reservoirs,
// so a pass hands its neighbours those two, 52 B/px, at the trace depth; the G-buffer planes are
// read by the denoiser alone (after the frame's last pass, within kDenoiseRows of the band: the
// world positions of k_firefly at kWposHalo, the history fix's taps at 34) and by the next frame's
// temporal accumulation as its history (histRows), so they travel once per frame.
const int kGbufPlanes[] = {VXPT_BUF_DEPTH, VXPT_BUF_NORMAL_ROUGH, VXPT_BUF_GEO_NORMAL_THIN,
                           VXPT_BUF_ALBEDO, VXPT_BUF_MATERIAL, VXPT_BUF_MAT_PARAM};
// a host-side write to a G-buffer plane leaves the slots' tap records stale (rebuilt before the next
// trace reads them)
bool is_gbuf_plane(int which) { return (which >= VXPT_BUF_DEPTH && which <= VXPT_BUF_MAT_PARAM) ||
                                       (which >= VXPT_BUF_PREV_NORMAL_ROUGH && which <= VXPT_BUF_PREV_MATERIAL); }
void gbuf_written(vxpt_ctx *c, int which) {
    if (which == VXPT_BUF_MOTION) c->motionZero = false;
    if (is_gbuf_plane(which))
        for (GSlot &g : c->gb) g.recStale = true;
}
const int kHistoryBufs[] = {VXPT_BUF_PREV_ILLUM, VXPT_BUF_PREV_FAST, VXPT_BUF_PREV_HIST_LEN};

void band_rows(int H, int world, int rank, int &y0, int &y1) {
    const int per = (H + 8 * world - 1) / (8 * world) * 8;
    y0 = std::min(H, rank * per);
    y1 = std::min(H, y0 + per);
}

// the equal bands' boundaries: band r = rows [s[r], s[r + 1])
std::vector<int> equal_splits(int H, int world) {
    std::vector<int> s(world + 1, 0);
    for (int r = 0; r < world; ++r) band_rows(H, world, r, s[r], s[r + 1]);
    return s;
}

// an uneven partition (vxpt_band_comm_init_rows): 0 = s[0] < s[1] < ... < s[n] = H, inner
// boundaries 8-aligned (vxpt_set_band), every band at least the ReSTIR halo tall when n > 1
bool splits_valid(const int32_t *s, int n, int H, int minRows) {
    if (!s || n < 1 || s[0] != 0 || s[n] != H) return false;
    for (int k = 0; k < n; ++k)
        if (s[k + 1] - s[k] < (n > 1 ? minRows : 1) || (k > 0 && (s[k] & 7))) return false;
    return true;
}

struct Halo { int peer, sy, sn, ry, rn; };
// rows rank sends to / receives from each band neighbour of the partition s (both sides of a
// border move min(rows, the two band heights) rows)
std::vector<Halo> halo_plan(const std::vector<int> &s, int rank, int rows) {
    std::vector<Halo> plan;
    const int world = (int)s.size() - 1;
    const int y0 = s[rank], y1 = s[rank + 1];
    if (rank > 0) {
        const int n = std::min(rows, std::min(y1 - y0, s[rank] - s[rank - 1]));
        plan.push_back({rank - 1, y0, n, y0 - n, n});
    }
    if (rank < world - 1) {
        const int n = std::min(rows, std::min(y1 - y0, s[rank + 2] - s[rank + 1]));
        plan.push_back({rank + 1, y1 - n, n, y1, n});
    }
    return plan;
}

// the context's partition: its row_splits, or the equal bands
std::vector<int> splits_of(const vxpt_ctx *c) {
    return (int)c->splits.size() == c->nranks + 1 ? c->splits : equal_splits(c->H, c->nranks);
}

// Halo depths of a banded frame whose camera moved between passes (cur vs prev).  A band's
// pixels reproject to rows prevCam.dir_to_uv(hit - prevCam.pos).y * H: the ReSTIR temporal taps
// read the previous pass's G-buffer and reservoirs within 64 rows of that row (Restir.h:348-381,
// truncated row), the temporal accumulation its histories within its bicubic footprint (-1..+2
// around floor(row - 0.5), TemporalAccumulation.h:29-215).  For a rotation the reprojection does
// not depend on depth: the extreme rows over the band come from the pixel corners on the band's
// first and last row boundaries (all columns) plus a 33-column grid over every row; 2 rows of
// margin cover host/device rounding.  A translation t makes a pixel's row depend on its hit
// distance d: row(d) = (d a.y + b.y) / (d a.z + b.z) with a = worldToUv dir, b = worldToUv t, a
// Moebius map of d, monotone on [nearDepth, inf) while its denominator stays positive there -- so
// with a lower bound nearDepth on every primary hit's distance the extremes are the rows at
// nearDepth and at infinity (the rotation's), sampled on a 129-column grid.  Without such a bound
// (nearDepth <= 0) a translated camera is refused; so is a point behind the previous camera or a
// halo deeper than a neighbouring band (the plan only reaches ranks r +/- 1).  An unmoved camera
// keeps the static depths (72 / 2).
bool band_halo_rows(const CamDev &cam, const CamDev &pc, int W, int H, const std::vector<int> &splits,
                    int &traceRows, int &histRows, std::string &err, float nearDepth = 0.0f) {
    const int world = (int)splits.size() - 1;
    traceRows = kTraceHalo;
    histRows = 2;
    if (world <= 1) return true;
    if (std::memcmp(&cam, &pc, sizeof(CamDev)) == 0) return true;
    const V3 t = cam.pos - pc.pos;
    const bool moved = t.x != 0.0f || t.y != 0.0f || t.z != 0.0f;
    if (moved && !(nearDepth > 0.0f)) {
        err = "banded frames need a camera that does not translate between passes, or a lower bound on the "
              "primary hits' distance (depth-dependent reprojection)";
        return false;
    }
    const V3 b = m3_apply(pc.worldToUv, t);
    const int cols = moved ? 128 : 32;
    int minBand = H;
    float reach = 0.0f;  // rows beyond its band any band pixel reprojects to
    for (int r = 0; r < world; ++r) {
        const int y0 = splits[r], y1 = splits[r + 1];
        if (y1 <= y0) continue;
        minBand = std::min(minBand, y1 - y0);
        float lo = 1e30f, hi = -1e30f;
        bool behind = false;
        auto sample = [&](float u, float v) {
            const V3 d = cam.uv_to_dir(V2(u, v));
            const V3 n = m3_apply(pc.worldToUv, d);
            if (!(n.z > 0.0f)) { behind = true; return; }
            const float py = n.y / n.z * (float)H;
            lo = std::min(lo, py);
            hi = std::max(hi, py);
            if (moved) {  // the hit at the nearest distance
                const V3 m = n * nearDepth + b;
                if (!(m.z > 0.0f)) { behind = true; return; }
                const float pm = m.y / m.z * (float)H;
                lo = std::min(lo, pm);
                hi = std::max(hi, pm);
            }
        };
        for (int x = 0; x <= W; ++x) {
            sample((float)x / (float)W, (float)y0 / (float)H);
            sample((float)x / (float)W, (float)y1 / (float)H);
        }
        for (int y = y0; y <= y1; ++y)
            for (int k = 0; k <= cols; ++k) sample((float)k / (float)cols, (float)y / (float)H);
        if (behind) {
            err = "the camera moved so far that part of a band lies behind the previous camera";
            return false;
        }
        if (r > 0) reach = std::max(reach, (float)y0 - lo);
        if (r < world - 1) reach = std::max(reach, hi - (float)y1);
    }
    const int d = (int)std::ceil(std::max(reach, 0.0f)) + 2;
    traceRows = std::max(kTraceHalo, 64 + d + 1);
    histRows = std::max(2, d + 2);
    if (traceRows > minBand) {
        err = "the camera moved " + std::to_string(d) + " rows between passes: a " + std::to_string(traceRows) +
              "-row halo exceeds the " + std::to_string(minBand) + "-row bands";
        return false;
    }
    return true;
}

// A lower bound on the distance from p to any primary hit: the nearest non-air cell's box, grown by
// meshGrow cells on every side (instanced meshes may overhang their cell; 1 unless a loaded mesh
// reaches further), over the host mirror of the world, within 64 cells of p's cell (beyond that,
// 63 - grow is the bound).  Empty space outside the world holds no geometry.  The search walks
// Chebyshev rings of 4^3 bricks around p's brick, visits the cells of non-empty bricks only
// (hNonAir) and stops once a ring cannot hold anything closer.
float nearest_surface(const vxpt_ctx *c, V3 p) {
    const int WX = c->cx * 32, WY = c->cy * 32, WZ = c->cz * 32;
    if (c->hIds.empty() || WX == 0 || c->hNonAir.empty()) return 1e30f;
    constexpr int kRings = 64;
    const float grow = c->meshGrow;
    const float cap = (float)(kRings - 1) - grow;
    auto gap = [&](float v, float lo, float hi) { return v < lo ? lo - v : (v > hi ? v - hi : 0.0f); };
    const int px = (int)std::floor(p.x), py = (int)std::floor(p.y), pz = (int)std::floor(p.z);
    const int bx0 = px >> 2, by0 = py >> 2, bz0 = pz >> 2;  // (arithmetic shift: floor for negatives)
    const int BX = WX / 4, BY = WY / 4, BZ = WZ / 4;
    float best = 1e30f;
    auto brick = [&](int bx, int by, int bz) {
        if (bx < 0 || by < 0 || bz < 0 || bx >= BX || by >= BY || bz >= BZ) return;
        const size_t b = brick_lin(c, bx, by, bz);
        if (!c->hNonAir[b]) return;
        const float dx = gap(p.x, 4.0f * bx - grow, 4.0f * bx + 4.0f + grow);
        const float dy = gap(p.y, 4.0f * by - grow, 4.0f * by + 4.0f + grow);
        const float dz = gap(p.z, 4.0f * bz - grow, 4.0f * bz + 4.0f + grow);
        if (std::sqrt(dx * dx + dy * dy + dz * dz) >= best) return;
        for (int lc = 0; lc < 64; ++lc) {
            if (!c->hBricks[b * 64 + lc]) continue;
            const int x = bx * 4 + (lc & 3), z = bz * 4 + ((lc >> 2) & 3), y = by * 4 + (lc >> 4);
            const float ex = gap(p.x, (float)x - grow, (float)(x + 1) + grow);
            const float ey = gap(p.y, (float)y - grow, (float)(y + 1) + grow);
            const float ez = gap(p.z, (float)z - grow, (float)(z + 1) + grow);
            best = std::min(best, std::sqrt(ex * ex + ey * ey + ez * ez));
        }
    };
    // cells within Chebyshev distance 64 of p's cell lie within 17 bricks of p's brick; a cell
    // further out is >= 64 - grow away, past the cap
    for (int r = 0; r <= kRings / 4 + 1; ++r) {
        // every brick of ring r is at least 4 (r - 1) - grow away along its farthest axis
        if (best <= 4.0f * (float)(r - 1) - grow) break;
        for (int dy = -r; dy <= r; ++dy)
            for (int dz = -r; dz <= r; ++dz) {
                const bool face = dy == -r || dy == r || dz == -r || dz == r;
                if (face) {
                    for (int dx = -r; dx <= r; ++dx) brick(bx0 + dx, by0 + dy, bz0 + dz);
                } else {
                    brick(bx0 - r, by0 + dy, bz0 + dz);
                    if (r > 0) brick(bx0 + r, by0 + dy, bz0 + dz);
                }
            }
    }
    return std::min(best, cap);
}

char *buffer_rows(vxpt_ctx *c, int which, int y, size_t &rowBytes) {
    void *p, *mirror;
    size_t n;
    buffer_ptr(c, which, p, n, false, &mirror);
    rowBytes = n / (size_t)c->H;
    return static_cast<char *>(p) + (size_t)y * rowBytes;
}

// Halo exchange of `bufs` over `rows` rows for every context of the frame
// (one with RCCL, all of this process's bands when linked).
// With overlap (RCCL only) the exchange runs on the context's exchange stream
// after the rows' producer and the next trace pass's temporal-reuse kernel waits
// for it (do_trace); the trace passes touch neither the sent rows nor the
// received ones before that kernel (they write the other G-buffer slot and
// reservoir parity).
// several buffers with their own halo depths in one group (one RCCL launch, one sync point)
// after (RCCL, overlap): the exchange starts once that event has completed instead of behind the
// context stream's work so far (the tap records: after the producing pass's first half)
int exchange_set(std::vector<vxpt_ctx *> &cs, const std::vector<std::pair<int, int>> &bufRows, bool overlap = false,
                 hipEvent_t after = nullptr);

int exchange(std::vector<vxpt_ctx *> &cs, const std::vector<int> &bufs, int rows, bool overlap = false) {
    std::vector<std::pair<int, int>> br;
    for (int b : bufs) br.emplace_back(b, rows);
    return exchange_set(cs, br, overlap);
}

#define BANDCHK_(expr)                  \
    do {                                \
        if (int r_ = (expr)) return r_; \
    } while (0)
// a vxpt_band_stats timing event recorded on st (collection on), its pool index
int stat_mark(vxpt_ctx *c, hipStream_t st, size_t &idx) {
    auto &b = c->bst;
    if (b.used == b.pool.size()) {
        hipEvent_t e;
        HIPCHK(c, hipEventCreate(&e));
        b.pool.push_back(e);
    }
    idx = b.used++;
    HIPCHK(c, hipEventRecord(b.pool[idx], st));
    return 0;
}
// the collected spans' times into the running totals, their events back to the pool (every span's
// events have completed: the caller synchronised the context and exchange streams)
constexpr size_t kStatPoolFold = 512;
int stat_fold(vxpt_ctx *c) {
    auto &b = c->bst;
    for (const auto &sp : b.spans) {
        float ms = 0.0f;
        HIPCHK(c, hipEventElapsedTime(&ms, b.pool[sp.e0], b.pool[sp.e1]));
        b.ms[sp.kind] += ms;
    }
    b.spans.clear();
    b.used = 0;
    return VXPT_OK;
}
int stat_sync_fold(vxpt_ctx *c) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->commStream) HIPCHK(c, hipStreamSynchronize(c->commStream));
    return stat_fold(c);
}
// the bytes a halo plan entry sends, to the neighbour above (peer < rank) or below
void stat_bytes(vxpt_ctx *c, const Halo &h, size_t rowBytes) {
    (h.peer < c->rank ? c->bst.up : c->bst.down) += (double)h.sn * (double)rowBytes;
}

int exchange_set(std::vector<vxpt_ctx *> &cs, const std::vector<std::pair<int, int>> &bufRows, bool overlap,
                 hipEvent_t after) {
    if (cs.size() == 1 && cs[0]->comm) {
        vxpt_ctx *c = cs[0];
        hipStream_t st = c->stream;
        if (overlap) {
            if (!after) {
                HIPCHK(c, hipEventRecord(c->haloReady, c->stream));
                after = c->haloReady;
            }
            HIPCHK(c, hipStreamWaitEvent(c->commStream, after, 0));
            if (c->exDoneRec) HIPCHK(c, hipStreamWaitEvent(c->commStream, c->exDone, 0));
            st = c->commStream;
        } else if (c->haloPending) {
            HIPCHK(c, hipStreamWaitEvent(c->stream, c->haloDone, 0));
        }
        size_t m0 = 0, m1 = 0;
        if (c->bst.on) BANDCHK_(stat_mark(c, st, m0));
        if (ncclGroupStart() != ncclSuccess) return fail(c, VXPT_ERR_HIP, "ncclGroupStart");
        ncclResult_t rc = ncclSuccess;
        for (const auto &br : bufRows)
            for (const Halo &h : halo_plan(splits_of(c), c->rank, br.second)) {
                const int b = br.first;
                size_t rb;
                char *send = buffer_rows(c, b, h.sy, rb);
                char *recv = buffer_rows(c, b, h.ry, rb);
                if (rc == ncclSuccess) rc = ncclSend(send, (size_t)h.sn * rb, ncclUint8, h.peer, c->comm, st);
                if (rc == ncclSuccess) rc = ncclRecv(recv, (size_t)h.rn * rb, ncclUint8, h.peer, c->comm, st);
                if (c->bst.on) stat_bytes(c, h, rb);
            }
        const ncclResult_t re = ncclGroupEnd();  // closes the group whatever failed inside it
        if (rc != ncclSuccess)
            return fail(c, VXPT_ERR_HIP, std::string("ncclSend/ncclRecv (halo exchange): ") + ncclGetErrorString(rc));
        if (re != ncclSuccess)
            return fail(c, VXPT_ERR_HIP, std::string("ncclGroupEnd (halo exchange): ") + ncclGetErrorString(re));
        if (c->bst.on) {
            BANDCHK_(stat_mark(c, st, m1));
            c->bst.spans.push_back({m0, m1, overlap ? 1 : 0});
            ++c->bst.groups;
            if (!overlap) ++c->bst.groupsOrdered;
        }
        if (overlap) {
            HIPCHK(c, hipEventRecord(c->haloDone, c->commStream));
            c->haloPending = true;
        } else {
            HIPCHK(c, hipEventRecord(c->exDone, c->stream));
            c->exDoneRec = true;
        }
        return VXPT_OK;
    }
    // linked contexts of one process: device copies from each neighbour's own rows
    // (never written by an exchange), after every band finished the producing pass
    for (vxpt_ctx *c : cs) HIPCHK(c, hipStreamSynchronize(c->stream));
    for (vxpt_ctx *c : cs) {
        size_t m0 = 0, m1 = 0;
        if (c->bst.on) BANDCHK_(stat_mark(c, c->stream, m0));
        for (const auto &br : bufRows)
            for (const Halo &h : halo_plan(splits_of(c), c->rank, br.second)) {
                const int b = br.first;
                size_t rb;
                char *dst = buffer_rows(c, b, h.ry, rb);
                const char *src = buffer_rows(cs[h.peer], b, h.ry, rb);
                HIPCHK(c, hipMemcpyAsync(dst, src, (size_t)h.rn * rb, hipMemcpyDeviceToDevice, c->stream));
                // this band's rows the neighbour copies: what an RCCL rank sends
                if (c->bst.on) stat_bytes(c, h, rb);
            }
        if (c->bst.on) {
            BANDCHK_(stat_mark(c, c->stream, m1));
            c->bst.spans.push_back({m0, m1, 0});
            ++c->bst.groups;
            ++c->bst.groupsOrdered;
        }
    }
    for (vxpt_ctx *c : cs) HIPCHK(c, hipStreamSynchronize(c->stream));
    return VXPT_OK;
}

int atrous_rows(int step) { return step + (step > 4 ? step / 4 : 0); }  // Atrous.h:79-84 jitter above step 4

#define BANDCHK(expr)              \
    do {                           \
        if (int r_ = (expr)) return r_; \
    } while (0)
#define FOR_BANDS(expr)                 \
    do {                                \
        for (vxpt_ctx *c : cs) BANDCHK(expr); \
    } while (0)

// One banded OfflineBackend::renderFrame over cs (vxpt_render_frame's order).
// the last banded frame's timings (its events complete: after a sync of the context streams)
void band_timings(std::vector<vxpt_ctx *> &cs) {
    for (vxpt_ctx *c : cs) {
        float t = 0, d = 0, f = 0;
        hipEventElapsedTime(&t, c->ev[6], c->ev[1]);
        hipEventElapsedTime(&d, c->ev[2], c->ev[3]);
        hipEventElapsedTime(&f, c->ev[6], c->ev[7]);
        c->timing.trace_ms = t;   // the band's trace passes and their halo exchanges
        c->timing.denoise_ms = d; // the band's denoiser passes and their halo exchanges
        c->timing.frame_ms = f;
    }
}

// sync = false (a run of frames, vxpt_render_frames): enqueue the frame and return, so that the host
// enqueues the next frame while this one runs; the caller syncs after the last.
// pipe (the pipelined run, vxpt_render_frames' order for bands): when it holds plans, they are this
// frame's first pass-halves, enqueued by the previous frame's call beside its last second half, and
// this call opens with their second halves; with pipeNext this call leaves the next frame's first
// pass-halves in it (their first halves run beside this frame's last second half and its exchange,
// the denoiser chain after them), and the next call gates its later first halves on the host behind
// this frame's chain (vxpt_render_frames' host gate: no front stream parked behind a wait for it).
int band_frame(std::vector<vxpt_ctx *> &cs, const vxpt_denoise_params *p, int frame, int spp, bool sync = true,
               std::vector<PassPlan> *pipe = nullptr, bool pipeNext = false) {
    const int it0 = frame * spp;
    // halo depths for this frame's camera motion; the previous frame exchanged its last pass's
    // rows and the histories for its own camera: top them up before the first pass reads them
    int traceRows = kTraceHalo, histRows = 2;
    {
        vxpt_ctx *c0 = cs[0];
        std::string err;
        // a translated camera: the nearest surface bounds every primary hit's distance
        const bool moved = c0->cam.pos.x != c0->prevCam.pos.x || c0->cam.pos.y != c0->prevCam.pos.y ||
                           c0->cam.pos.z != c0->prevCam.pos.z;
        float nearDepth = 0.0f;
        bool reused = false;
        auto search = [&]() {
            nearDepth = nearest_surface(c0, c0->cam.pos);
            c0->nearPos = c0->cam.pos;
            c0->nearDist = nearDepth;
            c0->nearVersion = c0->worldVersion;
        };
        if (moved) {
            const V3 dp = c0->cam.pos - c0->nearPos;
            const float reuse = c0->nearDist - std::sqrt(dp.x * dp.x + dp.y * dp.y + dp.z * dp.z);
            reused = c0->nearVersion == c0->worldVersion && reuse >= 0.75f * c0->nearDist && reuse > 0.0f;
            if (reused) nearDepth = reuse;
            else search();
        }
        bool ok = band_halo_rows(c0->cam, c0->prevCam, c0->W, c0->H, splits_of(c0), traceRows, histRows, err, nearDepth);
        if (!ok && reused) {  // the reused bound is looser than a fresh search: search before refusing
            search();
            ok = band_halo_rows(c0->cam, c0->prevCam, c0->W, c0->H, splits_of(c0), traceRows, histRows, err, nearDepth);
        }
        if (!ok) return fail(c0, VXPT_ERR_STATE, err.c_str());
    }
    // the G-buffer planes' depth: the denoiser's reads, or the next temporal accumulation's history
    const int planeRows = std::max(kDenoiseRows, histRows);
    if (frame > 0 && (traceRows > cs[0]->haloTraceRows || histRows > cs[0]->haloHistRows ||
                      planeRows > cs[0]->haloPlaneRows)) {
        std::vector<std::pair<int, int>> br;
        br.emplace_back(VXPT_BUF_TAP_RECORD, traceRows);
        br.emplace_back(((it0 - 1) & 1) ? VXPT_BUF_RES_ODD : VXPT_BUF_RES_EVEN, traceRows);
        for (int b : kGbufPlanes) br.emplace_back(b, planeRows);
        for (int b : kHistoryBufs) br.emplace_back(b, histRows);
        BANDCHK(exchange_set(cs, br, false));
    }
    for (vxpt_ctx *c : cs) {
        c->haloTraceRows = traceRows;
        c->haloHistRows = histRows;
        c->haloPlaneRows = planeRows;
    }
    for (vxpt_ctx *c : cs)  // no span of this frame is open yet: a full pool is folded here
        if (c->bst.on && c->bst.used >= kStatPoolFold) BANDCHK(stat_sync_fold(c));
    for (vxpt_ctx *c : cs) HIPCHK(c, hipEventRecord(c->ev[6], c->stream));
    std::vector<size_t> mk(cs.size() * 3, 0);  // vxpt_band_stats: trace start, trace end, denoiser end
    for (size_t k = 0; k < cs.size(); ++k)
        if (cs[k]->bst.on) BANDCHK(stat_mark(cs[k], cs[k]->stream, mk[3 * k]));
    const bool piped = pipe && pipe->size() == cs.size();
    for (int s = 0; s < spp; ++s) {
        if (s == 0 && piped) {
            for (size_t k = 0; k < cs.size(); ++k) BANDCHK(trace_back(cs[k], (*pipe)[k], false));
            pipe->clear();
            // the later first halves are enqueued once the previous frame's chain has finished (chain_gate)
            for (vxpt_ctx *c : cs)
                if (chain_gate(c, spp)) HIPCHK(c, hipEventSynchronize(c->ev[7]));
        } else {
            FOR_BANDS(do_trace(c, it0 + s, 0, spp > 1, s == 0, 1.0f / (float)spp, s > 0, false, s + 1 == spp));
        }
        if (s + 1 == spp && pipe && pipeNext) {  // the next frame's first pass-halves
            pipe->resize(cs.size());
            for (size_t k = 0; k < cs.size(); ++k)
                BANDCHK(trace_front(cs[k], it0 + spp, 0, spp > 1, true, 1.0f / (float)spp, true, (*pipe)[k], spp == 1));
        }
        const int res = ((it0 + s) & 1) ? VXPT_BUF_RES_ODD : VXPT_BUF_RES_EVEN;
        if (s + 1 < spp) {
            // all but the last pass: the next pass's temporal taps' inputs -- the tap records on the
            // exchange stream once the pass's first half wrote them (beside its second half; the next
            // pass's k_restir waits for them), the reservoirs in stream order after its second half
            // (the next second half opens with k_restir: nothing to overlap them with; round 4 sent
            // both after the second half on the exchange stream)
            hipEvent_t recDone = cs.size() == 1 && cs[0]->comm ? cs[0]->frontDone[cs[0]->lastSet] : nullptr;
            BANDCHK(exchange_set(cs, {{VXPT_BUF_TAP_RECORD, traceRows}}, true, recDone));
            BANDCHK(exchange_set(cs, {{res, traceRows}}, false));
        } else {
            // the last pass: its planes for the denoiser, and the denoiser input (radiance, or the spp
            // average) for the firefly filter's 3x3 neighbours.  Its reservoirs go out at the trace
            // depth after the firefly filter has rewritten them (below); without the filter, here.
            for (vxpt_ctx *c : cs) c->denoiseInputIsAccum = spp > 1;
            std::vector<std::pair<int, int>> br{{VXPT_BUF_TAP_RECORD, traceRows}, {VXPT_BUF_ILLUM, 2},
                                                {res, p->enable_firefly_filter ? 2 : traceRows}};
            for (int b : kGbufPlanes) br.emplace_back(b, planeRows);
            BANDCHK(exchange_set(cs, br, false));
        }
    }
    for (size_t k = 0; k < cs.size(); ++k) {
        vxpt_ctx *c = cs[k];
        c->denoiseInputIsAccum = spp > 1;
        // the chain after the next frame's first pass-half (pipelined), so it runs alone -- with the
        // chain gate (without it the later first halves run beside the chain anyway: no wait)
        if (pipe && pipeNext && pipe->size() == cs.size() && chain_gate(c, spp))
            HIPCHK(c, hipStreamWaitEvent(c->stream, c->frontDone[(*pipe)[k].set], 0));
        HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
        HIPCHK(c, hipEventRecord(c->ev[2], c->stream));
    }
    for (size_t k = 0; k < cs.size(); ++k)
        if (cs[k]->bst.on) BANDCHK(stat_mark(cs[k], cs[k]->stream, mk[3 * k + 1]));
    const int it = it0 + spp, used = it > 0 ? it - 1 : 0;
    std::vector<std::pair<int, int>> deferred;  // halo rows no pass reads before the next group
    auto exg = [&](std::vector<std::pair<int, int>> br) {
        br.insert(br.end(), deferred.begin(), deferred.end());
        deferred.clear();
        return exchange_set(cs, br);
    };
    auto to_rows = [](const std::vector<int> &bufs, int rows) {
        std::vector<std::pair<int, int>> br;
        for (int bf : bufs) br.emplace_back(bf, rows);
        return br;
    };
    if (!p->enable_firefly_filter) FOR_BANDS(run_pass(c, p, 11, 0, 0));
    if (p->enable_firefly_filter) {  // + world positions
        FOR_BANDS(run_pass(c, p, 0, used & 1, 0));
        // the filtered reservoirs (read by the next frame's first temporal taps) and radiance (read by
        // the history clamp's neighbourhood) ride along with the next group instead of one of their own
        deferred.emplace_back((used & 1) ? VXPT_BUF_RES_ODD : VXPT_BUF_RES_EVEN, traceRows);
        deferred.emplace_back(VXPT_BUF_ILLUM, 2);
    }
    const std::vector<int> hist(std::begin(kHistoryBufs), std::end(kHistoryBufs));
    if (frame == 0) {
        FOR_BANDS(run_pass(c, p, 12, 0, 0));
        BANDCHK(exg(to_rows(hist, histRows)));
    }
    // Ghost rows (the default chain, frames > 0): the history clamp and the a-trous steps compute the
    // rows the later steps read outside the band themselves (run_pass margins), so the chain exchanges
    // twice -- after the temporal pass and after the history fix -- instead of after every pass.  The
    // margins, backwards from the output (margin 0): a step at margin m reads its input at m + its reach
    // (a-trous rows of the step; 2 for the LDS a-trous and the clamp's 5x5), 8-aligned.  The history fix
    // (its taps 34 rows away) stays at margin 0: ghost rows for it would cost 34 more rows of every pass
    // before it.  Its inputs at the clamp's margin + 2 come in the two groups; the clamp's histories at
    // its margin serve the next frame's temporal pass (histRows <= that margin: no exchange).
    std::vector<int> atrousSteps;  // steps 2, 4, ..., 2^(2n+1): the last one (pass 10) writes the output
    for (int idx = 1; idx <= 2 * p->atrous_iteration_num + 1; ++idx) atrousSteps.push_back(1 << idx);
    std::vector<int> stepMargin(atrousSteps.size(), 0);
    int smemMargin = 0, clampMargin = 0;
    {
        int m = 0;
        for (int k = (int)atrousSteps.size() - 1; k >= 0; --k) {
            stepMargin[k] = m;
            m = (m + atrous_rows(atrousSteps[k]) + 7) / 8 * 8;
        }
        smemMargin = m;
        clampMargin = (smemMargin + 2 + 7) / 8 * 8;
    }
    const bool ghost = cs.size() > 0 && cs[0]->tune.ghost_rows && frame > 0 && p->enable_temporal_accumulation &&
                       p->enable_history_fix && p->enable_history_clamping && p->enable_spatial_filtering &&
                       p->atrous_iteration_num > 0 &&
                       // the clamp's pixel planes and the a-trous taps' world positions / normals, read at
                       // up to the LDS a-trous margin + 2, are there already (the last pass's planes, the
                       // firefly pass's positions)
                       clampMargin <= planeRows && smemMargin + 2 <= kWposHalo;
    int fin = 0;
    if (ghost) {
        FOR_BANDS(run_pass(c, p, 2, 0, 0));
        // the history fix's ping taps (34 rows) and the clamp's inputs at its margin: ping and the history
        // length at the pixel, the radiance in its 5x5 (the firefly-filtered values; the deferred 2-row
        // radiance entry is this one)
        std::vector<std::pair<int, int>> br{{VXPT_BUF_PING, std::max(34, clampMargin)}, {VXPT_BUF_PONG, 2},
                                            {VXPT_BUF_HIST_LEN, clampMargin}, {VXPT_BUF_ILLUM, clampMargin + 2}};
        for (const auto &d : deferred)
            if (d.first != VXPT_BUF_ILLUM) br.push_back(d);
        deferred.clear();
        BANDCHK(exchange_set(cs, br));
        FOR_BANDS(run_pass(c, p, 3, 0, 0));
        BANDCHK(exchange_set(cs, {{VXPT_BUF_PONG, clampMargin + 2}}));  // the clamp's 5x5 of the fixed history
        FOR_BANDS(run_pass(c, p, 4, 0, 0, clampMargin));
        if (histRows > clampMargin) BANDCHK(exchange_set(cs, to_rows(hist, histRows)));
        FOR_BANDS(run_pass(c, p, 5, 0, 0, smemMargin));
        for (size_t k = 0; k < atrousSteps.size(); ++k) {
            const int pass = k + 1 == atrousSteps.size() ? 10 : (k % 2 == 0 ? 6 : 7);
            FOR_BANDS(run_pass(c, p, pass, atrousSteps[k], it, stepMargin[k]));
        }
        for (vxpt_ctx *c : cs) c->haloHistRows = std::max(histRows, clampMargin);
        FOR_BANDS(run_pass(c, p, 14, 0, 0));
    }
    if (p->enable_temporal_accumulation && frame > 0 && !ghost) {
        FOR_BANDS(run_pass(c, p, 2, 0, 0));
        // HistoryFix taps: 2 x (2^3 + 1) rows of ping; pong for its 2-row stencils
        BANDCHK(exg({{VXPT_BUF_PING, 34}, {VXPT_BUF_PONG, 2}}));
        fin = 1;
        if (p->enable_history_fix) {
            FOR_BANDS(run_pass(c, p, 3, 0, 0));
            BANDCHK(exg({{VXPT_BUF_PONG, 2}}));
            fin = 2;
        }
        if (p->enable_history_clamping) {
            FOR_BANDS(run_pass(c, p, 4, 0, 0));
            BANDCHK(exg(to_rows(hist, histRows)));
            fin = 3;
        }
    }
    bool outDone = ghost;
    if (p->enable_spatial_filtering && !ghost) {
        FOR_BANDS(run_pass(c, p, 5, 0, 0));
        BANDCHK(exg({{VXPT_BUF_PING, atrous_rows(2)}}));
        fin = 1;
        if (p->atrous_iteration_num > 0) {
            int idx = 1, step = 2;
            while (idx < 2 * p->atrous_iteration_num) {
                FOR_BANDS(run_pass(c, p, 6, step, it));
                step = 1 << ++idx;
                BANDCHK(exg({{VXPT_BUF_PONG, atrous_rows(step)}}));
                FOR_BANDS(run_pass(c, p, 7, step, it));
                step = 1 << ++idx;
                BANDCHK(exg({{VXPT_BUF_PING, atrous_rows(step)}}));
            }
            FOR_BANDS(run_pass(c, p, 10, step, it));
            fin = 2;
            outDone = true;
        }
    }
    if (!deferred.empty()) BANDCHK(exg({}));  // nothing after the firefly pass exchanged (chain switches)
    if (!outDone) FOR_BANDS(run_pass(c, p, 13, fin, 0));
    if (!ghost) FOR_BANDS(run_pass(c, p, 14, 0, 0));
    for (vxpt_ctx *c : cs) {
        HIPCHK(c, hipEventRecord(c->ev[3], c->stream));
        HIPCHK(c, hipEventRecord(c->ev[7], c->stream));
    }
    for (size_t k = 0; k < cs.size(); ++k) {
        vxpt_ctx *c = cs[k];
        if (!c->bst.on) continue;
        BANDCHK(stat_mark(c, c->stream, mk[3 * k + 2]));
        c->bst.spans.push_back({mk[3 * k], mk[3 * k + 1], 2});
        c->bst.spans.push_back({mk[3 * k + 1], mk[3 * k + 2], 3});
        ++c->bst.frames;
    }
    if (!sync) return VXPT_OK;
    for (vxpt_ctx *c : cs) HIPCHK(c, hipStreamSynchronize(c->stream));
    band_timings(cs);
    for (vxpt_ctx *c : cs)
        if (c->bst.on) BANDCHK(stat_sync_fold(c));
    return VXPT_OK;
}

}  // namespace

// =====================================================================  C ABI
extern "C" {

const char *vxpt_last_error(const vxpt_ctx *c) { return c ? c->err.c_str() : "null context"; }

int vxpt_create(const vxpt_config *cfg, vxpt_ctx **out) {
    if (!cfg || !out) return VXPT_ERR_ARG;
    *out = nullptr;
    if (cfg->width <= 0 || cfg->height <= 0) return VXPT_ERR_ARG;  // any size: partial 8x8 trace tiles and 16x16 denoise tiles are masked
    // the trace pass keeps 4 ray queues per path segment, kQueues in all (vx_internal.hpp)
    if (cfg->total_bounce_limit > kQueues / 4 || cfg->diffuse_bounce_limit > 16) return VXPT_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= cfg->device) return VXPT_ERR_NODEV;
    auto *c = new vxpt_ctx();
    c->W = cfg->width; c->H = cfg->height; c->dev = cfg->device;
    c->rowBegin = cfg->row_begin; c->rowEnd = cfg->row_end;
    if (c->rowEnd <= c->rowBegin) { c->rowBegin = 0; c->rowEnd = c->H; }
    if (cfg->total_bounce_limit > 0) c->totalBounce = cfg->total_bounce_limit;
    if (cfg->diffuse_bounce_limit > 0) c->diffuseBounce = cfg->diffuse_bounce_limit;
    c->dataDir = cfg->data_dir ? cfg->data_dir : "data";
    c->yamlPost = default_post();
    c->yamlDenoise = default_denoise();
    *out = c;
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (hipStream_t &fs : c->frontStreams) HIPCHK(c, hipStreamCreateWithFlags(&fs, hipStreamNonBlocking));
    // tuning state_sets = 3: a third wavefront state set, so a first half may run beside the two
    // previous second halves (C3: 6.40 -> 6.39 ms per frame, within noise: the overlapped halves
    // already fill the chip; two sets are the default)
    for (int k = 0; k < kMaxSets; ++k)
        for (hipEvent_t *e : {&c->frontDone[k], &c->backDone[k]})
            HIPCHK(c, hipEventCreateWithFlags(e, hipEventDisableTiming | hipEventDisableSystemFence));
    HIPCHK(c, hipEventCreateWithFlags(&c->frontGate, hipEventDisableTiming | hipEventDisableSystemFence));
    HIPCHK(c, hipDeviceGetAttribute(&c->numCU, hipDeviceAttributeMultiprocessorCount, c->dev));
    // timing markers only (every read of them follows a stream synchronisation): no system-scope
    // fence, so a marker neither writes back / invalidates the L2 nor delays the next kernel
    for (auto &e : c->ev) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    const size_t n = (size_t)c->W * c->H;
    const size_t tiles16 = (size_t)((c->W + 15) / 16) * ((c->H + 15) / 16);  // denoiser tiles
    for (auto &g : c->gb) {
        if (dalloc(c, g.normalRough, n) || dalloc(c, g.geoNormalThin, n) || dalloc(c, g.albedo, n) ||
            dalloc(c, g.matParam, n) || dalloc(c, g.depth, n) || dalloc(c, g.material, n) || dalloc(c, g.rec, 2 * n))
            return VXPT_ERR_HIP;
    }
    if (dalloc(c, c->illum, n) || dalloc(c, c->accum, n) || dalloc(c, c->motion, n) || dalloc(c, c->res, 2 * n) ||
        dalloc(c, c->ping, n) || dalloc(c, c->pong, n) || dalloc(c, c->prevIllum, n) || dalloc(c, c->prevFast, n) ||
        dalloc(c, c->output, n) || dalloc(c, c->histLen, n) || dalloc(c, c->prevHistLen, n) ||
        dalloc(c, c->wpos, n) || dalloc(c, c->ffCount, tiles16) || dalloc(c, c->ffIndex, tiles16 * 256) ||
        dalloc(c, c->ffColor, tiles16 * 256) || dalloc(c, c->ffRes, tiles16 * 256) ||
        dalloc(c, c->ffCand, tiles16 * 256) || dalloc(c, c->ffCandCount, 1) ||
        dalloc(c, c->hfList, tiles16 * 256) || dalloc(c, c->hfCount, tiles16))
        return VXPT_ERR_HIP;
    c->illumSet[0] = c->illum;
    c->accumBuf[0] = c->accum;
    if (dalloc(c, c->accumBuf[1], n)) return VXPT_ERR_HIP;
    for (int k = 1; k < kMaxSets; ++k)  // (a third set's plane too: vxpt_set_tuning may enable it)
        if (dalloc(c, c->illumSet[k], n)) return VXPT_ERR_HIP;
    // tables
    const std::string t = c->dataDir + "/tables/";
    std::vector<uint8_t> so, sc, rk, f0, f1, f2, f3;
    if (!read_file(t + "bn_sobol.u8", so) || !read_file(t + "bn_scramble.u8", sc) || !read_file(t + "bn_rank.u8", rk) ||
        !read_file(t + "sky_datasets.f32", f0) || !read_file(t + "sky_datasets_rad.f32", f1) ||
        !read_file(t + "solar_datasets.f32", f2) || !read_file(t + "limb_darkening.f32", f3) ||
        so.size() != 65536 || sc.size() != 131072 || rk.size() != 131072 || f0.size() != 2160 || f1.size() != 240 ||
        f2.size() != 7200 || f3.size() != 240)
        return fail(c, VXPT_ERR_IO, "cannot read tables from " + t);
    if (upload_vec(c, c->bnSobol, so.data(), so.size()) || upload_vec(c, c->bnScramble, sc.data(), sc.size()) ||
        upload_vec(c, c->bnRank, rk.data(), rk.size()) ||
        upload_vec(c, c->solar, (const float *)f2.data(), 1800) || upload_vec(c, c->limb, (const float *)f3.data(), 60))
        return VXPT_ERR_HIP;
    std::memcpy(c->tabSky, f0.data(), sizeof(c->tabSky));
    std::memcpy(c->tabSkyRad, f1.data(), sizeof(c->tabSkyRad));
    // default material table: terrain materials of data/assets/materials.yaml
    const float rough[13] = {0.5f, 0.8f, 0.9f, 0.85f, 0.9f, 0.8f, 0.7f, 0.85f, 0.6f, 0.7f, 0.65f, 0.75f, 0.75f};
    for (int b = 1; b <= 12; ++b) c->mats[b] = MatDev{{1.f, 1.f, 1.f}, rough[b], 0.0f, 0, b - 1, 0};
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VXPT_OK;
}

void vxpt_destroy(vxpt_ctx *c) {
    if (!c) return;
    hipSetDevice(c->dev);
    for (hipStream_t fs : c->frontStreams)
        if (fs) hipStreamSynchronize(fs);
    if (c->stream) hipStreamSynchronize(c->stream);
    for (void *p : c->allocs) hipFree(p);
    for (int k = 0; k < kMaxSets; ++k)
        for (hipEvent_t e : {c->frontDone[k], c->backDone[k]})
            if (e) hipEventDestroy(e);
    if (c->frontGate) hipEventDestroy(c->frontGate);
    for (hipStream_t fs : c->frontStreams)
        if (fs) hipStreamDestroy(fs);
    for (hipEvent_t e : c->chainEv) hipEventDestroy(e);
    for (hipEvent_t e : c->bst.pool) hipEventDestroy(e);
    for (auto &e : c->ev)
        if (e) hipEventDestroy(e);
    for (auto &e : c->runEv)
        if (e) hipEventDestroy(e);
    if (c->stream) hipStreamDestroy(c->stream);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->commStream) hipStreamDestroy(c->commStream);
    if (c->haloReady) hipEventDestroy(c->haloReady);
    if (c->haloDone) hipEventDestroy(c->haloDone);
    if (c->exDone) hipEventDestroy(c->exDone);
    delete c;
}

int vxpt_load_settings(vxpt_ctx *c) {
    if (!c) return VXPT_ERR_ARG;
    // global_settings.yaml: denoising + sky sections (GlobalSettings.cpp:69-492)
    std::ifstream f(c->dataDir + "/settings/global_settings.yaml");
    if (!f) return fail(c, VXPT_ERR_IO, "missing settings/global_settings.yaml");
    vxpt_denoise_params d = default_denoise();
    vxpt_post_params pp = default_post();
    std::string line, section;
    while (std::getline(f, line)) {
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        if (trim(line).empty()) continue;
        const bool indented = line[0] == ' ' || line[0] == '\t';
        const size_t col = line.find(':');
        if (col == std::string::npos) continue;
        const std::string key = trim(line.substr(0, col)), val = trim(line.substr(col + 1));
        if (!indented) { section = key; continue; }
        if (section == "denoising") {
            const float v = (float)std::atof(val.c_str());
            if (key == "enableTemporalAccumulation") d.enable_temporal_accumulation = as_bool(val);
            else if (key == "enableHistoryFix") d.enable_history_fix = as_bool(val);
            else if (key == "enableHistoryClamping") d.enable_history_clamping = as_bool(val);
            else if (key == "enableSpatialFiltering") d.enable_spatial_filtering = as_bool(val);
            else if (key == "enableFireflyFilter") d.enable_firefly_filter = as_bool(val);
            else if (key == "maxAccumulatedFrameNum") d.max_accumulated_frame_num = v;
            else if (key == "maxFastAccumulatedFrameNum") d.max_fast_accumulated_frame_num = v;
            else if (key == "phiLuminance") d.phi_luminance = v;
            else if (key == "lobeAngleFraction") d.lobe_angle_fraction = v;
            else if (key == "roughnessFraction") d.roughness_fraction = v;
            else if (key == "depthThreshold") d.depth_threshold = v;
            else if (key == "atrousIterationNum") d.atrous_iteration_num = (int)v;
            else if (key == "disocclusionThreshold") d.disocclusion_threshold = v;
            else if (key == "disocclusionThresholdAlternate") d.disocclusion_threshold_alternate = v;
            else if (key == "denoisingRange") d.denoising_range = v;
        } else if (section == "postprocess") {  // GlobalSettings.cpp:277-355
            const float v = (float)std::atof(val.c_str());
            const int b = as_bool(val) ? 1 : 0;
            if (key == "manualExposure") pp.manual_exposure = v;
            else if (key == "toneMappingCurve") pp.tone_mapping_curve = (int)v;
            else if (key == "whitePoint") pp.white_point = v;
            else if (key == "contrast") pp.contrast = v;
            else if (key == "saturation") pp.saturation = v;
            else if (key == "gain") pp.gain = v;
            else if (key == "lift") pp.lift = v;
            else if (key == "enableBloom") pp.enable_bloom = b;
            else if (key == "bloomThreshold") pp.bloom_threshold = v;
            else if (key == "bloomIntensity") pp.bloom_intensity = v;
            else if (key == "bloomRadius") pp.bloom_radius = v;
            else if (key == "enableAutoExposure") pp.enable_auto_exposure = b;
            else if (key == "exposureSpeed") pp.exposure_speed = v;
            else if (key == "exposureMin") pp.exposure_min = v;
            else if (key == "exposureMax") pp.exposure_max = v;
            else if (key == "exposureCompensation") pp.exposure_compensation = v;
            else if (key == "histogramMinPercent") pp.histogram_min_percent = v;
            else if (key == "histogramMaxPercent") pp.histogram_max_percent = v;
            else if (key == "targetLuminance") pp.target_luminance = v;
            else if (key == "enableVignette") pp.enable_vignette = b;
            else if (key == "vignetteStrength") pp.vignette_strength = v;
            else if (key == "vignetteRadius") pp.vignette_radius = v;
            else if (key == "vignetteSmoothness") pp.vignette_smoothness = v;
            else if (key == "enableLensFlare") pp.enable_lens_flare = b;
            else if (key == "lensFlareIntensity") pp.lens_flare_intensity = v;
            else if (key == "lensFlareGhostSpacing") pp.lens_flare_ghost_spacing = v;
            else if (key == "lensFlareGhostCount") pp.lens_flare_ghost_count = (int)v;
            else if (key == "lensFlareHaloRadius") pp.lens_flare_halo_radius = v;
            else if (key == "lensFlareSunSize") pp.lens_flare_sun_size = v;
            else if (key == "lensFlareDistortion") pp.lens_flare_distortion = v;
        } else if (section == "sky") {
            const float v = (float)std::atof(val.c_str());
            if (key == "timeOfDay") c->skyParams[0] = v;
            else if (key == "sunAxisAngle") c->skyParams[1] = v;
            else if (key == "sunAxisRotate") c->skyParams[2] = v;
            else if (key == "skyBrightness") c->skyParams[3] = v;
        }
    }
    c->yamlDenoise = d;
    c->yamlPost = pp;
    // materials.yaml (order == material index, MaterialManager.cpp:84-97) + blocks.yaml
    std::ifstream fm(c->dataDir + "/assets/materials.yaml");
    if (!fm) return fail(c, VXPT_ERR_IO, "missing assets/materials.yaml");
    std::vector<std::string> ids;
    std::vector<std::map<std::string, std::string>> props, texs;
    while (std::getline(fm, line)) {
        const std::string tl = trim(line);
        if (tl.rfind("- id:", 0) == 0) {
            ids.push_back(trim(tl.substr(5)));
            props.emplace_back();
            texs.emplace_back();
        } else if (tl.rfind("properties:", 0) == 0 && !props.empty()) {
            props.back() = parse_flow_map(tl);
        } else if (tl.rfind("textures:", 0) == 0 && !texs.empty()) {
            texs.back() = parse_flow_map(tl);
        }
    }
    std::ifstream fb(c->dataDir + "/assets/blocks.yaml");
    if (!fb) return fail(c, VXPT_ERR_IO, "missing assets/blocks.yaml");
    while (std::getline(fb, line)) {
        const std::string tl = trim(line);
        if (tl.rfind("- {", 0) != 0) continue;
        auto m = parse_flow_map(tl);
        const int bid = std::atoi(m["id"].c_str());
        if (bid < 1 || bid > 12) continue;
        const auto it = std::find(ids.begin(), ids.end(), m["material"]);
        if (it == ids.end()) continue;
        const int mi = (int)(it - ids.begin());
        auto &p = props[mi];
        MatDev md{{1.f, 1.f, 1.f}, 0.5f, 0.0f, 0, mi, 0};  // MaterialProperties defaults (MaterialDefinition.h:18-28)
        if (p.count("roughness")) md.roughness = (float)std::atof(p["roughness"].c_str());
        if (p.count("metallic")) md.metallic = std::atof(p["metallic"].c_str()) != 0.0;
        if (p.count("translucency")) md.translucency = (float)std::atof(p["translucency"].c_str());
        if (p.count("is_thinfilm")) md.thin = as_bool(p["is_thinfilm"]);
        if (p.count("albedo")) {
            auto v = parse_list(p["albedo"]);
            if (v.size() == 3) { md.albedo[0] = v[0]; md.albedo[1] = v[1]; md.albedo[2] = v[2]; }
        }
        if (p.count("uv_scale")) md.uvScale = (float)std::atof(p["uv_scale"].c_str());
        if (p.count("use_world_grid_uv")) md.worldGridUV = as_bool(p["use_world_grid_uv"]) ? 1 : 0;
        static const char *kTexKeys[4] = {"albedo", "normal", "roughness", "metallic"};
        for (int k = 0; k < 4; ++k) c->texPath[bid][k] = texs[mi].count(kTexKeys[k]) ? texs[mi][kTexKeys[k]] : "";
        c->mats[bid] = md;
    }
    return VXPT_OK;
}

int vxpt_load_scene_camera(vxpt_ctx *c, const char *path, vxpt_camera *out) {
    if (!c || !out) return VXPT_ERR_ARG;
    std::string p = path ? path : (c->dataDir + "/scene/scene_export.yaml");
    std::ifstream f(p);
    if (!f) return fail(c, VXPT_ERR_IO, "cannot open " + p);
    std::string line, section;
    vxpt_camera cam{{35.6184f, 11.8733f, 42.0387f}, {-0.321564f, -0.0129988f, -0.946799f}, 90.0f};
    while (std::getline(f, line)) {
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        if (trim(line).empty()) continue;
        const size_t col = line.find(':');
        if (col == std::string::npos) continue;
        const std::string key = trim(line.substr(0, col)), val = trim(line.substr(col + 1));
        if (line[0] != ' ') { section = key; continue; }
        if (section != "camera") continue;
        auto v = parse_list(val);
        if (key == "position" && v.size() == 3) std::copy(v.begin(), v.end(), cam.pos);
        else if (key == "direction" && v.size() == 3) std::copy(v.begin(), v.end(), cam.dir);
        else if (key == "fov" && v.size() == 1) cam.fov_deg = v[0];
    }
    *out = cam;
    return VXPT_OK;
}

int vxpt_generate_terrain(vxpt_ctx *c, int cxn, int cyn, int czn, float heightScale, float freqDen, int flags) {
    if (!c || cxn <= 0 || cyn <= 0 || czn <= 0) return VXPT_ERR_ARG;
    const bool keepBalls = (flags & VXPT_TERRAIN_SHADER_BALLS) != 0, globalY = (flags & VXPT_TERRAIN_GLOBAL_Y) != 0;
    std::vector<uint8_t> ids((size_t)cxn * cyn * czn * 32768, 0);
    const Perlin noise(124);
    const float freq = 1.0f / freqDen, width = heightScale;
    for (int ch = 0; ch < cxn * cyn * czn; ++ch) {
        const int gox = (ch % cxn) * 32, goz = ((ch / cxn) % czn) * 32, goy = globalY ? (ch / (cxn * czn)) * 32 : 0;
        float hmap[32][32];
        for (int z = 0; z < 32; ++z)
            for (int x = 0; x < 32; ++x) {
                const float n = noise.octave01((float)(gox + x) * freq, (float)(goz + z) * freq, 4);
                float h = std::fmaf(n, 1.4f, -0.7f);  // nvcc --fmad=true contraction of n*1.4f-0.7f
                h = std::fmax(0.1f, (h + 0.25f) * width);
                hmap[z][x] = std::fmin(h, width * 0.9f);
            }
        for (int y = 0; y < 32; ++y)
            for (int z = 0; z < 32; ++z)
                for (int x = 0; x < 32; ++x) {
                    const float h = hmap[z][x];
                    uint8_t id = 0;
                    const float yy = (float)(goy + y);
                    if (yy < h) {
                        const float d = h - yy;
                        if (h < width * (0.25f + 0.05f)) id = d < 3.5f ? 1 : 7;
                        else if (h < width * (0.25f + 0.6f) && h > width * (0.25f + 0.3f)) id = d < 5.5f ? 3 : 7;
                        else id = d < 1.5f ? 2 : (d < 5.5f ? 3 : 7);
                    }
                    const int gx = gox + x, gz = goz + z;
                    if (keepBalls && y == 7 && gz == 43 && gx >= 30 && gx <= 39) {
                        static const uint8_t ball[10] = {17, 21, 22, 23, 24, 25, 26, 27, 28, 29};
                        id = ball[gx - 30];
                    }
                    ids[(size_t)ch * 32768 + x + 32 * (z + 32 * y)] = id;
                }
    }
    return vxpt_upload_voxels(c, ids.data(), cxn, cyn, czn);
}

int refresh_instances(vxpt_ctx *c, bool lights, bool full);  // instanced meshes (+ lights), after the grid changed

int vxpt_upload_voxels(vxpt_ctx *c, const uint8_t *ids, int cxn, int cyn, int czn) {
    if (!c || !ids || cxn <= 0 || cyn <= 0 || czn <= 0) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    c->cx = cxn; c->cy = cyn; c->cz = czn;
    const size_t n = (size_t)cxn * cyn * czn * 32768;
    c->hIds.assign(ids, ids + n);
    ++c->worldVersion;
    if (int r = upload_vec(c, c->voxels, c->hIds.data(), n)) return r;
    if (int r = build_occupancy(c, c->hIds.data())) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return refresh_instances(c, true, true);
}

int vxpt_upload_materials(vxpt_ctx *c, const vxpt_material *m, int n) {
    if (!c || !m || n < 1 || n >= kBlockTypes) return VXPT_ERR_ARG;
    for (int b = 1; b <= n; ++b) {
        const vxpt_material &s = m[b - 1];
        const MatDev old = c->mats[b];
        c->mats[b] = MatDev{{s.albedo[0], s.albedo[1], s.albedo[2]}, s.roughness, s.translucency, s.metallic,
                            s.material_id, s.thinfilm};
        if (b > 12) {  // instanced blocks keep their emissive / world-grid set-up (vxpt_load_models)
            c->mats[b].emissive = old.emissive;
            c->mats[b].worldGridUV = old.worldGridUV;
            c->mats[b].uvScale = old.uvScale;
        }
    }
    return VXPT_OK;
}

int vxpt_set_sky(vxpt_ctx *c, float tod, float axisAngle, float axisRotate, float brightness) {
    if (!c) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    // sun direction (Sky.cu:363-368)
    V3 axis(1.0f, std::cos(axisAngle * kPiOver180), std::sin(axisAngle * kPiOver180));
    axis *= V3(std::sin(axisRotate * kPiOver180), 1.0f, std::cos(axisRotate * kPiOver180));
    axis = normalize(axis);
    const float angle = std::fmod(tod * kPi, kTwoPi);
    c->sunDir = normalized_c(q_rotate3(axis, angle, cross(V3(0, 1, 0), axis)));
    // updateSkyState (Sky.cu:57-83), CPU fit
    float cfg[90], rad[10];
    const float elevation = (kPi / 2.0f) - std::acos(c->sunDir.y);
    const float se = std::pow(elevation / (kPi / 2.0f), (1.0f / 3.0f));
    for (int ch = 0; ch < 10; ++ch) {
        for (int i = 0; i < 9; ++i) cfg[ch * 9 + i] = fit6(c->tabSky + ch * 54, se, i, 9);
        rad[ch] = fit6(c->tabSkyRad + ch * 6, se, 0, 1);
    }
    const int sw = 1024, sh = 512, uw = 32, uh = 32;
    if (!c->sky.p) {
        if (dalloc(c, c->sky.p, (size_t)sw * sh) || dalloc(c, c->sun.p, (size_t)uw * uh) ||
            dalloc(c, c->skyPdf.p, (size_t)sw * sh) || dalloc(c, c->sunPdf.p, (size_t)uw * uh))
            return VXPT_ERR_HIP;
        c->sky.n = (size_t)sw * sh; c->sun.n = (size_t)uw * uh;
    }
    HIPCHK(c, hipEventRecord(c->ev[4], c->stream));
    HIPCHK(c, launch_sky(cfg, rad, c->solar.p, c->limb.p, c->sunDir, brightness, c->sky.p, c->sun.p, c->skyPdf.p,
                         c->sunPdf.p, sw, sh, uw, uh, c->stream));
    std::vector<float> pdf((size_t)sw * sh), spdf((size_t)uw * uh);
    HIPCHK(c, hipMemcpyAsync(pdf.data() + (size_t)sw * (sh / 2), c->skyPdf.p + (size_t)sw * (sh / 2),
                             (size_t)sw * (sh / 2) * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    double upper = 0.0;
    for (size_t i = (size_t)sw * (sh / 2); i < (size_t)sw * sh; ++i) upper += (double)pdf[i];
    HIPCHK(c, launch_sky_lower(c->sky.p, c->skyPdf.p, sw, sh, (float)upper, c->stream));
    HIPCHK(c, hipMemcpyAsync(pdf.data(), c->skyPdf.p, pdf.size() * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(spdf.data(), c->sunPdf.p, spdf.size() * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipEventRecord(c->ev[5], c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float s1, s2;
    c->hSkyAlias = build_alias(pdf, s1);
    const std::vector<AliasBin> sunA = build_alias(spdf, s2);
    c->sunLuminance = s2;
    if (upload_vec(c, c->skyAlias, c->hSkyAlias.data(), c->hSkyAlias.size()) ||
        upload_vec(c, c->sunAlias, sunA.data(), sunA.size()))
        return VXPT_ERR_HIP;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float ms = 0;
    hipEventElapsedTime(&ms, c->ev[4], c->ev[5]);
    c->timing.sky_ms = ms;
    c->skyReady = true;
    return VXPT_OK;
}

int vxpt_set_camera(vxpt_ctx *c, const vxpt_camera *cur, const vxpt_camera *prev) {
    if (!c || !cur) return VXPT_ERR_ARG;
    c->cam = make_camera(c->W, c->H, *cur, &c->camYaw, &c->camPitch);
    c->prevCam = make_camera(c->W, c->H, prev ? *prev : *cur, nullptr, nullptr);
    return VXPT_OK;
}

// TextureManager::initWithMaterialPaths + LoadTexturesFromPaths (TextureManager.cu:133-330):
// every texture the cube materials name, in sorted path order (= texture id); decoded, square
// power-of-two, expanded to RGBA8 (1 channel -> (v,0,0,1), 2 -> (v,a,0,1), 3 -> (r,g,b,1): the
// unorm reads of the BC4/BC5/BC7 formats), levels 0..log2(size)-2 by 2x2 box averages truncated
// to 8 bits (fillMipmapKernel, :82-117, and its CPU twin, :390-414).  BC7 itself is not
// reproduced (NVTT): the texels are the uncompressed ones.
int vxpt_load_textures(vxpt_ctx *c, const char *root, int *loaded) {
    if (!c) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    const std::string base = root ? root : c->dataDir;
    std::vector<std::string> paths;
    for (int b = 1; b <= 12; ++b)
        for (int k = 0; k < 4; ++k)
            if (!c->texPath[b][k].empty()) paths.push_back(c->texPath[b][k]);
    std::sort(paths.begin(), paths.end());
    paths.erase(std::unique(paths.begin(), paths.end()), paths.end());
    std::vector<uchar4> texels;
    std::vector<TexInfo> table;
    std::map<std::string, int> idOf;
    for (const std::string &pth : paths) {
        int w, h, ch;
        std::vector<uint8_t> px;
        if (!decode_png(base + "/" + pth, w, h, ch, px)) continue;  // the reference skips it too (:180-187)
        if (w != h || w < 4 || (w & (w - 1)) != 0) continue;
        int maxLod = 0;
        while ((4 << maxLod) < w) ++maxLod;  // log2(w) - 2
        if (maxLod >= kMaxTexLevels) continue;
        TexInfo ti{};
        ti.size = w;
        ti.maxLod = maxLod;
        ti.off[0] = (unsigned)texels.size();
        texels.resize(texels.size() + (size_t)w * w);
        uchar4 *l0 = texels.data() + ti.off[0];
        for (size_t i = 0; i < (size_t)w * w; ++i) {
            const uint8_t *q = px.data() + i * ch;
            l0[i] = ch == 1 ? make_uchar4(q[0], 0, 0, 255)
                  : ch == 2 ? make_uchar4(q[0], q[1], 0, 255)
                  : ch == 3 ? make_uchar4(q[0], q[1], q[2], 255) : make_uchar4(q[0], q[1], q[2], q[3]);
        }
        for (int l = 1; l <= maxLod; ++l) {
            const int S = w >> l, P = S * 2;
            ti.off[l] = (unsigned)texels.size();
            texels.resize(texels.size() + (size_t)S * S);
            const uchar4 *src = texels.data() + ti.off[l - 1];
            uchar4 *dst = texels.data() + ti.off[l];
            for (int y = 0; y < S; ++y)
                for (int x = 0; x < S; ++x) {
                    const uchar4 a = src[(2 * y) * P + 2 * x], b2 = src[(2 * y) * P + 2 * x + 1];
                    const uchar4 c2 = src[(2 * y + 1) * P + 2 * x], d = src[(2 * y + 1) * P + 2 * x + 1];
                    dst[y * S + x] = make_uchar4((a.x + b2.x + c2.x + d.x) >> 2, (a.y + b2.y + c2.y + d.y) >> 2,
                                                 (a.z + b2.z + c2.z + d.z) >> 2, (a.w + b2.w + c2.w + d.w) >> 2);
                }
        }
        idOf[pth] = (int)table.size();
        table.push_back(ti);
    }
    for (int b = 1; b <= 12; ++b)
        for (int k = 0; k < 4; ++k) {
            const auto it = idOf.find(c->texPath[b][k]);
            c->mats[b].tex[k] = it == idOf.end() ? -1 : it->second;
        }
    c->hTex = table;
    c->nTexels = texels.size();
    if (!table.empty()) {
        if (int r = upload_vec(c, c->texels, texels.data(), texels.size())) return r;
        if (int r = upload_vec(c, c->texTable, table.data(), table.size())) return r;
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    c->texEnabled = table.empty() ? 0 : 1;
    if (loaded) *loaded = (int)table.size();
    return VXPT_OK;
}

// ---------------------------------------------------------------- instanced meshes + lights
namespace {

// VoxelEngine::collectInstanceTransforms (VoxelEngine.cu:323-384): for every instanced
// object (block 13..29 -> object id = block - 1), every cell holding the block -- or, for a
// light with a paired base, holding the base block -- is an instance of the object; a light
// cell also registers an instance of its base.  Instance id = PositionToInstanceId
// (VoxelMath.h:120-133: first instanced block + object * W^3 + x + W * (z + W * y), every
// coordinate clamped to W - 1, W = the world's x extent); ids are kept in a set per object
// (Scene.h:77) and a later cell with the same id overwrites the transform.
uint32_t instance_id(const vxpt_ctx *c, unsigned obj, unsigned x, unsigned y, unsigned z) {
    int first = kBlockTypes;
    for (int b = 0; b < kBlockTypes; ++b)
        if (c->blocks[b].instanced) { first = b; break; }
    const unsigned W = (unsigned)c->cx * 32u;
    x = x < W - 1 ? x : W - 1;
    y = y < W - 1 ? y : W - 1;
    z = z < W - 1 ? z : W - 1;
    return (unsigned)first + obj * W * W * W + (x + W * (z + W * y));
}

void collect_instances(vxpt_ctx *c) {
    c->instances.clear();
    if (c->hIds.empty()) return;
    int first = kBlockTypes;
    for (int b = 0; b < kBlockTypes; ++b)
        if (c->blocks[b].instanced) { first = b; break; }
    const unsigned W = (unsigned)c->cx * 32u, H = (unsigned)c->cy * 32u, D = (unsigned)c->cz * 32u;
    std::map<int, std::map<unsigned, std::array<unsigned, 3>>> byObject;
    auto inst_id = [&](unsigned obj, unsigned x, unsigned y, unsigned z) { return instance_id(c, obj, x, y, z); };
    // one pass over the cells: what each block id contributes (its own object; a base block
    // also the objects of the lights paired with it; a paired light also its base's object)
    std::vector<int> contrib[kBlockTypes];
    for (int obj = first - 1; obj < kBlockTypes - 1; ++obj) {
        const int block = obj + 1, base = c->blocks[block].lightBase;
        contrib[block].push_back(obj);
        if (base > 0 && base < kBlockTypes) {
            contrib[base].push_back(obj);
            contrib[block].push_back(base - 1);
        }
    }
    for (unsigned x = 0; x < W; ++x)  // the reference's x, y, z order (last write wins)
        for (unsigned y = 0; y < H; ++y)
            for (unsigned z = 0; z < D; ++z) {
                const size_t ch = (x >> 5) + (size_t)c->cx * ((z >> 5) + (size_t)c->cz * (y >> 5));
                const int id = c->hIds[ch * 32768 + (x & 31) + 32 * ((z & 31) + 32 * (y & 31))];
                if (id < first || id >= kBlockTypes) continue;
                for (int obj : contrib[id]) byObject[obj][inst_id(obj, x, y, z)] = {x, y, z};
            }
    for (const auto &o : byObject)
        for (const auto &i : o.second)
            c->instances.insert(c->instances.end(),
                                {o.first, (int32_t)i.first, (int32_t)i.second[0], (int32_t)i.second[1], (int32_t)i.second[2]});
}

// VoxelEngine::countLightTriangles / generateInstanceLights (VoxelEngine.cu:386-520) and
// buildAliasTable (:150-192): the emissive objects in object order, each instance's
// triangles in a row, one launch per object; then the weights' alias table (build_alias,
// the same construction as the sky's) and their sum (accumulatedLocalLightLuminance).
int build_lights(vxpt_ctx *c) {
    c->lightMap.clear();
    c->nLights = 0;
    c->localLightLum = 0.0f;
    size_t total = 0;
    for (size_t k = 0; k < c->instances.size(); k += 5) {
        const auto &bd = c->blocks[c->instances[k] + 1];
        if (bd.emissive) total += (size_t)bd.triangles;
    }
    if (total == 0) return VXPT_OK;
    if (c->lights.n < total) {
        if (dalloc(c, c->lights.p, total)) return VXPT_ERR_HIP;
        c->lights.n = total;
    }
    if (c->lightWeight.n < total) {
        if (dalloc(c, c->lightWeight.p, total)) return VXPT_ERR_HIP;
        c->lightWeight.n = total;
    }
    // all emissive meshes' triangles and instance cells, uploaded once
    std::vector<float> tri;
    std::vector<int> cells;
    struct Run { size_t tri, cell; int nTri, nInst; V3 rad; };
    std::vector<Run> runs;
    for (size_t k = 0; k < c->instances.size();) {
        const int obj = c->instances[k];
        const auto &bd = c->blocks[obj + 1];
        size_t e = k;
        while (e < c->instances.size() && c->instances[e] == obj) e += 5;
        if (bd.emissive && bd.triangles > 0) {
            Run r{tri.size(), cells.size(), bd.triangles, (int)((e - k) / 5),
                  V3(bd.emission[0], bd.emission[1], bd.emission[2])};
            tri.insert(tri.end(), bd.pos.begin(), bd.pos.end());
            for (size_t i = k; i < e; i += 5) {
                cells.insert(cells.end(), {c->instances[i + 2], c->instances[i + 3], c->instances[i + 4]});
                c->lightMap.insert(c->lightMap.end(),
                                   {(uint32_t)c->instances[i + 1], (uint32_t)c->nLights, (uint32_t)bd.triangles});
                c->nLights += (unsigned)bd.triangles;
            }
            runs.push_back(r);
        }
        k = e;
    }
    if (int r = upload_vec(c, c->lightTri, tri.data(), tri.size())) return r;
    if (int r = upload_vec(c, c->lightInst, cells.data(), cells.size())) return r;
    size_t off = 0;
    for (const Run &r : runs) {
        HIPCHK(c, launch_tri_lights(c->lightTri.p + r.tri, r.nTri, c->lightInst.p + r.cell, r.nInst, r.rad,
                                    c->lights.p + off, c->lightWeight.p + off, c->stream));
        off += (size_t)r.nTri * r.nInst;
    }
    std::vector<float> w(total);
    HIPCHK(c, hipMemcpyAsync(w.data(), c->lightWeight.p, total * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const std::vector<AliasBin> bins = build_alias(w, c->localLightLum);
    if (int r = upload_vec(c, c->lightAlias, bins.data(), bins.size())) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VXPT_OK;
}

}  // namespace

// every loaded mesh's BLAS (object space), concatenated
int build_blas(vxpt_ctx *c) {
    c->hBlas.clear();
    c->hBlasTri.clear();
    c->hBlasUV.clear();
    c->hBlasTriId.clear();
    c->hRoot.assign(kBlockTypes, make_int2(-1, -1));
    for (int b = 0; b < kBlockTypes; ++b) {
        const auto &bd = c->blocks[b];
        if (!bd.instanced || bd.triangles == 0) continue;
        std::vector<float> box((size_t)bd.triangles * 6);
        for (int t = 0; t < bd.triangles; ++t)
            for (int k = 0; k < 3; ++k) {
                const float *v = &bd.pos[(size_t)t * 9];
                box[(size_t)t * 6 + k] = std::min(v[k], std::min(v[3 + k], v[6 + k]));
                box[(size_t)t * 6 + 3 + k] = std::max(v[k], std::max(v[3 + k], v[6 + k]));
            }
        std::vector<BvhNode> nodes;
        std::vector<int> order;
        int depth = 0;
        if (!build_bvh(box, 4, nodes, order, &depth)) return fail(c, VXPT_ERR_STATE, "mesh BVH too deep");
        c->hRoot[b] = make_int2((int)c->hBlas.size(), (int)c->hBlasTriId.size());
        c->hBlas.insert(c->hBlas.end(), nodes.begin(), nodes.end());
        for (int t : order) {
            c->hBlasTri.insert(c->hBlasTri.end(), bd.pos.begin() + (size_t)t * 9, bd.pos.begin() + (size_t)t * 9 + 9);
            c->hBlasUV.insert(c->hBlasUV.end(), bd.uv.begin() + (size_t)t * 6, bd.uv.begin() + (size_t)t * 6 + 6);
            c->hBlasTriId.push_back(t);
        }
    }
    if (!c->hBlas.empty()) {
        if (int r = upload_vec(c, c->blas, c->hBlas.data(), c->hBlas.size())) return r;
        if (int r = upload_vec(c, c->blasTri, c->hBlasTri.data(), c->hBlasTri.size())) return r;
        if (int r = upload_vec(c, c->blasUV, c->hBlasUV.data(), c->hBlasUV.size())) return r;
        if (int r = upload_vec(c, c->blasTriId, c->hBlasTriId.data(), c->hBlasTriId.size())) return r;
    }
    return upload_vec(c, c->blasRoot, c->hRoot.data(), c->hRoot.size());
}

// the world's TLAS over the instances whose block type has a mesh
int build_tlas(vxpt_ctx *c) {
    std::vector<MeshInst> mi;
    std::vector<float> box;
    for (size_t k = 0; k < c->instances.size(); k += 5) {
        const int block = c->instances[k] + 1;
        const int2 r = c->hRoot.empty() ? make_int2(-1, -1) : c->hRoot[block];
        if (r.x < 0) continue;
        const BvhNode &root = c->hBlas[r.x];
        const float cell[3] = {(float)c->instances[k + 2], (float)c->instances[k + 3], (float)c->instances[k + 4]};
        mi.push_back(MeshInst{{cell[0], cell[1], cell[2]}, block, (int)(k / 5)});
        for (int a = 0; a < 3; ++a) box.push_back(root.lo[a] + cell[a]);
        for (int a = 0; a < 3; ++a) box.push_back(root.hi[a] + cell[a]);
    }
    std::vector<BvhNode> nodes;
    std::vector<int> order;
    int depth = 0;
    if (!build_bvh(box, 2, nodes, order, &depth)) return fail(c, VXPT_ERR_STATE, "instance BVH too deep");
    std::vector<MeshInst> sorted;
    for (int i : order) sorted.push_back(mi[i]);
    c->nMeshInst = (int)sorted.size();
    if (c->nMeshInst == 0) return VXPT_OK;
    if (int r = upload_vec(c, c->tlas, nodes.data(), nodes.size())) return r;
    return upload_vec(c, c->meshInst, sorted.data(), sorted.size());
}

// VoxelEngine::updateLight (VoxelEngine.cu:658-709) after the light table was rebuilt from
// prevN lights: the remap table (light_map.hpp), uploaded for the next trace pass, which applies
// it to the previous reservoirs (Restir.h:48-79).
int light_update(vxpt_ctx *c, unsigned prevN) {
    const std::vector<int> remap = light_id_map(c->lightState, c->lightMap, prevN, c->nLights);
    if (prevN > 0) {
        if (int r = upload_vec(c, c->lightRemap, remap.data(), remap.size())) return r;
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    c->prevNumLights = prevN;
    c->lightsDirty = 1;
    return VXPT_OK;
}

// lights: rebuild the light table as a light update (full: scene init / reload; otherwise of the
// type the edits made it), or keep it (an edit of no emissive block, VoxelEngine.cu:1206, 1278)
int refresh_instances(vxpt_ctx *c, bool lights, bool full) {
    if (!c->modelsLoaded) return VXPT_OK;
    collect_instances(c);
    if (int r = build_tlas(c)) return r;
    if (lights) {
        if (full) c->lightState.incremental = false;
        const unsigned prevN = c->nLights;
        if (int r = build_lights(c)) return r;
        if (int r = light_update(c, prevN)) return r;
    }
    // per instance row: cell + block, and its first light record (-1: not an emissive instance)
    const size_t n = c->instances.size() / 5;
    if (n == 0) return VXPT_OK;
    std::vector<int4> rows(n);
    std::vector<int> rowLight(n, -1);
    std::map<uint32_t, int> firstLight;
    for (size_t k = 0; k < c->lightMap.size(); k += 3) firstLight[c->lightMap[k]] = (int)c->lightMap[k + 1];
    for (size_t i = 0; i < n; ++i) {
        const int32_t *r = &c->instances[i * 5];
        rows[i] = make_int4(r[2], r[3], r[4], r[0] + 1);
        // the light mapping is by instance id within the emissive object's run (closesthit.cu:869-899)
        const auto it = firstLight.find((uint32_t)r[1]);
        if (it != firstLight.end() && c->blocks[r[0] + 1].emissive) rowLight[i] = it->second;
    }
    if (int r = upload_vec(c, c->meshRow, rows.data(), rows.size())) return r;
    return upload_vec(c, c->meshRowLight, rowLight.data(), rowLight.size());
}

static MeshDev mesh_dev(const vxpt_ctx *c) {
    return MeshDev{c->tlas.p, c->meshInst.p, c->blas.p, c->blasTri.p, c->blasTriId.p, c->blasRoot.p, c->nMeshInst};
}

// closest instanced-mesh hit of n rays (8 floats each: o, tmin, d, tmax): out 4 floats (t, u, v,
// hit), ids 2 ints (instance row, triangle)
int vxpt_mesh_probe(vxpt_ctx *c, const float *rays, int n, int cull, float *out, int32_t *ids) {
    if (!c || !rays || !out || !ids || n < 0) return VXPT_ERR_ARG;
    if (n == 0) return VXPT_OK;
    HIPCHK(c, hipSetDevice(c->dev));
    if (c->hRoot.empty()) c->hRoot.assign(kBlockTypes, make_int2(-1, -1));
    if (!c->blasRoot.p)
        if (int r = upload_vec(c, c->blasRoot, c->hRoot.data(), c->hRoot.size())) return r;
    // the probe's scratch grows with the largest call and lives with the context
    if (int r = upload_vec(c, c->probeRays, rays, (size_t)n * 8)) return r;
    if (grow(c, c->probeOut, (size_t)n * 4) || grow(c, c->probeIds, (size_t)n * 2)) return VXPT_ERR_HIP;
    HIPCHK(c, launch_mesh_probe(mesh_dev(c), c->probeRays.p, n, cull, c->probeOut.p, c->probeIds.p, c->stream));
    HIPCHK(c, hipMemcpyAsync(out, c->probeOut.p, (size_t)n * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(ids, c->probeIds.p, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VXPT_OK;
}

// visibility rays against the instanced meshes: occluded[i] = 1 iff any triangle, either face,
// lies in [tmin, tmax] of ray i (8 floats: o, tmin, d, tmax)
int vxpt_mesh_occluded(vxpt_ctx *c, const float *rays, int n, uint8_t *occluded) {
    if (!c || !rays || !occluded || n < 0) return VXPT_ERR_ARG;
    if (n == 0) return VXPT_OK;
    HIPCHK(c, hipSetDevice(c->dev));
    if (c->hRoot.empty()) c->hRoot.assign(kBlockTypes, make_int2(-1, -1));
    if (!c->blasRoot.p)
        if (int r = upload_vec(c, c->blasRoot, c->hRoot.data(), c->hRoot.size())) return r;
    if (int r = upload_vec(c, c->probeRays, rays, (size_t)n * 8)) return r;
    if (grow(c, c->probeOcc, (size_t)n)) return VXPT_ERR_HIP;
    HIPCHK(c, launch_mesh_occluded(mesh_dev(c), c->probeRays.p, n, c->probeOcc.p, c->stream));
    HIPCHK(c, hipMemcpyAsync(occluded, c->probeOcc.p, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VXPT_OK;
}

// blocks.yaml (ids 13..29) + models.yaml + materials.yaml emission, then the OBJ meshes
int vxpt_load_models(vxpt_ctx *c, const char *root, int *loaded) {
    if (!c) return VXPT_ERR_ARG;
    const std::string dir = root ? root : c->dataDir;
    std::string line;
    std::map<std::string, std::string> modelFile;
    {
        std::ifstream f(c->dataDir + "/assets/models.yaml");
        if (!f) return fail(c, VXPT_ERR_IO, "missing assets/models.yaml");
        while (std::getline(f, line)) {
            const std::string tl = trim(line);
            if (tl.rfind("- {", 0) != 0) continue;
            auto m = parse_flow_map(tl);
            modelFile[m["id"]] = m["file"];
        }
    }
    std::map<std::string, std::map<std::string, std::string>> matProps;
    std::map<std::string, int> matIndex;  // MaterialParameter.materialId: the material's index in materials.yaml
    {
        std::ifstream f(c->dataDir + "/assets/materials.yaml");
        if (!f) return fail(c, VXPT_ERR_IO, "missing assets/materials.yaml");
        std::string cur;
        while (std::getline(f, line)) {
            const std::string tl = trim(line);
            if (tl.rfind("- id:", 0) == 0) {
                cur = trim(tl.substr(5));
                const int k = (int)matIndex.size();
                matIndex.emplace(cur, k);
            } else if (tl.rfind("properties:", 0) == 0) {
                matProps[cur] = parse_flow_map(tl);
            }
        }
    }
    std::ifstream fb(c->dataDir + "/assets/blocks.yaml");
    if (!fb) return fail(c, VXPT_ERR_IO, "missing assets/blocks.yaml");
    for (auto &b : c->blocks) b = vxpt_ctx::BlockDef{};
    int nLoaded = 0;
    while (std::getline(fb, line)) {
        const std::string tl = trim(line);
        if (tl.rfind("- {", 0) != 0) continue;
        auto m = parse_flow_map(tl);
        const int bid = std::atoi(m["id"].c_str());
        if (bid < 1 || bid >= kBlockTypes) continue;
        auto &bd = c->blocks[bid];
        bd.instanced = as_bool(m["instanced"]);
        bd.baseLight = as_bool(m["base_light"]);
        bd.lightBase = m.count("light_base") ? std::atoi(m["light_base"].c_str()) : 0;
        bd.model = m.count("model") ? m["model"] : "";
        // BlockManager::isEmissive: the block's flag or its material's; radiance from the material
        auto &mp = matProps[m["material"]];
        bd.emissive = as_bool(m["emissive"]) || as_bool(mp["is_emissive"]);
        if (as_bool(mp["is_emissive"]) && mp.count("emissive_radiance")) {
            const auto v = parse_list(mp["emissive_radiance"]);
            if (v.size() == 3) std::copy(v.begin(), v.end(), bd.emission);
        }
        if (bd.instanced) {
            // MaterialManager::createMaterialParameter (MaterialManager.cpp:150-190) for the mesh's
            // shading: an emissive material's albedo is its radiance (no textures on mesh materials here)
            MatDev md{{1.f, 1.f, 1.f}, 0.5f, 0.0f, 0, matIndex.count(m["material"]) ? matIndex[m["material"]] : 0, 0};
            if (mp.count("albedo")) {
                const auto v = parse_list(mp["albedo"]);
                if (v.size() == 3) std::copy(v.begin(), v.end(), md.albedo);
            }
            if (mp.count("roughness")) md.roughness = (float)std::atof(mp["roughness"].c_str());
            if (mp.count("metallic")) md.metallic = std::atof(mp["metallic"].c_str()) != 0.0;
            if (mp.count("translucency")) md.translucency = (float)std::atof(mp["translucency"].c_str());
            if (mp.count("is_thinfilm")) md.thin = as_bool(mp["is_thinfilm"]);
            if (mp.count("uv_scale")) md.uvScale = (float)std::atof(mp["uv_scale"].c_str());
            if (mp.count("use_world_grid_uv")) md.worldGridUV = as_bool(mp["use_world_grid_uv"]) ? 1 : 0;
            md.emissive = as_bool(mp["is_emissive"]) ? 1 : 0;
            if (md.emissive) std::copy(bd.emission, bd.emission + 3, md.albedo);
            c->mats[bid] = md;
        }
        if (!bd.instanced || bd.model.empty() || !modelFile.count(bd.model)) continue;
        if (load_obj(dir + "/" + modelFile[bd.model], bd.pos, bd.uv)) {
            bd.triangles = (int)(bd.pos.size() / 9);
            bd.pos.resize((size_t)bd.triangles * 9);
            bd.uv.resize((size_t)bd.triangles * 6);
            if (bd.triangles > 0) ++nLoaded;
        }
    }
    c->modelsLoaded = true;
    if (loaded) *loaded = nLoaded;
    // the farthest any loaded mesh reaches outside its unit cell (its instance is the cell's
    // translation): banded frames bound the primary hits' distance with it (nearest_surface)
    c->meshGrow = 1.0f;
    for (int b = 0; b < kBlockTypes; ++b)
        for (float v : c->blocks[b].pos) c->meshGrow = std::max(c->meshGrow, std::max(-v, v - 1.0f));
    ++c->worldVersion;  // a cached nearest-surface search used the old growth
    HIPCHK(c, hipSetDevice(c->dev));
    if (int r = build_blas(c)) return r;
    return refresh_instances(c, true, true);
}

int vxpt_get_model(vxpt_ctx *c, int block_id, float *pos, float *uv, int cap_triangles, int *n_triangles) {
    if (!c || block_id < 0 || block_id >= kBlockTypes) return VXPT_ERR_ARG;
    const auto &bd = c->blocks[block_id];
    if (n_triangles) *n_triangles = bd.triangles;
    const int n = std::min(cap_triangles, bd.triangles);
    if (pos && n > 0) std::copy(bd.pos.begin(), bd.pos.begin() + (size_t)n * 9, pos);
    if (uv && n > 0) std::copy(bd.uv.begin(), bd.uv.begin() + (size_t)n * 6, uv);
    return VXPT_OK;
}

int vxpt_get_instances(vxpt_ctx *c, int32_t *out, int cap, int *n_instances) {
    if (!c) return VXPT_ERR_ARG;
    const int n = (int)(c->instances.size() / 5);
    if (n_instances) *n_instances = n;
    if (out) std::copy(c->instances.begin(), c->instances.begin() + (size_t)std::min(cap, n) * 5, out);
    return VXPT_OK;
}

int vxpt_get_light_remap(vxpt_ctx *c, int32_t *remap, int cap, int *prev_num_lights, int *pending) {
    if (!c || cap < 0) return VXPT_ERR_ARG;
    if (prev_num_lights) *prev_num_lights = (int)c->prevNumLights;
    if (pending) *pending = c->lightsDirty;
    const int n = std::min(cap, (int)c->prevNumLights);
    if (remap && n > 0) {
        HIPCHK(c, hipSetDevice(c->dev));
        HIPCHK(c, hipMemcpyAsync(remap, c->lightRemap.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return VXPT_OK;
}

int vxpt_get_lights(vxpt_ctx *c, uint32_t *mapping, int cap, int *n_mapped, uint32_t *n_lights, float *local_luminance) {
    if (!c) return VXPT_ERR_ARG;
    const int n = (int)(c->lightMap.size() / 3);
    if (n_mapped) *n_mapped = n;
    if (mapping) std::copy(c->lightMap.begin(), c->lightMap.begin() + (size_t)std::min(cap, n) * 3, mapping);
    if (n_lights) *n_lights = c->nLights;
    if (local_luminance) *local_luminance = c->localLightLum;
    return VXPT_OK;
}

int vxpt_enable_textures(vxpt_ctx *c, int on) {
    if (!c) return VXPT_ERR_ARG;
    c->texEnabled = (on && !c->hTex.empty()) ? 1 : 0;
    return VXPT_OK;
}

// the loaded table: per texture size, maxLod, then maxLod + 1 level offsets (in texels)
int vxpt_texture_table(vxpt_ctx *c, int32_t *out, int cap, int *n_textures, int64_t *n_texels) {
    if (!c) return VXPT_ERR_ARG;
    int k = 0;
    for (const TexInfo &t : c->hTex) {
        if (out && k + 2 + t.maxLod + 1 > cap) return VXPT_ERR_ARG;
        if (out) {
            out[k] = t.size;
            out[k + 1] = t.maxLod;
            for (int l = 0; l <= t.maxLod; ++l) out[k + 2 + l] = (int32_t)t.off[l];
        }
        k += 2 + t.maxLod + 1;
    }
    if (n_textures) *n_textures = (int)c->hTex.size();
    if (n_texels) *n_texels = (int64_t)c->nTexels;
    return VXPT_OK;
}

int vxpt_set_camera_angles(vxpt_ctx *c, const float pos[3], float yaw, float pitch, float fovDeg) {
    if (!c || !pos) return VXPT_ERR_ARG;
    c->prevCam = c->cam;  // historyCamera = camera (mainOffline.cpp:278-279)
    c->cam = make_camera_angles(c->W, c->H, pos, yaw, pitch, fovDeg);
    c->camYaw = yaw;
    c->camPitch = pitch;
    return VXPT_OK;
}

// VoxelEngine::performRayTraversal (VoxelEngine.cu:1040-1166): a unit-step walk of the camera
// ray over the host grid; the last empty cell before the first non-empty one is where a block
// would be placed.  out: hit, hit x, y, z, hit id, has space, place x, y, z, cells walked
int vxpt_pick_block(vxpt_ctx *c, int32_t out[10]) {
    if (!c || !out) return VXPT_ERR_ARG;
    if (c->hIds.empty()) return fail(c, VXPT_ERR_STATE, "no voxels uploaded");
    for (int i = 0; i < 10; ++i) out[i] = 0;
    const int W = c->cx * 32, H = c->cy * 32, D = c->cz * 32;
    const V3 o = c->cam.pos;
    V3 d = c->cam.dir;
    const float len = std::sqrt(d.x * d.x + d.y * d.y + d.z * d.z);
    if (len <= 1e-8f) return VXPT_OK;
    d = V3(d.x / len, d.y / len, d.z / len);
    int x = (int)std::floor(o.x), y = (int)std::floor(o.y), z = (int)std::floor(o.z);
    const int stx = d.x > 0.0f ? 1 : -1, sty = d.y > 0.0f ? 1 : -1, stz = d.z > 0.0f ? 1 : -1;
    auto delta = [](float v) { return std::fabs(v) < 1e-8f ? FLT_MAX : 1.0f / std::fabs(v); };
    auto first = [](float v, int cell, int step, float orig) {
        const float bound = step > 0 ? (float)(cell + 1) : (float)cell;
        return std::fabs(v) < 1e-8f ? FLT_MAX : (bound - orig) / v;
    };
    const float tdx = delta(d.x), tdy = delta(d.y), tdz = delta(d.z);
    float tmx = first(d.x, x, stx, o.x), tmy = first(d.y, y, sty, o.y), tmz = first(d.z, z, stz, o.z);
    int n = 0;
    while (n++ < 1000) {
        if (x < 0 || x >= W || y < 0 || y >= H || z < 0 || z >= D) break;
        const int id = c->hIds[(size_t)((x >> 5) + c->cx * ((z >> 5) + c->cz * (y >> 5))) * 32768 + (x & 31) +
                                32 * ((z & 31) + 32 * (y & 31))];
        if (id == 0) {
            out[5] = 1; out[6] = x; out[7] = y; out[8] = z;
        } else {
            out[0] = 1; out[1] = x; out[2] = y; out[3] = z; out[4] = id;
            break;
        }
        if (tmx < tmy) {
            if (tmx < tmz) { x += stx; tmx += tdx; }
            else { z += stz; tmz += tdz; }
        } else {
            if (tmy < tmz) { y += sty; tmy += tdy; }
            else { z += stz; tmz += tdz; }
        }
    }
    out[9] = n;
    return VXPT_OK;
}

int vxpt_set_block(vxpt_ctx *c, int x, int y, int z, int block_id) {
    if (!c) return VXPT_ERR_ARG;
    if (c->hIds.empty()) return fail(c, VXPT_ERR_STATE, "no voxels uploaded");
    HIPCHK(c, hipSetDevice(c->dev));
    int old = 0;
    if (x >= 0 && y >= 0 && z >= 0 && x < c->cx * 32 && y < c->cy * 32 && z < c->cz * 32) {
        const size_t ch = (size_t)(x >> 5) + (size_t)c->cx * ((z >> 5) + (size_t)c->cz * (y >> 5));
        old = c->hIds[ch * 32768 + (x & 31) + 32 * ((z & 31) + 32 * (y & 31))];
    }
    if (int r = set_block(c, x, y, z, block_id)) return r;
    // the instance set only changes with an instanced block
    const auto inst = [&](int id) { return id > 0 && id < kBlockTypes && c->blocks[id].instanced; };
    if (!inst(old) && !inst(block_id)) return VXPT_OK;
    // deleteInstancedBlock / addInstancedBlock of an emissive block (VoxelEngine.cu:1206-1212,
    // 1278-1284): an incremental light update with the light instance removed / changed.  A light
    // base alone also carries its light's instance here (the instance set is always the grid's,
    // collectInstanceTransforms), so its edit counts as that light's.
    const auto light_obj = [&](int id) {
        if (!inst(id) || !c->modelsLoaded) return -1;
        if (c->blocks[id].emissive) return id - 1;
        for (int l = 1; l < kBlockTypes; ++l)
            if (c->blocks[l].instanced && c->blocks[l].emissive && c->blocks[l].lightBase == id) return l - 1;
        return -1;
    };
    const int lo = old != block_id ? light_obj(old) : -1, ln = old != block_id ? light_obj(block_id) : -1;
    if (lo >= 0) c->lightState.removed.insert(instance_id(c, lo, x, y, z));
    if (ln >= 0) c->lightState.changed.insert(instance_id(c, ln, x, y, z));
    if (lo >= 0 || ln >= 0) c->lightState.incremental = true;
    return refresh_instances(c, lo >= 0 || ln >= 0, false);
}

// VoxelEngine::update's click (VoxelEngine.cu:906-975): block 0 deletes the picked block,
// another id is placed in the last empty cell before it.  out = the pick (vxpt_pick_block)
int vxpt_click_block(vxpt_ctx *c, int block_id, int32_t out[10]) {
    int32_t pk[10];
    if (int r = vxpt_pick_block(c, pk)) return r;
    if (out) std::memcpy(out, pk, sizeof(pk));
    if (block_id == 0) {
        if (pk[0]) return vxpt_set_block(c, pk[1], pk[2], pk[3], 0);
    } else if (pk[5] && pk[0]) {
        return vxpt_set_block(c, pk[6], pk[7], pk[8], block_id);
    }
    return VXPT_OK;
}

// WorldSceneManager chunk files (WorldSceneManager.cpp:240-307): each 32^3 chunk's bytes in
// <chunk_dir>/<FNV-1a 64 of the bytes, 16 hex digits>.bin; the scene yaml (SceneConfig.cpp:116-151)
// lists them under `chunks:` with the camera and `chunk_config`.
static std::string fnv1a_hex(const uint8_t *p, size_t n) {
    unsigned long long h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) {
        h ^= (unsigned long long)p[i];
        h *= 1099511628211ull;
    }
    char buf[17];
    std::snprintf(buf, sizeof buf, "%016llx", h);
    return buf;
}

int vxpt_save_world(vxpt_ctx *c, const char *scene_yaml, const char *chunk_dir) {
    if (!c || !scene_yaml || !chunk_dir) return VXPT_ERR_ARG;
    if (c->hIds.empty()) return fail(c, VXPT_ERR_STATE, "no voxels uploaded");
    std::error_code ec;
    std::filesystem::create_directories(chunk_dir, ec);
    const int nch = c->cx * c->cy * c->cz;
    std::vector<std::string> hashes(nch);
    for (int i = 0; i < nch; ++i) {
        const uint8_t *d = c->hIds.data() + (size_t)i * 32768;
        hashes[i] = fnv1a_hex(d, 32768);
        std::ofstream f(std::filesystem::path(chunk_dir) / (hashes[i] + ".bin"), std::ios::binary | std::ios::trunc);
        f.write((const char *)d, 32768);
        if (!f.good()) return fail(c, VXPT_ERR_IO, "cannot write chunk " + std::to_string(i));
    }
    std::ofstream y(scene_yaml, std::ios::trunc);
    if (!y) return fail(c, VXPT_ERR_IO, std::string("cannot write ") + scene_yaml);
    auto f3 = [](V3 v) {
        std::ostringstream o;
        o << "[" << v.x << ", " << v.y << ", " << v.z << "]";
        return o.str();
    };
    y << "# Scene Configuration File\n# Generated automatically\n\n"
      << "camera:\n  position: " << f3(c->cam.pos) << "\n  direction: " << f3(c->cam.dir)
      << "\n  up: " << f3(V3(0.0f, 1.0f, 0.0f)) << "\n  fov: " << 90.0f << "\n\n"
      << "character:\n  position: " << f3(V3(16.0f, 10.0f, 16.0f)) << "\n  rotation: " << f3(V3(0.0f))
      << "\n  scale: " << f3(V3(1.0f)) << "\n"
      << "\nchunk_config:\n  chunksX: " << c->cx << "\n  chunksY: " << c->cy << "\n  chunksZ: " << c->cz << "\n"
      << "\nchunks:\n";
    for (int i = 0; i < nch; ++i) y << "  " << i << ": " << hashes[i] << "\n";
    return y.good() ? VXPT_OK : fail(c, VXPT_ERR_IO, "scene yaml write failed");
}

// WorldSceneManager::LoadScene (:365-458): the camera and every listed chunk file; a world of
// another chunk configuration keeps the runtime one (records past it are errors), and without a
// world yet the scene's configuration is used.  The world is then rebuilt (VoxelEngine::reload).
int vxpt_load_world(vxpt_ctx *c, const char *scene_yaml, const char *chunk_dir, vxpt_camera *cam_out) {
    if (!c || !scene_yaml || !chunk_dir) return VXPT_ERR_ARG;
    std::ifstream f(scene_yaml);
    if (!f) return fail(c, VXPT_ERR_IO, std::string("cannot open ") + scene_yaml);
    std::string line, section;
    int cfg[3] = {0, 0, 0};
    std::vector<std::pair<int, std::string>> recs;
    while (std::getline(f, line)) {
        line = trim(line);
        if (line.empty() || line[0] == '#') continue;
        if (line.back() == ':') { section = line.substr(0, line.size() - 1); continue; }
        const size_t col = line.find(':');
        if (col == std::string::npos) continue;
        const std::string key = trim(line.substr(0, col)), val = trim(line.substr(col + 1));
        if (section == "chunk_config") {
            if (key == "chunksX") cfg[0] = std::atoi(val.c_str());
            else if (key == "chunksY") cfg[1] = std::atoi(val.c_str());
            else if (key == "chunksZ") cfg[2] = std::atoi(val.c_str());
        } else if (section == "chunks" && !key.empty() && std::isdigit((unsigned char)key[0])) {
            recs.emplace_back(std::atoi(key.c_str()), val);
        }
    }
    if (cam_out && vxpt_load_scene_camera(c, scene_yaml, cam_out) != VXPT_OK) return VXPT_ERR_IO;
    if (c->hIds.empty()) {
        if (cfg[0] <= 0 || cfg[1] <= 0 || cfg[2] <= 0) return fail(c, VXPT_ERR_STATE, "no world and no chunk_config");
        c->cx = cfg[0]; c->cy = cfg[1]; c->cz = cfg[2];
        c->hIds.assign((size_t)c->cx * c->cy * c->cz * 32768, 0);
    }
    const int nch = c->cx * c->cy * c->cz;
    std::vector<uint8_t> ids = c->hIds;
    bool ok = true;
    for (const auto &r : recs) {
        if (r.first < 0 || r.first >= nch) { ok = false; continue; }
        const auto path = std::filesystem::path(chunk_dir) / (r.second + ".bin");
        std::error_code ec;
        if (std::filesystem::file_size(path, ec) != 32768 || ec) { ok = false; continue; }
        std::ifstream in(path, std::ios::binary);
        in.read((char *)ids.data() + (size_t)r.first * 32768, 32768);
        if (in.gcount() != 32768) ok = false;
    }
    if (int r = vxpt_upload_voxels(c, ids.data(), c->cx, c->cy, c->cz)) return r;
    return ok ? VXPT_OK : fail(c, VXPT_ERR_IO, "some chunk records could not be loaded");
}

int vxpt_get_camera(vxpt_ctx *c, int which, float *o) {
    if (!c || !o) return VXPT_ERR_ARG;
    const CamDev &k = which ? c->prevCam : c->cam;
    const float v[32] = {k.pos.x, k.pos.y, k.pos.z, k.dir.x, k.dir.y, k.dir.z,
                         k.uvToWorld.m00, k.uvToWorld.m10, k.uvToWorld.m20, k.uvToWorld.m01, k.uvToWorld.m11,
                         k.uvToWorld.m21, k.uvToWorld.m02, k.uvToWorld.m12, k.uvToWorld.m22,
                         k.worldToUv.m00, k.worldToUv.m10, k.worldToUv.m20, k.worldToUv.m01, k.worldToUv.m11,
                         k.worldToUv.m21, k.worldToUv.m02, k.worldToUv.m12, k.worldToUv.m22,
                         k.res.x, k.res.y, k.invRes.x, k.invRes.y, k.tanHalfFov.x, k.tanHalfFov.y, c->camYaw, c->camPitch};
    std::memcpy(o, v, sizeof(v));
    return VXPT_OK;
}

int vxpt_trace(vxpt_ctx *c, int32_t it, uint32_t flags) {
    if (!c) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    const bool accum = (flags & VXPT_TRACE_ACCUMULATE) != 0;
    const int spp = (int)((flags >> 8) & 0xFF);
    if (accum && spp < 1) return fail(c, VXPT_ERR_ARG, "VXPT_TRACE_ACCUMULATE needs the spp in flag bits 8..15");
    c->denoiseInputIsAccum = accum;
    int r = do_trace(c, it, flags, accum, (flags & VXPT_TRACE_ACCUM_FIRST) != 0, accum ? 1.0f / (float)spp : 1.0f);
    if (r) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float ms = 0;
    hipEventElapsedTime(&ms, c->ev[0], c->ev[1]);
    c->timing.trace_ms = ms;
    return VXPT_OK;
}

int vxpt_denoise(vxpt_ctx *c, const vxpt_denoise_params *p, int32_t frameNum, int32_t it) {
    if (!c) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    int r = do_denoise(c, p, frameNum, it);
    if (r) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float ms = 0;
    hipEventElapsedTime(&ms, c->ev[2], c->ev[3]);
    c->timing.denoise_ms = ms;
    return VXPT_OK;
}

int vxpt_denoise_pass(vxpt_ctx *c, const vxpt_denoise_params *p, int pass, int arg, int arg2) {
    if (!c) return VXPT_ERR_ARG;
    if (!p) p = &c->yamlDenoise;
    HIPCHK(c, hipSetDevice(c->dev));
    if (int r = run_pass(c, p, pass, arg, arg2)) return r;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VXPT_OK;
}

int vxpt_render_frame(vxpt_ctx *c, const vxpt_denoise_params *p, int32_t frameNum, int32_t spp) {
    if (!c || spp < 1) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    if (c->comm) {
        std::vector<vxpt_ctx *> cs{c};
        return band_frame(cs, p ? p : &cs[0]->yamlDenoise, frameNum, spp);
    }
    const int it0 = frameNum * spp;
    HIPCHK(c, hipEventRecord(c->ev[6], c->stream));
    for (int s = 0; s < spp; ++s)
        if (int r = do_trace(c, it0 + s, 0, spp > 1, s == 0, 1.0f / (float)spp, s > 0, false, s + 1 == spp)) return r;
    HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
    c->denoiseInputIsAccum = spp > 1;
    int r = do_denoise(c, p, frameNum, it0 + spp);
    if (r) return r;
    HIPCHK(c, hipEventRecord(c->ev[7], c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float t = 0, d = 0, f = 0;
    hipEventElapsedTime(&t, c->ev[6], c->ev[1]);
    hipEventElapsedTime(&d, c->ev[2], c->ev[3]);
    hipEventElapsedTime(&f, c->ev[6], c->ev[7]);
    c->timing.trace_ms = t;
    c->timing.denoise_ms = d;
    c->timing.frame_ms = f;
    return VXPT_OK;
}

int vxpt_render_frames(vxpt_ctx *c, const vxpt_denoise_params *p, int32_t frame0, int32_t nFrames, int32_t spp) {
    if (!c || spp < 1 || nFrames < 1 || frame0 < 0) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    const auto hostT0 = std::chrono::steady_clock::now();
    auto hostMs = [&]() {
        return (float)(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - hostT0).count() /
                       nFrames);
    };
    if (c->comm) {  // banded: pipelined like the single-context loop below (band_frame), one sync at the end
        std::vector<vxpt_ctx *> cs{c};
        if (!c->runEv[0])
            for (hipEvent_t &e : c->runEv) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
        HIPCHK(c, hipEventRecord(c->runEv[0], c->stream));
        std::vector<PassPlan> pipe;  // the next frame's first pass-halves (band_frame)
        for (int f = 0; f < nFrames; ++f)
            if (int r = band_frame(cs, p ? p : &c->yamlDenoise, frame0 + f, spp, false, &pipe, f + 1 < nFrames))
                return r;
        HIPCHK(c, hipEventRecord(c->runEv[1], c->stream));
        const float host = hostMs();
        HIPCHK(c, hipStreamSynchronize(c->stream));
        band_timings(cs);  // the last frame's trace / denoiser split
        c->timing.host_ms = host;
        if (c->bst.on)
            if (int r = stat_sync_fold(c)) return r;
        float f = 0;
        hipEventElapsedTime(&f, c->runEv[0], c->runEv[1]);
        c->timing.frame_ms = f / (float)nFrames;
        return VXPT_OK;
    }
    const float scale = 1.0f / (float)spp;
    // events around every denoiser chain: the chains run alone (below), so the frames' trace time is
    // the whole minus their sum.  A chain starts when both the frame's last second half (context
    // stream) and the next frame's first half (its front stream) have finished.  A marker right behind
    // the cross-stream wait is not reliably stamped after the wait (measured 10-40 us early), so an
    // empty one-wave kernel follows the wait and the chain's start marker follows that kernel: the
    // chain is timed from its first kernel's launch, as in a frame call -- the hand-off's own latency
    // (~12 us in a kernel trace: the context stream's first launch after the front stream's last
    // kernel) stays in the frame time, not in the chain's.
    while (c->chainEv.size() < (size_t)3 * nFrames) {
        hipEvent_t e;
        HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
        c->chainEv.push_back(e);
    }
    HIPCHK(c, hipEventRecord(c->ev[6], c->stream));
    PassPlan pend;
    bool havePend = false, pendBackQueued = false;
    std::vector<char> frontMarked(nFrames, 0);  // chainEv[3f + 2] recorded in this run
    for (int f = 0; f < nFrames; ++f) {
        const int it0 = (frame0 + f) * spp;
        for (int s = 0; s < spp; ++s) {
            PassPlan pl;
            if (s == 0 && havePend) {
                pl = pend;
                havePend = false;
                if (pendBackQueued) {  // its second half is already behind the previous chain
                    pendBackQueued = false;
                    continue;
                }
            } else if (int r = trace_front(c, it0 + s, 0, spp > 1, s == 0, scale, s > 0, pl, s + 1 == spp)) {
                return r;
            }
            if (int r = trace_back(c, pl, false)) return r;
        }
        if (f + 1 < nFrames) {
            // The next frame's first pass-half runs beside this frame's last second half.  It writes
            // a G-buffer slot that is neither this frame's (the denoiser's input) nor the history
            // the denoiser compares against, the other radiance set, and its own state set; the
            // motion plane it stores is all zeros (static world) like the one the denoiser reads.
            if (int r = trace_front(c, it0 + spp, 0, spp > 1, true, scale, true, pend, spp == 1)) return r;
            havePend = true;
            // the denoiser starts after it, so it runs alone and its timing stays its own.  (Running
            // all of the chain but its firefly stage on a third stream beside the next frame's first
            // pass was measured: 6.02 -> 5.92 ms per frame, but the overlapped chain took ~3x as long
            // and k_restir beside it +0.5 ms; removed)
            // (chains after such a first half measure 0.40 instead of 0.36 ms, every chain kernel 5-10 %
            // slower with the GPU idle beside them; an L2 write-back of the first half's dirty lines
            // before the chain changed nothing -- the frame is still 0.14 ms shorter this way)
            if (!pend.a.primaryOnly && chain_gate(c, spp)) {
                frontMarked[f] = 1;
                HIPCHK(c, hipEventRecord(c->chainEv[3 * f + 2], front_stream(c, pend.set)));
                HIPCHK(c, hipStreamWaitEvent(c->stream, c->frontDone[pend.set], 0));
                HIPCHK(c, launch_stream_mark(c->stream));
                HIPCHK(c, hipEventRecord(c->chainEv[3 * f], c->stream));
            }
        }
        c->denoiseInputIsAccum = spp > 1;
        const bool waited = havePend && !pend.a.primaryOnly && chain_gate(c, spp);
        if (!waited) HIPCHK(c, hipEventRecord(c->chainEv[3 * f], c->stream));
        if (int r = do_denoise(c, p, frame0 + f, it0 + spp)) return r;
        HIPCHK(c, hipEventRecord(c->chainEv[3 * f + 1], c->stream));
        if (havePend) {  // later first halves wait for the denoiser (it reads the old history slot)
            // on the host: the next frame's first second half goes behind the chain on the context
            // stream, then the host waits for the chain before it enqueues any later first half.  A
            // first half parked on a front stream behind a wait for the chain (the device-side gate)
            // slows every kernel launch of the chain (measured: 0.39 ms against 0.36 with the front
            // streams sharing the context stream's hardware queue).
            if (int r = trace_back(c, pend, false)) return r;
            pendBackQueued = true;
            if (chain_gate(c, spp)) HIPCHK(c, hipEventSynchronize(c->chainEv[3 * f + 1]));
        }
    }
    HIPCHK(c, hipEventRecord(c->ev[7], c->stream));
    c->timing.host_ms = hostMs();
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float dsum = 0, f = 0;
    for (int k = 0; k < nFrames; ++k) {
        float a = 0, b = 0, e = 0;
        hipEventElapsedTime(&a, c->ev[6], c->chainEv[3 * k]);
        hipEventElapsedTime(&e, c->ev[6], c->chainEv[3 * k + 1]);
        if (frontMarked[k] && hipEventElapsedTime(&b, c->ev[6], c->chainEv[3 * k + 2]) == hipSuccess)
            a = std::max(a, b);
        dsum += e - a;
    }
    hipEventElapsedTime(&f, c->ev[6], c->ev[7]);
    (void)hipGetLastError();  // a failed timing read must not surface as a later launch's error
    c->timing.trace_ms = (f - dsum) / (float)nFrames;  // per frame, the chains excluded
    c->timing.denoise_ms = dsum / (float)nFrames;        // the mean chain
    c->timing.frame_ms = f / (float)nFrames;
    return VXPT_OK;
}

int vxpt_set_band(vxpt_ctx *c, int row_begin, int row_end) {
    if (!c) return VXPT_ERR_ARG;
    if (row_end <= row_begin) { row_begin = 0; row_end = c->H; }
    // bands start on an 8-row boundary: 8x8 trace tiles and the firefly filter's 8x4 tiles stay whole
    if (row_begin < 0 || row_end > c->H || (row_begin & 7) || ((row_end & 7) && row_end != c->H))
        return fail(c, VXPT_ERR_ARG, "band rows must be 8-aligned and inside the frame");
    c->rowBegin = row_begin;
    c->rowEnd = row_end;
    return VXPT_OK;
}

int vxpt_row_bytes(vxpt_ctx *c, int which) {
    void *p, *mirror;
    size_t n;
    if (!c || !buffer_ptr(c, which, p, n, false, &mirror) || (which >= 32 && which <= 34) ||
        which == VXPT_BUF_RESERVOIRS)
        return VXPT_ERR_ARG;
    return (int)(n / (size_t)c->H);
}

int vxpt_copy_rows(vxpt_ctx *c, int which, int y, int rows, void *dev, int to_buffer) {
    if (!c || !dev || rows < 0 || y < 0 || y + rows > c->H) return VXPT_ERR_ARG;
    const int rb = vxpt_row_bytes(c, which);
    if (rb <= 0) return fail(c, VXPT_ERR_ARG, "buffer has no row layout");
    void *p, *mirror;
    size_t n;
    buffer_ptr(c, which, p, n, false, &mirror);
    HIPCHK(c, hipSetDevice(c->dev));
    char *row = static_cast<char *>(p) + (size_t)y * rb;
    if (to_buffer) gbuf_written(c, which);
    if (to_buffer) HIPCHK(c, hipMemcpyAsync(row, dev, (size_t)rows * rb, hipMemcpyDeviceToDevice, c->stream));
    else HIPCHK(c, hipMemcpyAsync(dev, row, (size_t)rows * rb, hipMemcpyDeviceToDevice, c->stream));
    return VXPT_OK;
}

// the halo exchange of the band schedule for the buffers of `mask` (bit b = buffer id b < 32), over the
// context's RCCL communicator, enqueued on its stream
int vxpt_exchange_halo(vxpt_ctx *c, uint32_t mask, int rows) {
    if (!c || rows < 0) return VXPT_ERR_ARG;
    if (c->nranks <= 1 || mask == 0 || rows == 0) return VXPT_OK;
    if (!c->comm) return fail(c, VXPT_ERR_STATE, "no band communicator (vxpt_band_comm_init; linked contexts exchange inside vxpt_render_frame_linked)");
    std::vector<std::pair<int, int>> br;
    for (int b = 0; b < 32; ++b) {
        if (!((mask >> b) & 1u)) continue;
        void *ptr, *mirror;
        size_t n;
        if (!buffer_ptr(c, b, ptr, n, false, &mirror) || b == VXPT_BUF_RESERVOIRS)
            return fail(c, VXPT_ERR_ARG, "buffer has no row layout");
        gbuf_written(c, b);
        br.emplace_back(b, rows);
    }
    HIPCHK(c, hipSetDevice(c->dev));
    std::vector<vxpt_ctx *> cs{c};
    return exchange_set(cs, br, false);
}

// ProjectSunToScreen (PostProcessingPipeline.cu:187-206) on the host, like the reference;
// sunLuminance = SkyModel::getAccumulatedSunLuminance, 1 when not positive (:569-571)
static void sun_projection(vxpt_ctx *c, int &on, int &px, int &py, float &u, float &v, float &lum) {
    const V3 uvw = m3_apply(c->cam.worldToUv, normalize(c->sunDir));
    on = 0; px = py = 0; u = v = 0.0f;
    if (uvw.z > 0.0f) {
        const float uu = uvw.x / uvw.z, vv = uvw.y / uvw.z;
        if (!(uu < 0.0f || uu > 1.0f || vv < 0.0f || vv > 1.0f)) {
            on = 1;
            u = uu; v = vv;
            px = std::min(std::max((int)(uu * c->W), 0), c->W - 1);
            py = std::min(std::max((int)(vv * c->H), 0), c->H - 1);
        }
    }
    lum = c->sunLuminance > 0.0f ? c->sunLuminance : 1.0f;
}

int vxpt_get_sun_projection(vxpt_ctx *c, float out6[6]) {
    if (!c || !out6) return VXPT_ERR_ARG;
    int on, px, py;
    float u, v, lum;
    sun_projection(c, on, px, py, u, v, lum);
    out6[0] = (float)on; out6[1] = (float)px; out6[2] = (float)py; out6[3] = u; out6[4] = v; out6[5] = lum;
    return VXPT_OK;
}

int vxpt_get_denoise_params(vxpt_ctx *c, vxpt_denoise_params *out) {
    if (!c || !out) return VXPT_ERR_ARG;
    *out = c->yamlDenoise;
    return VXPT_OK;
}

int vxpt_get_post_params(vxpt_ctx *c, vxpt_post_params *out) {
    if (!c || !out) return VXPT_ERR_ARG;
    *out = c->yamlPost;
    return VXPT_OK;
}

namespace {

// the context's post-process arguments (allocating its buffers on first use)
int post_args(vxpt_ctx *c, const vxpt_post_params *pp, float dtMs, PostArgs &a) {
    if (!pp) pp = &c->yamlPost;
    const size_t n = (size_t)c->W * c->H;
    if (!c->frame) {
        if (dalloc(c, c->bloomA, n) || dalloc(c, c->bloomB, n) ||
            dalloc(c, c->frame, n) || dalloc(c, c->postHist, kPostHist) || dalloc(c, c->postState, 4))
            return VXPT_ERR_HIP;
        const float init[4] = {0.18f, 1.0f, 0.0f, 0.0f};  // m_currentAvgLuminance (PostProcessingPipeline.cu:433)
        HIPCHK(c, hipMemcpyAsync(c->postState, init, sizeof(init), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipMemsetAsync(c->postHist, 0, kPostHist * sizeof(unsigned), c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    a = PostArgs{};
    a.W = c->W; a.H = c->H;
    a.y0 = c->rowBegin; a.y1 = c->rowEnd;
    a.p = {pp->manual_exposure, pp->tone_mapping_curve, pp->white_point, pp->contrast, pp->saturation, pp->lift,
           pp->gain, pp->enable_bloom, pp->bloom_threshold, pp->bloom_intensity, pp->bloom_radius,
           pp->enable_auto_exposure, pp->exposure_speed, pp->exposure_min, pp->exposure_max,
           pp->exposure_compensation, pp->histogram_min_percent, pp->histogram_max_percent, pp->target_luminance,
           pp->enable_vignette, pp->vignette_strength, pp->vignette_radius, pp->vignette_smoothness,
           pp->enable_lens_flare, pp->lens_flare_intensity, pp->lens_flare_ghost_spacing,
           pp->lens_flare_ghost_count, pp->lens_flare_halo_radius, pp->lens_flare_sun_size,
           pp->lens_flare_distortion, pp->draw_crosshair};
    a.input = c->output;
    a.bloomA = c->bloomA; a.bloomB = c->bloomB; a.frame = c->frame;
    a.depth = c->gb[c->last].depth;
    a.hist = c->postHist;
    a.state = c->postState;
    a.dtMs = dtMs;
    sun_projection(c, a.sunOnScreen, a.sunPx, a.sunPy, a.sunU, a.sunV, a.sunLuminance);
    return VXPT_OK;
}

// A banded frame's post-process (PostProcessingPipeline::Execute over bands): the denoiser
// output's 1-row halo (the bloom extract's vertical neighbours), each band's histogram + bloom
// rows, the histogram (+ sun flag) summed over the bands -- an RCCL all-reduce of 257 u32, or a
// host sum for linked contexts -- so that every band adapts the same exposure, the horizontally
// blurred bloom's halo for the vertical taps, then exposure + compose of the band's rows.
int band_post(std::vector<vxpt_ctx *> &cs, const vxpt_post_params *pp, float dtMs) {
    std::vector<PostArgs> as(cs.size());
    for (size_t k = 0; k < cs.size(); ++k) BANDCHK(post_args(cs[k], pp, dtMs, as[k]));
    const int half = post_bloom_half(as[0]);
    if (half > 0 && half > cs[0]->rowEnd - cs[0]->rowBegin)
        return fail(cs[0], VXPT_ERR_ARG, "bloom radius exceeds the band height");
    BANDCHK(exchange_set(cs, {{VXPT_BUF_OUTPUT, 1}}));
    for (size_t k = 0; k < cs.size(); ++k) HIPCHK(cs[k], launch_post_phase1(as[k], cs[k]->stream));
    const bool reduce = as[0].p.enableAutoExposure || (as[0].p.enableLensFlare && as[0].sunOnScreen);
    if (reduce) {
        if (cs.size() == 1 && cs[0]->comm) {
            vxpt_ctx *c = cs[0];
            if (ncclAllReduce(c->postHist, c->postHist, kPostHist, ncclUint32, ncclSum, c->comm, c->stream) != ncclSuccess)
                return fail(c, VXPT_ERR_HIP, "ncclAllReduce (post histogram)");
        } else {
            std::vector<unsigned> sum(kPostHist, 0u), h(kPostHist);
            for (vxpt_ctx *c : cs) {
                HIPCHK(c, hipMemcpyAsync(h.data(), c->postHist, kPostHist * 4, hipMemcpyDeviceToHost, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
                for (int i = 0; i < kPostHist; ++i) sum[i] += h[i];
            }
            for (vxpt_ctx *c : cs) {
                HIPCHK(c, hipMemcpyAsync(c->postHist, sum.data(), kPostHist * 4, hipMemcpyHostToDevice, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
            }
        }
    }
    if (half > 0) BANDCHK(exchange_set(cs, {{VXPT_BUF_BLOOM, half}}));
    for (size_t k = 0; k < cs.size(); ++k) HIPCHK(cs[k], launch_post_phase2(as[k], cs[k]->stream));
    return VXPT_OK;
}

}  // namespace

int vxpt_postprocess(vxpt_ctx *c, const vxpt_post_params *pp, float dtMs) {
    if (!c) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    if (c->comm && c->nranks > 1) {
        std::vector<vxpt_ctx *> cs{c};
        return band_post(cs, pp, dtMs);
    }
    PostArgs a;
    if (int r = post_args(c, pp, dtMs, a)) return r;
    HIPCHK(c, launch_postprocess(a, c->stream));
    return VXPT_OK;
}

int vxpt_postprocess_linked(vxpt_ctx **cs, int n, const vxpt_post_params *pp, float dtMs) {
    if (!cs || n < 1) return VXPT_ERR_ARG;
    std::vector<vxpt_ctx *> v(cs, cs + n);
    for (int k = 0; k < n; ++k)
        if (!cs[k] || cs[k]->rank != k || cs[k]->nranks != n) return VXPT_ERR_STATE;
    HIPCHK(cs[0], hipSetDevice(cs[0]->dev));
    if (int r = band_post(v, pp, dtMs)) return r;
    for (vxpt_ctx *c : v) HIPCHK(c, hipStreamSynchronize(c->stream));
    return VXPT_OK;
}


int vxpt_band_comm_id(void *id, size_t bytes) {
    if (!id || bytes < sizeof(ncclUniqueId)) return VXPT_ERR_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return VXPT_ERR_HIP;
    std::memcpy(id, &u, sizeof(u));
    return VXPT_OK;
}

int vxpt_band_comm_init(vxpt_ctx *c, const void *id, size_t bytes, int nranks, int rank) {
    return vxpt_band_comm_init_rows(c, id, bytes, nranks, rank, nullptr);
}

int vxpt_band_comm_init_rows(vxpt_ctx *c, const void *id, size_t bytes, int nranks, int rank, const int32_t *row_splits) {
    if (!c || !id || bytes < sizeof(ncclUniqueId) || nranks < 1 || rank < 0 || rank >= nranks) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    std::vector<int> s = equal_splits(c->H, nranks);
    if (row_splits) {
        if (!splits_valid(row_splits, nranks, c->H, kTraceHalo))
            return fail(c, VXPT_ERR_ARG, "row_splits: 0 = s[0] < ... < s[n] = height, 8-aligned, bands >= 72 rows");
        s.assign(row_splits, row_splits + nranks + 1);
    }
    const int y0 = s[rank], y1 = s[rank + 1];
    if (nranks > 1 && (y1 - y0 < kTraceHalo))
        return fail(c, VXPT_ERR_ARG, "bands must be at least 72 rows tall (ReSTIR halo)");
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    if (c->comm) ncclCommDestroy(c->comm);
    c->comm = nullptr;
    c->exDoneRec = false;
    if (ncclCommInitRank(&c->comm, nranks, u, rank) != ncclSuccess) return fail(c, VXPT_ERR_HIP, "ncclCommInitRank");
    if (!c->commStream) HIPCHK(c, hipStreamCreateWithFlags(&c->commStream, hipStreamNonBlocking));
    // the exchange stream's events keep the system-scope fence: the rows a peer GPU wrote over xGMI must
    // be visible to the kernel that waits for them (without it one band measured ~1 % faster, within the
    // run-to-run spread: not worth a stale-cache risk)
    if (!c->haloReady) HIPCHK(c, hipEventCreateWithFlags(&c->haloReady, hipEventDisableTiming));
    if (!c->haloDone) HIPCHK(c, hipEventCreateWithFlags(&c->haloDone, hipEventDisableTiming));
    if (!c->exDone) HIPCHK(c, hipEventCreateWithFlags(&c->exDone, hipEventDisableTiming | hipEventDisableSystemFence));
    c->nranks = nranks;
    c->rank = rank;
    c->splits = s;
    return vxpt_set_band(c, y0, y1);
}

int vxpt_band_link(vxpt_ctx **cs, int n) { return vxpt_band_link_rows(cs, n, nullptr); }

int vxpt_debug_clamp_decisions(vxpt_ctx *c, int on) {
    if (!c) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (on && !c->clampDbg)  // kept until the context goes (zero-filled)
        if (int r = dalloc(c, c->clampDbg, (size_t)c->W * c->H)) return r;
    c->clampDbgOn = on != 0;
    return VXPT_OK;
}

int vxpt_band_stats_enable(vxpt_ctx *c, int on) {
    if (!c) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipStreamSynchronize(c->stream));  // no recorded event of the last collection pending
    if (c->commStream) HIPCHK(c, hipStreamSynchronize(c->commStream));
    auto &b = c->bst;
    b.on = on != 0;
    b.used = 0;
    b.spans.clear();
    for (double &m : b.ms) m = 0.0;
    b.frames = b.groups = b.groupsOrdered = 0;
    b.up = b.down = 0.0;
    return VXPT_OK;
}

int vxpt_band_stats(vxpt_ctx *c, vxpt_band_stat *out) {
    if (!c || !out) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    if (int r = stat_sync_fold(c)) return r;
    const auto &b = c->bst;
    vxpt_band_stat s{};
    s.frames = b.frames;
    s.groups = b.groups;
    s.groups_ordered = b.groupsOrdered;
    s.bytes_up = b.up;
    s.bytes_down = b.down;
    s.row_begin = c->rowBegin;
    s.row_end = c->rowEnd;
    s.exchange_ms = (float)b.ms[0];
    s.exchange_overlap_ms = (float)b.ms[1];
    s.trace_ms = (float)b.ms[2];
    s.denoise_ms = (float)b.ms[3];
    *out = s;
    return VXPT_OK;
}

int vxpt_band_link_rows(vxpt_ctx **cs, int n, const int32_t *row_splits) {
    if (!cs || n < 1 || !cs[0]) return VXPT_ERR_ARG;
    std::vector<int> s = equal_splits(cs[0]->H, n);
    if (row_splits) {
        if (!splits_valid(row_splits, n, cs[0]->H, kTraceHalo))
            return fail(cs[0], VXPT_ERR_ARG, "row_splits: 0 = s[0] < ... < s[n] = height, 8-aligned, bands >= 72 rows");
        s.assign(row_splits, row_splits + n + 1);
    }
    for (int k = 0; k < n; ++k) {
        vxpt_ctx *c = cs[k];
        if (!c || c->W != cs[0]->W || c->H != cs[0]->H) return VXPT_ERR_ARG;
        const int y0 = s[k], y1 = s[k + 1];
        if (n > 1 && (y1 - y0 < kTraceHalo)) return fail(c, VXPT_ERR_ARG, "bands must be at least 72 rows tall");
        c->nranks = n;
        c->rank = k;
        c->splits = s;
        c->linked.assign(cs, cs + n);
        if (int r = vxpt_set_band(c, y0, y1)) return r;
    }
    return VXPT_OK;
}

// Every band's rows of a buffer into the root's buffer (the frame's output for one writer).  RCCL:
// grouped ncclSend to the root / ncclRecv of each band at the root, on the context streams.
namespace {
int band_gather(std::vector<vxpt_ctx *> &cs, int which, int root) {
    vxpt_ctx *c0 = cs[0];
    const int world = c0->nranks;
    if (root < 0 || root >= world) return fail(c0, VXPT_ERR_ARG, "root rank out of range");
    {
        void *ptr, *mirror;
        size_t n;
        if (!buffer_ptr(c0, which, ptr, n, false, &mirror) || which == VXPT_BUF_RESERVOIRS || (which >= 32 && which <= 34))
            return fail(c0, VXPT_ERR_ARG, "buffer has no row layout (or is not allocated yet)");
    }
    if (cs.size() == 1 && c0->comm) {
        size_t rb;
        // behind every halo group on the exchange stream too: one communicator's groups run in issue
        // order on every rank (a gather beside a pending halo group could pair differently per rank)
        if (c0->haloPending) HIPCHK(c0, hipStreamWaitEvent(c0->stream, c0->haloDone, 0));
        if (ncclGroupStart() != ncclSuccess) return fail(c0, VXPT_ERR_HIP, "ncclGroupStart");
        ncclResult_t rc = ncclSuccess;
        if (c0->rank == root) {
            const std::vector<int> sp = splits_of(c0);
            for (int r = 0; r < world && rc == ncclSuccess; ++r) {
                const int y0 = sp[r], y1 = sp[r + 1];
                if (r == root || y1 <= y0) continue;
                char *dst = buffer_rows(c0, which, y0, rb);
                rc = ncclRecv(dst, (size_t)(y1 - y0) * rb, ncclUint8, r, c0->comm, c0->stream);
            }
        } else if (c0->rowEnd > c0->rowBegin) {
            char *src = buffer_rows(c0, which, c0->rowBegin, rb);
            rc = ncclSend(src, (size_t)(c0->rowEnd - c0->rowBegin) * rb, ncclUint8, root, c0->comm, c0->stream);
        }
        const ncclResult_t re = ncclGroupEnd();
        if (rc != ncclSuccess)
            return fail(c0, VXPT_ERR_HIP, std::string("ncclSend/ncclRecv (gather): ") + ncclGetErrorString(rc));
        if (re != ncclSuccess)
            return fail(c0, VXPT_ERR_HIP, std::string("ncclGroupEnd (gather): ") + ncclGetErrorString(re));
        HIPCHK(c0, hipStreamSynchronize(c0->stream));
        return VXPT_OK;
    }
    for (vxpt_ctx *c : cs) HIPCHK(c, hipStreamSynchronize(c->stream));
    vxpt_ctx *dst = cs[root];
    for (int r = 0; r < (int)cs.size(); ++r) {
        if (r == root || cs[r]->rowEnd <= cs[r]->rowBegin) continue;
        size_t rb;
        char *d = buffer_rows(dst, which, cs[r]->rowBegin, rb);
        const char *src = buffer_rows(cs[r], which, cs[r]->rowBegin, rb);
        HIPCHK(dst, hipMemcpyAsync(d, src, (size_t)(cs[r]->rowEnd - cs[r]->rowBegin) * rb, hipMemcpyDeviceToDevice,
                                   dst->stream));
    }
    HIPCHK(dst, hipStreamSynchronize(dst->stream));
    return VXPT_OK;
}
}  // namespace

int vxpt_band_gather(vxpt_ctx *c, int which, int root) {
    if (!c) return VXPT_ERR_ARG;
    if (c->nranks <= 1) return VXPT_OK;
    if (!c->comm) return fail(c, VXPT_ERR_STATE, "no band communicator (linked contexts: vxpt_band_gather_linked)");
    HIPCHK(c, hipSetDevice(c->dev));
    std::vector<vxpt_ctx *> cs{c};
    return band_gather(cs, which, root);
}

int vxpt_band_gather_linked(vxpt_ctx **cs, int n, int which, int root) {
    if (!cs || n < 1) return VXPT_ERR_ARG;
    for (int k = 0; k < n; ++k)
        if (!cs[k] || cs[k]->rank != k || cs[k]->nranks != n) return VXPT_ERR_STATE;
    if (n == 1) return VXPT_OK;
    HIPCHK(cs[0], hipSetDevice(cs[0]->dev));
    std::vector<vxpt_ctx *> v(cs, cs + n);
    return band_gather(v, which, root);
}

int vxpt_bvh_depth(const float *boxes, int n, int leaf_max, int *max_depth, int *n_nodes) {
    if (!boxes || n < 0 || leaf_max < 1 || !max_depth) return VXPT_ERR_ARG;
    std::vector<float> box(boxes, boxes + (size_t)n * 6);
    std::vector<BvhNode> nodes;
    std::vector<int> order;
    const bool ok = build_bvh(box, leaf_max, nodes, order, max_depth);
    if (n_nodes) *n_nodes = (int)nodes.size();
    return ok ? VXPT_OK : VXPT_ERR_STATE;
}

int vxpt_band_rows(int height, int nranks, int rank, int *row_begin, int *row_end) {
    if (height < 1 || nranks < 1 || rank < 0 || rank >= nranks || !row_begin || !row_end) return VXPT_ERR_ARG;
    band_rows(height, nranks, rank, *row_begin, *row_end);
    return VXPT_OK;
}

// Cost-balanced band boundaries from measured band times.  block_cost holds the frame's cost per
// 8-row block (ceil(height / 8) entries, carried between calls; a negative first entry = no estimate
// yet): each band's blocks are scaled so they sum to its measured time (a band without an estimate
// spreads its time evenly), then the boundaries go where the cumulative cost crosses k / n of the
// total, on block boundaries, every band keeping >= 72 rows.
int vxpt_band_balance(int height, int nranks, const int32_t *row_splits, const float *band_ms, float *block_cost,
                      int32_t *out_splits) {
    if (height < 1 || nranks < 1 || !row_splits || !band_ms || !block_cost || !out_splits) return VXPT_ERR_ARG;
    if (!splits_valid(row_splits, nranks, height, nranks > 1 ? kTraceHalo : 1)) return VXPT_ERR_ARG;
    const int nb = (height + 7) / 8;
    if (nranks > 1 && (int64_t)nranks * kTraceHalo > height) return VXPT_ERR_ARG;
    if (block_cost[0] < 0.0f)
        for (int b = 0; b < nb; ++b) block_cost[b] = 0.0f;
    for (int k = 0; k < nranks; ++k) {
        if (!(band_ms[k] >= 0.0f)) return VXPT_ERR_ARG;
        const int b0 = row_splits[k] / 8, b1 = (row_splits[k + 1] + 7) / 8;
        double cur = 0.0;
        for (int b = b0; b < b1; ++b) cur += block_cost[b];
        for (int b = b0; b < b1; ++b)
            block_cost[b] = cur > 0.0 ? (float)(block_cost[b] * (band_ms[k] / cur)) : band_ms[k] / (float)(b1 - b0);
    }
    std::vector<double> cum(nb + 1, 0.0);
    for (int b = 0; b < nb; ++b) cum[b + 1] = cum[b] + block_cost[b];
    const int minBlocks = nranks > 1 ? kTraceHalo / 8 : 1;
    out_splits[0] = 0;
    int prev = 0;
    for (int k = 1; k < nranks; ++k) {
        const double target = cum[nb] * k / nranks;
        const int lo = prev + minBlocks;
        const int hi = (height - (nranks - k) * kTraceHalo) / 8;  // the bands after it keep 72 rows
        int best = lo;
        for (int b = lo; b <= hi; ++b)
            if (std::fabs(cum[b] - target) < std::fabs(cum[best] - target)) best = b;
        out_splits[k] = best * 8;
        prev = best;
    }
    out_splits[nranks] = height;
    return VXPT_OK;
}

int vxpt_halo_plan(int height, int nranks, int rank, int rows, int32_t *out, int *n_entries) {
    if (height < 1 || nranks < 1 || rank < 0 || rank >= nranks || rows < 0 || !out || !n_entries) return VXPT_ERR_ARG;
    const std::vector<Halo> plan = halo_plan(equal_splits(height, nranks), rank, rows);
    for (size_t k = 0; k < plan.size(); ++k) {
        const Halo &h = plan[k];
        const int32_t e[5] = {h.peer, h.sy, h.sn, h.ry, h.rn};
        std::memcpy(out + 5 * k, e, sizeof(e));
    }
    *n_entries = (int)plan.size();
    return VXPT_OK;
}

int vxpt_band_halo_rows(const vxpt_camera *cur, const vxpt_camera *prev, int width, int height, int nranks,
                        int *trace_rows, int *history_rows) {
    if (!cur || width < 1 || height < 1 || nranks < 1 || !trace_rows || !history_rows) return VXPT_ERR_ARG;
    const CamDev c = make_camera(width, height, *cur, nullptr, nullptr);
    const CamDev pc = make_camera(width, height, prev ? *prev : *cur, nullptr, nullptr);
    std::string err;
    return band_halo_rows(c, pc, width, height, equal_splits(height, nranks), *trace_rows, *history_rows, err)
               ? VXPT_OK : VXPT_ERR_STATE;
}

int vxpt_band_halo_rows_near(const vxpt_camera *cur, const vxpt_camera *prev, int width, int height, int nranks,
                             float near_depth, int *trace_rows, int *history_rows) {
    if (!cur || width < 1 || height < 1 || nranks < 1 || !trace_rows || !history_rows) return VXPT_ERR_ARG;
    const CamDev c = make_camera(width, height, *cur, nullptr, nullptr);
    const CamDev pc = make_camera(width, height, prev ? *prev : *cur, nullptr, nullptr);
    std::string err;
    return band_halo_rows(c, pc, width, height, equal_splits(height, nranks), *trace_rows, *history_rows, err,
                          near_depth) ? VXPT_OK : VXPT_ERR_STATE;
}

int vxpt_nearest_surface(vxpt_ctx *c, const float pos[3], float *dist) {
    if (!c || !pos || !dist) return VXPT_ERR_ARG;
    *dist = nearest_surface(c, V3(pos[0], pos[1], pos[2]));
    return VXPT_OK;
}

int vxpt_render_frame_linked(vxpt_ctx **cs, int n, const vxpt_denoise_params *p, int32_t frameNum, int32_t spp) {
    if (!cs || n < 1 || spp < 1) return VXPT_ERR_ARG;
    std::vector<vxpt_ctx *> v(cs, cs + n);
    for (int k = 0; k < n; ++k)
        if (!cs[k] || cs[k]->rank != k || cs[k]->nranks != n) return VXPT_ERR_STATE;
    HIPCHK(cs[0], hipSetDevice(cs[0]->dev));
    return band_frame(v, p ? p : &v[0]->yamlDenoise, frameNum, spp);
}

// the banded vxpt_render_frames' pipelined schedule (band_frame's pipe) over linked contexts
int vxpt_render_frames_linked(vxpt_ctx **cs, int n, const vxpt_denoise_params *p, int32_t frame0, int32_t nFrames,
                              int32_t spp) {
    if (!cs || n < 1 || spp < 1 || nFrames < 1 || frame0 < 0) return VXPT_ERR_ARG;
    std::vector<vxpt_ctx *> v(cs, cs + n);
    for (int k = 0; k < n; ++k)
        if (!cs[k] || cs[k]->rank != k || cs[k]->nranks != n) return VXPT_ERR_STATE;
    HIPCHK(cs[0], hipSetDevice(cs[0]->dev));
    std::vector<PassPlan> pipe;  // every band's next-frame first pass-halves
    for (int f = 0; f < nFrames; ++f)
        if (int r = band_frame(v, p ? p : &v[0]->yamlDenoise, frame0 + f, spp, false, &pipe, f + 1 < nFrames)) return r;
    for (vxpt_ctx *c : v) HIPCHK(c, hipStreamSynchronize(c->stream));
    band_timings(v);
    for (vxpt_ctx *c : v)
        if (c->bst.on) BANDCHK(stat_sync_fold(c));
    return VXPT_OK;
}


int vxpt_readback(vxpt_ctx *c, int which, void *host, size_t bytes) {
    if (!c || !host) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    void *p, *mirror;
    size_t n;
    if (!buffer_ptr(c, which, p, n, false, &mirror)) return fail(c, VXPT_ERR_ARG, "unknown buffer");
    if (bytes < n) return fail(c, VXPT_ERR_ARG, "host buffer too small");
    HIPCHK(c, hipMemcpyAsync(host, p, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VXPT_OK;
}

int vxpt_upload(vxpt_ctx *c, int which, const void *host, size_t bytes) {
    if (!c || !host) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    void *p, *mirror;
    size_t n;
    // sky, sun and voxels are derived state: set them through their own entry points
    if (!buffer_ptr(c, which, p, n, true, &mirror) || (which >= 32 && which <= 34))
        return fail(c, VXPT_ERR_ARG, "unknown or read-only buffer");
    if (bytes < n) return fail(c, VXPT_ERR_ARG, "host buffer too small");
    gbuf_written(c, which);
    HIPCHK(c, hipMemcpyAsync(p, host, n, hipMemcpyHostToDevice, c->stream));
    if (mirror) HIPCHK(c, hipMemcpyAsync(mirror, host, n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VXPT_OK;
}

int vxpt_get_sky_alias(vxpt_ctx *c, float *q, float *p, int32_t *alias, float *sunDir) {
    if (!c || !c->skyReady) return VXPT_ERR_STATE;
    for (size_t i = 0; i < c->hSkyAlias.size(); ++i) {
        if (q) q[i] = c->hSkyAlias[i].q;
        if (p) p[i] = c->hSkyAlias[i].p;
        if (alias) alias[i] = c->hSkyAlias[i].alias;
    }
    if (sunDir) { sunDir[0] = c->sunDir.x; sunDir[1] = c->sunDir.y; sunDir[2] = c->sunDir.z; }
    return VXPT_OK;
}

int vxpt_tuning_defaults(vxpt_tuning *out) {
    if (!out) return VXPT_ERR_ARG;
    *out = tuning_defaults();
    return VXPT_OK;
}

int vxpt_get_tuning(vxpt_ctx *c, vxpt_tuning *out) {
    if (!c || !out) return VXPT_ERR_ARG;
    *out = c->tune;
    return VXPT_OK;
}

int vxpt_set_tuning(vxpt_ctx *c, const vxpt_tuning *t) {
    if (!c || !t) return VXPT_ERR_ARG;
    if (!tuning_valid(*t)) return fail(c, VXPT_ERR_ARG, "tuning field out of range");
    HIPCHK(c, hipSetDevice(c->dev));
    // whatever is in flight used the old schedule's buffers
    for (hipStream_t fs : c->frontStreams) HIPCHK(c, hipStreamSynchronize(fs));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const bool tables = t->dda_boxes != c->tune.dda_boxes || t->box_cap != c->tune.box_cap ||
                        t->box_cap_up != c->tune.box_cap_up;
    c->tune = *t;
    c->nSets = t->state_sets;
    c->useBoxes = t->dda_boxes != 0;
    c->boxCap = t->box_cap;
    c->boxCapUp = t->box_cap_up;
    if (tables && c->useBoxes && c->nBricks > 0) {  // the current world's box tables, rebuilt whole
        const int BX = c->cx * 8, BY = c->cy * 8, BZ = c->cz * 8;
        brick_prefix(c);
        c->hBox.assign((size_t)8 * c->nBricks, 0u);
        for (int oct = 0; oct < 8; ++oct) box_fill(c, oct, 0, BX - 1, 0, BY - 1, 0, BZ - 1);
        if (int r = upload_vec(c, c->bbox, c->hBox.data(), c->hBox.size())) return r;
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return VXPT_OK;
}

int vxpt_timings(vxpt_ctx *c, vxpt_timing *out) {
    if (!c || !out) return VXPT_ERR_ARG;
    *out = c->timing;
    return VXPT_OK;
}

int vxpt_sync(vxpt_ctx *c) {
    if (!c) return VXPT_ERR_ARG;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return VXPT_OK;
}

void *vxpt_stream(vxpt_ctx *c) { return c ? (void *)c->stream : nullptr; }

}  // extern "C"

// probe kernel lives in trace.hip
namespace vx {
hipError_t launch_probe(const WorldDev &w, int n, const float *rays, int *out, float *t, int mode, hipStream_t st);
}

extern "C" int vxpt_probe_rays(vxpt_ctx *c, int n, const float *rays, int32_t *out6, float *t, int mode) {
    if (!c || n <= 0 || !rays || !out6 || !t) return VXPT_ERR_ARG;
    if (!c->voxels.p) return fail(c, VXPT_ERR_STATE, "no voxels");
    HIPCHK(c, hipSetDevice(c->dev));
    float *dr;
    int *dout;
    float *dt;
    HIPCHK(c, hipMalloc(&dr, (size_t)n * 8 * 4));
    HIPCHK(c, hipMalloc(&dout, (size_t)n * 6 * 4));
    HIPCHK(c, hipMalloc(&dt, (size_t)n * 4));
    HIPCHK(c, hipMemcpyAsync(dr, rays, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
    WorldDev w;
    fill_world(c, w);
    HIPCHK(c, launch_probe(w, n, dr, dout, dt, mode, c->stream));
    HIPCHK(c, hipMemcpyAsync(out6, dout, (size_t)n * 24, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(t, dt, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(dr);
    hipFree(dout);
    hipFree(dt);
    return VXPT_OK;
}

extern "C" int vxpt_trace_counters(vxpt_ctx *c, uint32_t *out, int cap) {
    if (!c || !out || cap < 48) return VXPT_ERR_ARG;
    if (!c->wb[c->lastSet].qCount) return fail(c, VXPT_ERR_STATE, "no trace buffers");
    HIPCHK(c, hipSetDevice(c->dev));
    std::vector<uint32_t> q(kQueueWords);
    HIPCHK(c, hipMemcpyAsync(q.data(), c->wb[c->lastSet].qCount, q.size() * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < 16; ++k) {
        out[3 * k] = q[k];
        for (int level = 1; level <= 2; ++level) {
            uint32_t n = 0;
            for (int sh = 0; sh < kShards; ++sh) n += q[2 * kQueues + (((level - 1) * kQueues + k) * kShards + sh) * 16];
            out[3 * k + level] = n;
        }
    }
    return VXPT_OK;
}

extern "C" int vxpt_probe_rng(vxpt_ctx *c, int n, const int32_t *q4, float *out) {
    if (!c || n <= 0 || !q4 || !out) return VXPT_ERR_ARG;
    HIPCHK(c, hipSetDevice(c->dev));
    int *dq;
    float *dout;
    HIPCHK(c, hipMalloc(&dq, (size_t)n * 16));
    HIPCHK(c, hipMalloc(&dout, (size_t)n * 4));
    HIPCHK(c, hipMemcpyAsync(dq, q4, (size_t)n * 16, hipMemcpyHostToDevice, c->stream));
    const BlueNoiseDev bn{c->bnSobol.p, c->bnScramble.p, c->bnRank.p};
    HIPCHK(c, launch_probe_rng(bn, n, dq, dout, c->stream));
    HIPCHK(c, hipMemcpyAsync(out, dout, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(dq);
    hipFree(dout);
    return VXPT_OK;
}
