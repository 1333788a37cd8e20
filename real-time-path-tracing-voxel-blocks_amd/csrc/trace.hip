// vxpt -- the path-tracing pass on gfx950, as a wavefront of small kernels.
//
// The reference runs one OptiX raygen program per pixel that traces the
// camera ray, shades the hit (closesthit.cu:10-852) and traces up to six more
// rays for NEE and ReSTIR-DI inside the shader (RayGen.cu:8-182).  A single
// HIP kernel doing the same needs all of that state live across every DDA
// loop: 256 VGPRs, one wave per SIMD, nothing to hide memory latency.  Here
// the pass is split at every ray: traversal kernels (k_closest, k_occluded)
// hold only the DDA state and run at high occupancy; shading kernels hold no
// traversal loop.  Per-pixel state between stages lives in HBM (WaveBufs),
// one slot per pixel in 8x8-tile order so every wave works on one tile.
//
// Per path segment (seg = 0 .. totalBounceLimit-1):
//   k_closest   camera ray (seg 0) / continuing path ray        -> hit
//   k_shade     miss: sky; hit: G-buffer, BSDF sample, sun/sky candidates,
//               BRDF candidate ray                               (closesthit.cu:10-414)
//   k_closest   BRDF candidate rays                              (closesthit.cu:415-520)
//   k_nee       BRDF candidate + RIS -> visibility ray           (closesthit.cu:520-625)
//   k_occluded  visibility rays
//   k_restir    seg 0: ReSTIR temporal taps -> bias-correction + final visibility rays
//               seg > 0: shade with the RIS sample               (closesthit.cu:626-851)
//   k_occluded  (seg 0) bias-correction + final visibility rays
//   k_finish    (seg 0) bias correction, final shading, reservoir store
// Every stage consumes the blue-noise dimensions in the reference's order
// (the sampler dimension travels in the path state), so results equal the
// one-thread-per-pixel program bit for bit.
#include "vx_device.hpp"

// occupancy bounds (waves per SIMD) of the traversal and shading kernels; the defaults are the
// measured best, the macros let experiment builds try others
#ifndef VX_WPE_QUEUE
#define VX_WPE_QUEUE 7  // round 5: 8 -> 7 waves (66-71 VGPRs, no spill): 1530.0 -> 1533.1 Mpaths/s, three runs each
#endif
#ifndef VX_WPE_RESUME
#define VX_WPE_RESUME 6
#endif
#ifndef VX_WPE_RESUME_CL  // the closest-hit resume (k_resume<false, *>)
#define VX_WPE_RESUME_CL 6
#endif
#ifndef VX_WPE_SHADE
#define VX_WPE_SHADE 5
#endif
#ifndef VX_WPE_NEE
#define VX_WPE_NEE 1
#endif
#ifndef VX_WPE_CLOSEST
#define VX_WPE_CLOSEST 8
#endif
#ifndef VX_WPE_FINISH
#define VX_WPE_FINISH 1
#endif
#ifndef VX_WPE_RESTIR
#define VX_WPE_RESTIR 1
#endif

namespace vx {
namespace {

// F_EMPTY: the pixel's reservoir is the empty one (a seg-0 miss or specular hit); k_finish stores it, so
// a pass's first half never writes reservoirs (the previous pass's temporal reuse may still read them)
constexpr int F_ALIVE = 1, F_HFD = 2, F_NEE = 4, F_RESTIR = 8, F_EMPTY = 16;
// the path's meta word, unpacked as (flags F_* | surface flags SF_* << 8, sampler dimension, total
// segments, diffuse segments); stored as 8 bytes (the flags and the two counts share a word: every
// kernel reads and writes it)
VX_D int4 load_meta(const WaveBufs &w, int s) {
    const int2 m = w.pMeta[s];
    return make_int4((m.x & 0xFF) | (((m.x >> 24) & 0xF) << 8), m.y, (m.x >> 8) & 0xFF, (m.x >> 16) & 0xFF);
}
VX_D void store_meta(const WaveBufs &w, int s, int4 m) {
    w.pMeta[s] = make_int2((m.x & 0xFF) | (m.z << 8) | (m.w << 16) | (((m.x >> 8) & 0xF) << 24), m.y);
}
constexpr float kFltMax = 3.402823466e+38f;

VX_D bool slot_pixel(const TraceArgs &a, int s, int &px, int &py) {
    const int tile = s >> 6, lane = s & 63;
    px = (tile % a.tilesX) * 8 + (lane & 7);
    py = a.y0 + (tile / a.tilesX) * 8 + (lane >> 3);
    return s < a.nSlots && px < a.W && py < a.y1;
}

// XCD-local work order (tuning xcd_order).  Workgroups are dispatched to the 8 XCDs in turn, so XCD x
// runs workgroups x, x + 8, ...: xcd_run gives them one contiguous run of [0, nb) instead (a bijection).
VX_D int xcd_run(int b, int nb) {
    const int q = nb >> 3, r = nb & 7, x = b & 7, j = b >> 3;
    return x * q + min(x, r) + j;
}
// A workgroup's 4 tiles of one tile row: each XCD's run of the tile grid cut into panels of
// ceil(rows / 8) tile rows walked column by column -- the random temporal taps (a disk of 64 px) or the
// bricks of the workgroups in flight on one XCD then fall in one window of its L2.  A bijection on
// [0, nb) when nb = bx x tile rows (the host enables it only then); only the order changes.
VX_D int xcd_panel_block(int b, int nb, int bx) {
    const int L = xcd_run(b, nb);
    const int tr = nb / bx, p = (tr + 7) >> 3;
    const int panel = L / (p * bx), k = L - panel * p * bx;
    const int rows = min(p, tr - panel * p);
    return (panel * p + k % rows) * bx + k / rows;
}

VX_D int4 pack_hit(const Hit &h) { return make_int4(h.x, h.y, h.z, (h.face & 15) | (h.id << 4) | (h.hit << 12)); }
VX_D Hit unpack_hit(int4 v, float t) {
    Hit h;
    h.x = v.x; h.y = v.y; h.z = v.z;
    h.face = v.w & 15; h.id = (v.w >> 4) & 255; h.hit = (v.w >> 12) & 1;
    h.t = t;
    return h;
}
VX_D V3 xyz(float4 v) { return V3(v.x, v.y, v.z); }
VX_D float4 f4(V3 v, float w) { return make_float4(v.x, v.y, v.z, w); }

// an empty asm that takes and returns the value in VGPRs: the reads producing it complete before this
// point -- several reads in flight together instead of one per branch (unpinned, the compiler sinks
// each read into the branch that uses it; k_restir, k_finish)
VX_D void vx_pin(float &v) { asm volatile("" : "+v"(v)); }
VX_D void vx_pin(int &v) { asm volatile("" : "+v"(v)); }
VX_D void vx_pin(V3 &v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z)); }
VX_D void vx_pin(float4 &v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }
VX_D void vx_pin(Reservoir &r) {
    asm volatile("" : "+v"(r.lightData), "+v"(r.uvData), "+v"(r.weightSum), "+v"(r.targetPdf), "+v"(r.M));
}

// a, b, c for k = 0, 1, 2, else d -- component by component (a select of whole float4s from an
// array goes through scratch memory)
VX_D float pick1(int k, float a, float b, float c, float d) { return k == 0 ? a : (k == 1 ? b : (k == 2 ? c : d)); }
VX_D float4 pick4(int k, float4 a, float4 b, float4 c, float4 d) {
    return make_float4(pick1(k, a.x, b.x, c.x, d.x), pick1(k, a.y, b.y, c.y, d.y), pick1(k, a.z, b.z, c.z, d.z),
                       pick1(k, a.w, b.w, c.w, d.w));
}

// temporal-reuse disk offset (Restir.h: concentric square-to-disk, radius 64)
VX_D V2 restir_disk(float r0, float r1) {
    const V2 u = V2(r0 * 2.0f - 1.0f, r1 * 2.0f - 1.0f);
    V2 dsk(0.0f, 0.0f);
    if (!(fabsf(u.x) < 1e-10f && fabsf(u.y) < 1e-10f)) {
        float th, r;
        if (fabsf(u.x) > fabsf(u.y)) { r = u.x; th = kPiOver4 * (u.y / u.x); }
        else { r = u.y; th = kPiOver2 - kPiOver4 * (u.x / u.y); }
        dsk = V2(cosf(th) * r, sinf(th) * r);
    }
    return dsk * 64.0f;
}

// ----------------------------------------------------------------- traversal
#ifdef VX_STATS
// traversal statistics (experiment builds only), per kind 8 counters:
// rays, waves, sum of per-wave max outer iterations, outer iterations by level
// (64^3 skip, 16^3 skip, 4^3 skip, brick walk), in-brick cell steps
__device__ unsigned long long g_stats[8 * 8];  // kinds 0-4 as tools/trace_stats.py, 5 = stragglers, 6 = straggler pieces
VX_D int wsum(int v) { for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o); return v; }
VX_D void stat_wave(int kind, bool active, const int *it) {
    const unsigned long long m = __ballot(active);
    int tot = 0;
    for (int k = 0; k < 4; ++k) tot += active ? it[k] : 0;
    int mx = tot;
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
    int v[5];
    for (int k = 0; k < 5; ++k) v[k] = wsum(active ? it[k] : 0);
    if ((threadIdx.x & 63) == 0 && m) {
        unsigned long long *g = g_stats + kind * 8;
        atomicAdd(&g[0], (unsigned long long)__popcll(m));
        atomicAdd(&g[1], 1ull);
        atomicAdd(&g[2], (unsigned long long)mx);
        for (int k = 0; k < 5; ++k) atomicAdd(&g[3 + k], (unsigned long long)v[k]);
    }
}
// per kind: per-ray outer iterations in this launch, histogram bins [0,2) [2,4) [4,8) ... [128,inf)
// (8 bins), rays going up (d.y > 0), rays ending on an event (hit / occluded), max iterations
__device__ unsigned long long g_hist[8 * 16];
VX_D void stat_ray(int kind, bool active, int its, float dy, bool event) {
    int b = 0;
    while (b < 7 && its >= (2 << b)) ++b;
    unsigned long long *g = g_hist + kind * 16;
    const bool lead = (threadIdx.x & 63) == 0;
    for (int k = 0; k < 8; ++k) {
        const unsigned long long m = __ballot(active && b == k);
        if (lead && m) atomicAdd(&g[k], (unsigned long long)__popcll(m));
    }
    const unsigned long long up = __ballot(active && dy > 0.0f), ev = __ballot(active && event);
    if (lead && up) atomicAdd(&g[8], (unsigned long long)__popcll(up));
    if (lead && ev) atomicAdd(&g[9], (unsigned long long)__popcll(ev));
    int mx = active ? its : 0;
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
    if (lead && mx) atomicMax(&g[10], (unsigned long long)mx);
}
#define VX_IT , iters
#else
#define VX_IT
#endif
// the pass's camera ray direction of pixel (px, py): jitter = sampler dimensions 0 and 1
VX_D V3 camera_ray(const TraceArgs &a, int px, int py) {
    const float j0 = bn_rand(a.bn, px, py, a.iterationIndex, 0), j1 = bn_rand(a.bn, px, py, a.iterationIndex, 1);
    const V2 uv = (V2((float)px, (float)py) + V2(j0, j1)) * a.cam.invRes;
    return a.cam.uv_to_dir(uv);
}

// North_star's "voxel bricks staged into LDS" for the camera walks (tuning lds_bricks): a workgroup's
// 256 camera rays leave one origin through a narrow frustum and read few distinct bricks (8.7
// distinct 128-B lines per workgroup on the C3 bench, tools/dda_sim), so each workgroup keeps a
// direct-mapped cache of (brick, ray octant) -> box entry + cube mask in LDS.  An entry is filled
// once, by the first lane that misses on an empty slot (atomicCAS claims it, the data is written,
// then the key is published) and never evicted; a lane that finds another key, or a slot being
// filled, reads global memory.  The entries are copies, so every walk is the global one.
constexpr int kLdsBrickSlots = 512;
struct BrickCacheLds {
    int key[kLdsBrickSlots];
    uint32_t box[kLdsBrickSlots];
    uint64_t cm[kLdsBrickSlots];
};
struct LdsBricks {
    BrickCacheLds *c;
    template <bool BOX>
    VX_D uint64_t fetch(const WorldDev &w, Dda &s, int nb) const {
        static_assert(BOX, "the LDS brick cache holds box-table entries");
        const int key = nb * 8 + octant_of(s.r);
        const int slot = key & (kLdsBrickSlots - 1);
        // acquire: pairs with the filler's release below, so the entry's data is read after its key
        const int k = __hip_atomic_load(&c->key[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        uint64_t m;
        if (k == key) {
            s.box = c->box[slot];
            m = c->cm[slot];
        } else {
            m = w.cellMask[nb];
            s.box = s.ob[nb];
            if (k == -1 && atomicCAS(&c->key[slot], -1, -2) == -1) {
                c->box[slot] = s.box;
                c->cm[slot] = m;
                __hip_atomic_store(&c->key[slot], key, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        s.dist = (int)(s.box & 0xFFu);
        return m;
    }
};

// mode 2: camera rays (RayGen.cu:102-126; initialises the path state);
// mode 0: continuing path rays (BRDF-candidate rays go through the compacted queue).
template <bool BOX, bool LDS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VX_WPE_CLOSEST))) void k_closest(TraceArgs a, int mode) {
    struct NoCache {};
    __shared__ std::conditional_t<LDS, BrickCacheLds, NoCache> cache;
    if constexpr (LDS) {
        for (int k = threadIdx.x; k < kLdsBrickSlots; k += 256) cache.key[k] = -1;
        __syncthreads();
    }
    const int blk = (a.xcdOrder & 2) ? xcd_panel_block(blockIdx.x, gridDim.x, a.tilesX >> 2) : blockIdx.x;
    const int s = blk * 256 + threadIdx.x;
    int px, py;
    bool active = slot_pixel(a, s, px, py);
    const WaveBufs &w = a.wb;
    if (mode == 2)  // the pass's queue counters (4 per segment, straggler shards), zeroed here rather than by a fill launch
        for (unsigned z = (unsigned)s; z < kQueueWords / 4; z += gridDim.x * 256u)
            reinterpret_cast<uint4 *>(w.qCount)[z] = make_uint4(0u, 0u, 0u, 0u);
    V3 o, d;
    float tmax = kRayMax;
    if (active) {
        if (mode == 2) {
            Rng rng{&a.bn, px, py, a.iterationIndex, 0};
            o = a.cam.pos;
            d = camera_ray(a, px, py);
            rng.idx = 2;
            // the path's throughput (1) and radiance (0) are not stored: segment 0's seg_end starts
            // from them (first = true); the camera ray itself only for the mesh kernels that read it
            // -- k_shade<false> and the primary-only G-buffer recompute it (camera_ray)
            if (!a.primaryOnly) {
                if (a.mesh.nInst > 0) {
                    w.pPos[s] = f4(o, kRayMax);
                    w.pDir[s] = f4(d, 0.0f);
                }
                store_meta(w, s, make_int4(F_ALIVE, rng.idx, 0, 0));
            }
        } else {
            active = (w.pMeta[s].x & F_ALIVE) != 0;
            if (active) {
                o = xyz(w.pPos[s]);
                d = xyz(w.pDir[s]);
            }
        }
    }
    int iters[5] = {0, 0, 0, 0, 0};
    if (active) {
        WorldDev wc = a.world;
        wc.brickSteps = wc.brickStepsCam;
        Hit h;
        if constexpr (LDS) h = dda_closest<BOX>(wc, o, d, tmax, nullptr, LdsBricks{&cache});
        else h = dda_closest<BOX>(wc, o, d, tmax VX_IT);
        w.cHit[s] = pack_hit(h);
        w.cT[s] = h.t;
    }
#ifdef VX_STATS
    stat_wave(mode, active, iters);
#endif
}

// ----------------------------------------------------------------- ray queues
// Secondary and visibility rays are produced compacted: each producing
// workgroup appends its rays to a queue (one atomic per workgroup) as
// {o xyz + tmin, d xyz + tmax, result id}, so the traversal kernels see only
// live rays.  Result ids: closest-hit rays write cHit/cT[id] (id = slot),
// visibility rays oHit[id] (id = 4*slot + k).
struct QRays {  // up to 4 rays of one slot (a local light is seen in a different direction from each origin)
    unsigned mask;
    int id0;
    V3 d0, d1, d2, d3;
    float x0, x1, x2, x3;  // tmax
    V3 o0, o1, o2, o3;
    float t0, t1, t2, t3;  // tmin
};

// direction class of a queued ray (sortMode 1: its octant; 2: octant x dominant axis), the key of
// the per-workgroup counting sort in block_enqueue
VX_D int ray_key(int mode, V3 d) {
    const int oct = (d.x > 0.0f ? 1 : 0) | (d.y > 0.0f ? 2 : 0) | (d.z > 0.0f ? 4 : 0);
    if (mode == 1) return oct;
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    const int dom = (ax >= ay && ax >= az) ? 0 : (ay >= az ? 1 : 2);
    return oct * 3 + dom;
}

// Appends every lane's rays (bits of r.mask) to queue q.  Every thread of the
// 256-thread workgroup must call it.  With a.sortMode the workgroup's rays are
// grouped by direction class (ray_key) inside its segment of the queue, so a
// traversal wave holds rays of one class (coherent walks and table lines); the
// order of rays within a queue never changes a result.
VX_D void block_enqueue(const TraceArgs &a, int q, const QRays &r) {
    __shared__ unsigned sTot[4], sBase[4];
    __shared__ unsigned sHist[32], sOff[32];
    const WaveBufs &w = a.wb;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int n = __popc(r.mask);
    if (a.sortMode) {
        if (threadIdx.x < 32) sHist[threadIdx.x] = 0u;
        __syncthreads();
        int key[4], rank[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            key[i] = 0;
            rank[i] = 0;
            if (!(r.mask & (1u << i))) continue;
            key[i] = ray_key(a.sortMode, i == 0 ? r.d0 : (i == 1 ? r.d1 : (i == 2 ? r.d2 : r.d3)));
            rank[i] = (int)atomicAdd(&sHist[key[i]], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned t = 0;
            for (int k = 0; k < 32; ++k) {
                sOff[k] = t;
                t += sHist[k];
            }
            sBase[0] = t ? atomicAdd(&w.qCount[q], t) : 0u;
        }
        __syncthreads();
        const unsigned base = sBase[0];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (!(r.mask & (1u << i))) continue;
            const int k = (int)(base + sOff[key[i]]) + rank[i];
            const V3 o = i == 0 ? r.o0 : (i == 1 ? r.o1 : (i == 2 ? r.o2 : r.o3));
            const float tmin = i == 0 ? r.t0 : (i == 1 ? r.t1 : (i == 2 ? r.t2 : r.t3));
            const V3 d = i == 0 ? r.d0 : (i == 1 ? r.d1 : (i == 2 ? r.d2 : r.d3));
            const float tmax = i == 0 ? r.x0 : (i == 1 ? r.x1 : (i == 2 ? r.x2 : r.x3));
            w.qO[k] = f4(o, tmin);
            w.qD[k] = f4(d, tmax);
            w.qId[k] = r.id0 + i;
        }
        return;
    }
    int incl = n;
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == 63) sTot[wv] = (unsigned)incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t0 = sTot[0], t1 = sTot[1], t2 = sTot[2], t3 = sTot[3];
        const unsigned base = (t0 + t1 + t2 + t3) ? atomicAdd(&w.qCount[q], t0 + t1 + t2 + t3) : 0u;
        sBase[0] = base;
        sBase[1] = base + t0;
        sBase[2] = base + t0 + t1;
        sBase[3] = base + t0 + t1 + t2;
    }
    __syncthreads();
    int k = (int)sBase[wv] + incl - n;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (!(r.mask & (1u << i))) continue;
        const V3 o = i == 0 ? r.o0 : (i == 1 ? r.o1 : (i == 2 ? r.o2 : r.o3));
        const float tmin = i == 0 ? r.t0 : (i == 1 ? r.t1 : (i == 2 ? r.t2 : r.t3));
        const V3 d = i == 0 ? r.d0 : (i == 1 ? r.d1 : (i == 2 ? r.d2 : r.d3));
        const float tmax = i == 0 ? r.x0 : (i == 1 ? r.x1 : (i == 2 ? r.x2 : r.x3));
        w.qO[k] = f4(o, tmin);
        w.qD[k] = f4(d, tmax);
        w.qId[k] = r.id0 + i;
        ++k;
    }
}

// tOnly (closest-hit rays of voxel worlds, whose one reader needs hit / miss only): the distance
// alone, kRayMax for a miss (a voxel hit is closer than the world's diagonal)
template <bool OCC>
VX_D void store_result(const WaveBufs &w, int id, int rc, const Hit &h, bool tOnly = false) {
    if (!OCC) {
        const Hit r = rc == DdaEvent ? h : Hit{0, 0, 0, 0, -1, 0, kRayMax};
        if (!tOnly) w.cHit[id] = pack_hit(r);
        w.cT[id] = r.t;
    } else {
        w.oHit[id] = rc == DdaEvent ? 1 : 0;
    }
}

// Traversal of queue q, one ray per lane (grid sized for the queue's
// capacity; workgroups past the queue's end leave at once).  A wave lasts as
// long as its longest walk and incoherent rays have a long tail of walk
// lengths, so this phase stops every walk after `cap` outer iterations and
// moves the unfinished ones -- their walk state -- to a straggler queue that
// k_resume finishes densely packed.  The straggler queue has 8 shards
// (workgroup b appends to shard b % 8, one atomic per workgroup on that
// shard's counter word) so no single word serialises the appends.
VX_D unsigned *straggler_count(const WaveBufs &w, int level, int q, int k) {
    return w.qCount + 2 * kQueues + (((level - 1) * kQueues + q) * kShards + k) * 16;
}

template <bool OCC, bool BOX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VX_WPE_QUEUE))) void k_queue(TraceArgs a, int q, int cap, int shardCap) {
    __shared__ unsigned sTot[4], sBase[4];
    const WaveBufs &w = a.wb;
    const unsigned n = w.qCount[q];
    if (blockIdx.x * 256 >= n) return;  // whole workgroup past the end
    const int nLive = (int)((n + 255) / 256);
    const unsigned i = ((a.xcdOrder & 4) ? xcd_run(blockIdx.x, nLive) : blockIdx.x) * 256 + threadIdx.x;
    const bool live = i < n;
    Hit h{0, 0, 0, 0, -1, 0, kRayMax};
    Dda st;
    int rc = DdaNone, id = 0;
#ifdef VX_STATS
    int iters[5] = {0, 0, 0, 0, 0};
    int *itp = iters;
#else
    int *itp = nullptr;
#endif
    if (live) {
        const float4 ro = w.qO[i], rd = w.qD[i];
        id = w.qId[i];
        rc = dda_begin<OCC, BOX>(a.world, xyz(ro), xyz(rd), ro.w, rd.w, st, h);
        // visibility walks may end above the cubes they can still reach (the sky exit, vx_device.hpp):
        // the rays toward the sun and sky that leave the terrain (closest-hit walks measured slower with it)
        for (int k = 0; rc == DdaRun && k < cap; ++k) rc = dda_iter<OCC, BOX, GlobalBricks, OCC>(a.world, st, h, itp);
    }
#ifdef VX_STATS
    stat_wave((q & 3) == 1 ? 1 : ((q & 3) == 2 ? 4 : 3), live, iters);
    stat_ray((q & 3) == 1 ? 1 : ((q & 3) == 2 ? 4 : 3), live, iters[0] + iters[1] + iters[2] + iters[3],
             live ? st.r.dy : 0.0f, rc == DdaEvent);
#endif
    if (live && rc != DdaRun) store_result<OCC>(w, id, rc, h, a.mesh.nInst == 0);
    // unfinished walks -> straggler queue
    const bool defer = live && rc == DdaRun;
    const unsigned long long m = __ballot(defer);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, shard = blockIdx.x % kShards;
    if (lane == 0) sTot[wv] = (unsigned)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t0 = sTot[0], t1 = sTot[1], t2 = sTot[2], t3 = sTot[3], tot = t0 + t1 + t2 + t3;
        const unsigned base = tot ? atomicAdd(straggler_count(w, 1, q, shard), tot) : 0u;
        sBase[0] = base;
        sBase[1] = base + t0;
        sBase[2] = base + t0 + t1;
        sBase[3] = base + t0 + t1 + t2;
    }
    __syncthreads();
    if (defer) {
        const unsigned k = (unsigned)(shard * shardCap) + sBase[wv] + (unsigned)__popcll(m & ((1ull << lane) - 1ull));
        const DdaSaved sv = dda_save(st, (int)i);
        w.sCell[0][k] = sv.cell;
        w.sT[0][k] = sv.t;
        w.sFace[0][k] = sv.face;
    }
}

// (A persistent traversal that keeps 64 walks per wave in flight and refills finished lanes from the
// queue head was measured slower than the capped walks + straggler resume below, 7.5-14.4 against
// 6.1 ms of trace per C3 frame, and removed: DESIGN.md §3.)

// Resumes the level-`level` stragglers of queue q (level 1: from k_queue,
// level 2: from the level-1 resume).  Each wave serves one shard (wave index
// % 8), 64 consecutive entries per round, striding over the shard (the fixed
// grid normally covers every straggler in one round).  With cap > 0 the walks
// stop after cap more iterations and the unfinished ones move on to the next
// level, same shard, one atomic per wave.
template <bool OCC, bool BOX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC ? VX_WPE_RESUME : VX_WPE_RESUME_CL))) void k_resume(TraceArgs a, int q, int level, int shardCap, int cap) {
    const WaveBufs &w = a.wb;
    const int t = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63, wv = t >> 6;
    // the shard's own wave count (any grid size: shards differ by one wave when 4 x gridDim.x is not a
    // multiple of kShards)
    const int shard = wv % kShards, step = ((int)gridDim.x * 4 - shard + kShards - 1) / kShards * 64;
    const int n = (int)*straggler_count(w, level, q, shard);
    const int in = (level - 1) & 1, out = level & 1;
    for (int j = (wv / kShards) * 64 + lane; j - lane < n; j += step) {
        const bool live = j < n;
        Hit h{0, 0, 0, 0, -1, 0, kRayMax};
        Dda st;
        int rc = DdaNone, id = 0, e = 0;
#ifdef VX_STATS
        int iters[5] = {0, 0, 0, 0, 0};
        int *itp = iters;
#else
        int *itp = nullptr;
#endif
        if (live) {
            const int k = shard * shardCap + j;
            const DdaSaved sv{w.sCell[in][k], w.sT[in][k], w.sFace[in][k]};
            e = sv.cell.w;
            const float4 ro = w.qO[e], rd = w.qD[e];
            id = w.qId[e];
            dda_resume<BOX>(a.world, xyz(ro), xyz(rd), ro.w, rd.w, sv, st);
            rc = DdaRun;
            for (int it = 0; rc == DdaRun && (cap <= 0 || it < cap); ++it)
                rc = dda_iter<OCC, BOX, GlobalBricks, OCC>(a.world, st, h, itp);  // sky exit: k_queue
        }
#ifdef VX_STATS
        stat_wave(5, live, iters);
        stat_ray(5, live, iters[0] + iters[1] + iters[2] + iters[3], live ? st.r.dy : 0.0f, rc == DdaEvent);
#endif
        if (live && rc != DdaRun) store_result<OCC>(w, id, rc, h, a.mesh.nInst == 0);
        const bool defer = live && rc == DdaRun;
        const unsigned long long m = __ballot(defer);
        if (m) {
            const int leader = __ffsll((long long)m) - 1;
            unsigned base = 0;
            if (lane == leader) base = atomicAdd(straggler_count(w, level + 1, q, shard), (unsigned)__popcll(m));
            base = __shfl(base, leader);
            if (defer) {
                const int k = shard * shardCap + (int)base + __popcll(m & ((1ull << lane) - 1ull));
                const DdaSaved sv = dda_save(st, e);
                w.sCell[out][k] = sv.cell;
                w.sT[out][k] = sv.t;
                w.sFace[out][k] = sv.face;
            }
        }
    }
}

// The level-`level` stragglers of queue q with each walk cut into up to G pieces, one lane each
// (vx_device.hpp seg_plan / dda_seg_start: the pieces together are the walk, its result the first
// piece's with an event): a wave takes 64 / G stragglers per round, so a long walk's chain of
// dependent brick loads is G shorter chains side by side.  A piece stops as soon as an earlier piece
// of its walk has an event.  Level 2 (after iter_cap2 more iterations one lane per walk) holds only
// the longest walks, where the pieces' setup pays.
template <bool OCC, bool BOX>
__global__ __launch_bounds__(256) void k_resume_split(TraceArgs a, int q, int level, int shardCap, int G) {
    const WaveBufs &w = a.wb;
    const int t = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63, wv = t >> 6;
    const int per = 64 / G, shard = wv % kShards;
    const int step = ((int)gridDim.x * 4 - shard + kShards - 1) / kShards * per;  // the shard's waves (k_resume)
    const int n = (int)*straggler_count(w, level, q, shard), in = (level - 1) & 1;
    const int g = lane % G, gbase = lane - g;
    const unsigned long long below = (1ull << lane) - (1ull << gbase);  // the earlier pieces' lanes
    const unsigned long long gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << gbase;
    for (int j0 = (wv / kShards) * per; j0 < n; j0 += step) {  // wave-uniform
        const int j = j0 + lane / G;
        const bool live = j < n;
        Hit h{0, 0, 0, 0, -1, 0, kRayMax};
        Dda st;
        int rc = DdaNone, id = 0;
#ifdef VX_STATS
        int iters[5] = {0, 0, 0, 0, 0};
#endif
        if (live) {
            const int k = shard * shardCap + j;
            const DdaSaved sv{w.sCell[in][k], w.sT[in][k], w.sFace[in][k]};
            const int e = sv.cell.w;
            const float4 ro = w.qO[e], rd = w.qD[e];
            id = w.qId[e];
            dda_resume<BOX>(a.world, xyz(ro), xyz(rd), ro.w, rd.w, sv, st);
            int D, cells;
            float te;
            const int pieces = seg_plan(a.world, st, G, D, cells, te);
            if (g < pieces) {
                int P0 = 0, P1 = 0;
                const float T0 = g > 0 ? seg_bound(st, D, g, pieces, cells, P0) : 0.0f;
                const float T1 = g + 1 < pieces ? seg_bound(st, D, g + 1, pieces, cells, P1) : rd.w;
                if (g == 0 || T0 < te) {
                    if (g > 0) dda_seg_start<BOX>(a.world, st, D, P0, T0);
                    st.tmax = fminf(T1, rd.w);
                    rc = DdaRun;
                }
            }
        }
        for (;;) {
            const bool run = rc == DdaRun;
            if (__ballot(run) == 0ull) break;
            if (run) rc = dda_iter<OCC, BOX, GlobalBricks, OCC>(a.world, st, h VX_IT);
            // (the ballot outside the condition: every lane's event must be seen)
            const unsigned long long evNow = __ballot(rc == DdaEvent);
            if (rc == DdaRun && (evNow & below)) rc = DdaNone;  // an earlier piece has it
        }
#ifdef VX_STATS
        stat_wave(6, iters[1] + iters[2] + iters[3] > 0, iters);  // the pieces that walked
#endif
        const unsigned long long ev = __ballot(rc == DdaEvent) & gmask;
        const int first = ev ? __ffsll((long long)ev) - 1 - gbase : 0;
        if (live && g == first) store_result<OCC>(w, id, ev ? DdaEvent : DdaNone, h, a.mesh.nInst == 0);
    }
}

// ----------------------------------------------------------------- shading
// the pass's tap record (GBuf::rec) of pixel pi, written wherever the G-buffer planes are
VX_D void store_rec(const TraceArgs &a, size_t pi, V3 n, float rough, bool metal, V3 alb, float depth) {
    a.cur.rec[2 * pi] = make_float4(n.x, n.y, n.z, bits_as_float(float_as_bits(rough) | (metal ? (int)0x80000000u : 0)));
    a.cur.rec[2 * pi + 1] = make_float4(alb.x, alb.y, alb.z, depth);
}
VX_D void store_planes_sky(const TraceArgs &a, size_t pi) {  // a seg-0 miss or emitter: the sky's G-buffer
    a.cur.albedo[pi] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
    a.cur.material[pi] = (float)0xFFFF;
    a.cur.normalRough[pi] = make_float4(0.0f, -1.0f, 0.0f, 0.0f);
    a.cur.geoNormalThin[pi] = make_float4(0.0f, -1.0f, 0.0f, 0.0f);
    a.cur.matParam[pi] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}
VX_D void store_rec_sky(const TraceArgs &a, size_t pi, float depth) {
    store_rec(a, pi, V3(0.0f, -1.0f, 0.0f), 0.0f, false, V3(1.0f), depth);
}

VX_D void path_end(const TraceArgs &a, int px, int py, V3 radiance, float primaryDist) {
    if (isnan(radiance.x) || isnan(radiance.y) || isnan(radiance.z)) radiance = V3(0.5f);  // RayGen.cu:175-178
    const size_t pi = (size_t)py * a.W + px;
    if (a.writePlanes) a.cur.depth[pi] = primaryDist;
    a.illum[pi] = make_float4(radiance.x, radiance.y, radiance.z, primaryDist);
}

// spp > 1: average the passes' radiance, depth from the last pass -- after the pass,
// in pass order (a pass's paths end in both of its halves).  One-segment passes do it at the end of
// k_finish (the pass's last kernel), for the slot's own pixel.
VX_D void accum_px(const TraceArgs &a, size_t pi) {
    const float4 r = a.illum[pi];
    float4 acc = a.accumFirst ? make_float4(0.f, 0.f, 0.f, 0.f) : a.accum[pi];
    acc.x += r.x * a.accumScale;
    acc.y += r.y * a.accumScale;
    acc.z += r.z * a.accumScale;
    acc.w = r.w;
    a.accum[pi] = acc;
}
__global__ __launch_bounds__(256) void k_accum(TraceArgs a) {
    int px, py;
    if (!slot_pixel(a, blockIdx.x * 256 + threadIdx.x, px, py)) return;
    accum_px(a, (size_t)py * a.W + px);
}

// End of one TraceNextPath segment (RayGen.cu:146-173): accumulate, apply the
// BSDF weight, bounce limits; writes the pass outputs when the path ends.  first: segment 0,
// whose throughput (1), radiance (0) and travelled distance (travelled0) are not in the path state.
VX_D void seg_end(const TraceArgs &a, int s, int px, int py, int4 &meta, V3 segRad, V3 bop, float pdf, bool terminate,
                  bool curDiffuse, bool first, float travelled0 = 0.0f, float primaryDist = -1.0f) {
    const WaveBufs &w = a.wb;
    const float4 rad4 = first ? make_float4(0.0f, 0.0f, 0.0f, travelled0) : w.pRad[s];
    V3 thr = first ? V3(1.0f) : xyz(w.pThr[s]), rad = xyz(rad4);
    rad += thr * segRad;
    const bool cont = !(terminate || pdf <= 0.0f || is_null(bop));
    if (cont) thr *= bop;
    bool done = !cont;
    meta.z += 1;
    if (curDiffuse) meta.w += 1;
    if (meta.z == a.totalBounceLimit || meta.w == a.diffuseBounceLimit) done = true;
    if (done) {
        // the primary distance: given by the caller (>= 0), else the path state's
        path_end(a, px, py, rad, primaryDist >= 0.0f ? primaryDist : w.pPos[s].w);
        meta.x &= ~(F_ALIVE | F_NEE | F_RESTIR);
    } else {
        w.pThr[s] = f4(thr, 0.0f);
        w.pRad[s] = f4(rad, rad4.w);  // .w: the path's travelled distance (ray cone)
    }
}

// The shaded surface between the shading kernels: sPos = front spawn point + hit t, sNrm = shading
// normal + roughness, sAlb = albedo + flags (SF_*), sGeo = the geometric normal only where it differs
// from the shading normal (SF_GEO), sWo = the view direction (recomputing segment 0's from the camera
// ray in the readers was slower: k_restir's registers).  A thin surface's back spawn point is in sBack (w = 1: the surface
// position -- the path's spawn point -- is the back one, closesthit.cu:288 + 321).  front / back:
// the spawn points of rays leaving it.  (The translucency is read only where the surface is hit.)
constexpr int SF_METAL = 1, SF_SKIPALB = 2, SF_THIN = 4, SF_GEO = 8;
struct SurfX { V3 front, back; bool thin; };
VX_D bool same_bits(V3 a, V3 b) {
    return float_as_bits(a.x) == float_as_bits(b.x) && float_as_bits(a.y) == float_as_bits(b.y) &&
           float_as_bits(a.z) == float_as_bits(b.z);
}
// seg 0: the shading normal, roughness and albedo are the pass's tap record's (pixel order, the
// G-buffer planes' values, written by every pass -- the planes only by a frame's last pass;
// recomputing the view direction from the camera ray as well was slower); flags = the meta word's SF_*
VX_D SurfS load_surf(const TraceArgs &a, int s, int px, int py, int seg, int meta, bool &skipAlbedo,
                     SurfX *x = nullptr) {
    const WaveBufs &w = a.wb;
    SurfS sf;
    const size_t pi = (size_t)py * a.W + px;
    const float4 p = w.sPos[s], n = seg == 0 ? a.cur.rec[2 * pi] : w.sNrm[s];
    const float4 al = seg == 0 ? a.cur.rec[2 * pi + 1] : w.sAlb[s];
    sf.pos = xyz(p); sf.depth = p.w;
    sf.normal = xyz(n); sf.roughness = seg == 0 ? bits_as_float(float_as_bits(n.w) & 0x7FFFFFFF) : n.w;
    const int fl = (meta >> 8) & 0xF;
    sf.geoNormal = (fl & SF_GEO) ? xyz(w.sGeo[s]) : sf.normal;
    sf.translucency = 0.0f;
    sf.albedo = xyz(al); sf.metallic = (fl & SF_METAL) != 0;
    sf.wo = xyz(w.sWo[s]);
    skipAlbedo = (fl & SF_SKIPALB) != 0;
    if (x) {
        x->front = sf.pos;
        x->back = sf.pos;
        x->thin = (fl & SF_THIN) != 0;
        if (x->thin) {
            const float4 b = w.sBack[s];
            x->back = xyz(b);
            if (b.w != 0.0f) sf.pos = x->back;
        }
    }
    return sf;
}

// closesthit.cu:328-340: 8 local-light candidates when the scene has lights; the sun is skipped
// below the horizon of a surface that is not a thin film
VX_D void mis_params(const SkyDev &k, const SurfS &sf, bool thin, int nLocal, int &nSun, int &nMis, float &sunMis,
                     float &skyMis, float &brdfMis) {
    const bool skipSun = !thin && (dot(sf.normal, k.sunDir) < 0.0f || dot(sf.geoNormal, k.sunDir) < 0.0f);
    nSun = skipSun ? 0 : 1;
    nMis = nLocal + nSun + 2;
    sunMis = float(nSun) / nMis;
    skyMis = 1.0f / nMis;
    brdfMis = 1.0f / nMis;
}

VX_D LSample invalid_ls() { return LSample{V3(0.f), V3(0.f), 0.f, LtInvalid}; }
// A light sample between kernels: its position / direction and, for the sun and the sky, the map
// texel it was built from (tex: the index sun_ls / sky_ls took), from which its radiance and pdf
// are rebuilt with the same arithmetic; a local light's radiance and pdf are stored (ls1).
VX_D void store_ls(const WaveBufs &w, int s, const LSample &ls, int tex) {
    w.ls0[s] = f4(ls.position, bits_as_float((ls.type << 24) | (tex & 0xFFFFFF)));
    if (ls.type == LtLocal) w.ls1[s] = f4(ls.radiance, ls.solidAnglePdf);
}
// load_ls in two steps (k_finish): the sun / sky map entry of a stored sample (sky entry 0 for other
// types, unused), then the sample -- load_ls's values
VX_D float4 ls_entry(const SkyDev &k, float4 p) {
    const int tb = float_as_bits(p.w), type = (tb >> 24) & 0xFF, tex = tb & 0xFFFFFF;
    if (type == LtSun) {
        const int sx = tex % k.sunW, sy = tex / k.sunW;
        return k.sun[(size_t)clampi(sy, 0, k.sunH - 1) * k.sunW + clampi(sx, 0, k.sunW - 1)];  // sun_ls_at
    }
    return k.sky[(type == LtLocal || type == LtInvalid) ? 0 : (size_t)tex];  // sky_ls_at
}
VX_D LSample load_ls_entry(const TraceArgs &a, int s, float4 p, float4 e) {
    const int type = (float_as_bits(p.w) >> 24) & 0xFF;
    if (type == LtLocal) {
        const float4 b = a.wb.ls1[s];
        return LSample{xyz(p), xyz(b), b.w, LtLocal};
    }
    if (type == LtInvalid) return invalid_ls();
    const SkyDev &k = a.sky;
    if (type == LtSun)
        return LSample{xyz(p), V3(e.x, e.y, e.z), (k.sunW * k.sunH) / (kTwoPi * (1.0f - k.sunCosMax)), LtSun};
    return LSample{xyz(p), V3(e.x, e.y, e.z), (k.skyW * k.skyH) / (4.0f * kPi), LtSky};
}
VX_D LSample load_ls(const TraceArgs &a, int s) {
    const WaveBufs &w = a.wb;
    const float4 p = w.ls0[s];
    const int tb = float_as_bits(p.w), type = (tb >> 24) & 0xFF, tex = tb & 0xFFFFFF;
    if (type == LtLocal) {
        const float4 b = w.ls1[s];
        return LSample{xyz(p), xyz(b), b.w, LtLocal};
    }
    if (type == LtInvalid) return invalid_ls();
    return type == LtSun ? sun_ls_at(a.sky, tex, xyz(p)) : sky_ls_at(a.sky, tex, xyz(p));
}

VX_D V3 shade_light(const SurfS &sf, bool skipAlbedo, const LSample &ls, const Reservoir &r) {
    const V3 alb = skipAlbedo ? V3(1.0f) : sf.albedo;  // closesthit.cu:829-841
    const V3 wi = light_dir(ls, sf.pos);
    V3 bsdf;
    float pdf;
    disney_eval(sf.normal, sf.geoNormal, wi, sf.wo, alb, sf.metallic, sf.roughness, bsdf, pdf);
    const float cosT = fmaxf(0.0f, dot(wi, sf.normal));
    return bsdf * cosT * ls.radiance * r.weightSum / ls.solidAnglePdf;
}

// The geometry of a closest hit: spawn points, geometric normal, material.  A mesh hit (face 15:
// x = instance row, y = triangle in BLAS leaf order, z = the mesh's triangle index, id = block)
// re-runs the walk's triangle test on the same operands for its barycentrics (identical t, u, v).
struct HitGeo {
    V3 front, back, ng;
    float u, v;
    bool mesh;
};
template <bool MESH>
VX_D HitGeo hit_geometry(const TraceArgs &a, const Hit &h, V3 o, V3 d) {
    HitGeo g;
    g.u = g.v = 0.0f;
    g.mesh = MESH && h.face == 15;
    if (!g.mesh) {
        hit_frame(h, o, d, g.front, g.back, g.ng);
        return g;
    }
    const int4 r = a.meshRow[h.x];
    const V3 cell((float)r.x, (float)r.y, (float)r.z);
    const float *t9 = a.mesh.tri + (size_t)h.y * 9;
    float t;
    tri_hit(V3(o.x - cell.x, o.y - cell.y, o.z - cell.z), d, t9, 0.0f, INFINITY, 1, t, g.u, g.v);
    mesh_spawn(V3(t9[0], t9[1], t9[2]), V3(t9[3], t9[4], t9[5]), V3(t9[6], t9[7], t9[8]), g.u, g.v, cell, g.front,
               g.back, g.ng);
    return g;
}
// interpolated texcoords of a mesh hit (closesthit.cu:189)
VX_D V2 mesh_tc(const TraceArgs &a, const Hit &h, float u, float v) {
    const float *t6 = a.meshUV + (size_t)h.y * 6;
    const float alpha = 1.0f - u - v;
    return V2(t6[0], t6[1]) * alpha + V2(t6[2], t6[3]) * u + V2(t6[4], t6[5]) * v;
}
// a ray leaving a thin-film surface toward dir starts on the side it leaves from
// (closesthit.cu:288, 457, 614, 799); other surfaces spawn at the front point
VX_D V3 spawn_toward(bool thin, V3 dir, V3 n, V3 front, V3 back) {
    return thin ? (dot(dir, n) > 0.0f ? front : back) : front;
}
// a visibility ray toward a light sample from p (closesthit.cu:606-633, 734-755): local lights
// are traced to 0.01 short of the sampled point
VX_D void light_ray(const LSample &ls, V3 p, float extra, V3 &dir, float &tmax) {
    dir = light_dir(ls, p);
    tmax = ls.type == LtLocal ? length(ls.position - p) - 0.01f - extra : kRayMax;
}

// closesthit / miss for the segment's ray; candidate generation for NEE
template <bool MESH>
VX_D void shade_slot(const TraceArgs &a, int seg, int s, QRays &qr) {
    int px, py;
    if (!slot_pixel(a, s, px, py)) return;
    const WaveBufs &w = a.wb;
    int4 meta = load_meta(w, s);
    if (!(meta.x & F_ALIVE)) return;
    meta.x &= ~(F_NEE | F_RESTIR);
    const size_t pi = (size_t)py * a.W + px;
    const Hit h = unpack_hit(w.cHit[s], w.cT[s]);
    V3 rayO, rayD;
    float primaryDist;
    if (!MESH && seg == 0) {  // the camera ray, as k_closest traced it (it stores no ray state)
        rayO = a.cam.pos;
        rayD = camera_ray(a, px, py);
        primaryDist = kRayMax;
    } else {
        const float4 p4 = w.pPos[s];
        rayO = xyz(p4);
        rayD = xyz(w.pDir[s]);
        primaryDist = p4.w;
    }
    Rng rng{&a.bn, px, py, a.iterationIndex, meta.y};

    if (!h.hit) {  // __miss__radiance (miss.cu:9-82)
        if (seg == 0) {
            meta.x |= F_EMPTY;
            if (a.writePlanes) store_planes_sky(a, pi);
            store_rec_sky(a, pi, kRayMax);
        }
        seg_end(a, s, px, py, meta, sky_emission(a.sky, rayD), V3(1.0f), 0.0f, true, false, seg == 0, 0.0f, primaryDist);
        store_meta(w, s, meta);
        return;
    }

    // __closesthit__radiance (closesthit.cu:10-316)
    const V3 wo = -rayD;
    const HitGeo g = hit_geometry<MESH>(a, h, rayO, rayD);
    V3 frontPos = g.front, backPos = g.back, ng = g.ng;
    if (seg == 0 && a.writeMotion) a.motion[pi] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const MatDev &m = (MESH && g.mesh) ? a.meshMats[h.id] : a.mats[h.id];
    if (MESH && m.emissive) {  // closesthit.cu:107-122: emits until the first diffuse bounce
        V3 e(0.0f);
        if (!(meta.x & F_HFD)) {
            e = V3(m.albedo[0], m.albedo[1], m.albedo[2]);
            if (seg == 0) {
                if (a.writePlanes) store_planes_sky(a, pi);
                store_rec_sky(a, pi, h.t);
            }
        }
        if (seg == 0) primaryDist = h.t;  // the primary distance (no reservoir is stored)
        seg_end(a, s, px, py, meta, e, V3(1.0f), 0.0f, true, false, seg == 0, 0.0f, primaryDist);
        store_meta(w, s, meta);
        return;
    }
    const bool thin = m.thin != 0;
    const V3 texPos = frontPos;  // world-grid uv: the front position before a thin-film swap
    if (MESH && thin && !(dot(wo, ng) > 0.0f)) {  // closesthit.cu:124-133
        ng = -ng;
        const V3 t = frontPos;
        frontPos = backPos;
        backPos = t;
    }
    SurfS sf;
    sf.geoNormal = ng;
    sf.wo = wo;
    sf.metallic = m.metallic != 0;
    float travelled = 0.0f;  // the path's travelled distance with textures (else unused: 0)
    if (a.texEnabled) {
        // ray cone (closesthit.cu:194-195): width = spread * the path's travelled distance
        travelled = (seg == 0 ? 0.0f : w.pRad[s].w) + h.t;
        if (seg > 0) w.pRad[s].w = travelled;
        sf.albedo = V3(m.albedo[0], m.albedo[1], m.albedo[2]);
        sf.roughness = m.roughness;
        apply_textures(a.texels, a.tex, m, texPos, ng, wo, ray_cone_spread(a.cam, px, py) * travelled, sf.albedo,
                       sf.roughness, sf.metallic, sf.normal, MESH && g.mesh,
                       (MESH && g.mesh) ? mesh_tc(a, h, g.u, g.v) : V2(0.0f, 0.0f));
    } else {
        sf.albedo = max3(V3(m.albedo[0], m.albedo[1], m.albedo[2]), V3(0.001f));
        sf.roughness = m.roughness;
        sf.normal = lerp3(ng, ng, 0.2f);
    }
    if (meta.x & F_HFD) sf.roughness = fminf(sf.roughness * 2.0f + 0.1f, 1.0f);
    const bool isDiffuse = sf.roughness > kRoughThresh;
    sf.translucency = m.translucency;
    if (seg == 0 && a.writePlanes) {
        a.cur.material[pi] = (float)m.materialId;
        a.cur.normalRough[pi] = make_float4(sf.normal.x, sf.normal.y, sf.normal.z, sf.roughness);
        a.cur.geoNormalThin[pi] = make_float4(sf.normal.x, sf.normal.y, sf.normal.z, thin ? 1.0f : 0.0f);
        a.cur.matParam[pi] = make_float4(sf.metallic ? 1.0f : 0.0f, sf.translucency, 0.0f, 0.0f);
    }
    V3 swi, sbop;
    float spdf;
    {
        const float u0 = rng.next(), u1 = rng.next(), u2 = rng.next(), u3 = rng.next();
        disney_sample(u0, u1, u2, u3, sf.normal, sf.geoNormal, wo, sf.albedo, sf.metallic, sf.translucency,
                      sf.roughness, swi, sbop, spdf);
    }
    const bool terminate = spdf <= 0.0f;
    bool skipAlbedo = false;
    if (seg == 0) {
        meta.x |= F_HFD;
        if (a.writePlanes) a.cur.albedo[pi] = make_float4(sf.albedo.x, sf.albedo.y, sf.albedo.z, 1.0f);
        store_rec(a, pi, sf.normal, sf.roughness, sf.metallic, sf.albedo, h.t);  // depth = the primary distance
        skipAlbedo = true;
        primaryDist = h.t;
    }
    const V3 spawnPos = spawn_toward(thin, swi, sf.normal, frontPos, backPos);
    // the continuation ray: a one-segment pass ends every path at its first diffuse surface
    // (k_finish), so only specular hits and multi-segment passes keep it
    if (!isDiffuse || a.segments > 1) {
        w.pPos[s] = f4(spawnPos, primaryDist);
        w.pDir[s] = f4(swi, spdf);
    }
    if (!isDiffuse) {
        if (seg == 0) meta.x |= F_EMPTY;
        seg_end(a, s, px, py, meta, V3(0.0f), sbop, spdf, terminate, false, seg == 0, travelled);
        meta.y = rng.idx;
        store_meta(w, s, meta);
        return;
    }

    // NEE candidates: local lights, sun and sky from their alias tables (closesthit.cu:318-414)
    sf.pos = spawnPos;
    sf.depth = h.t;
    const SkyDev &k = a.sky;
    const int nLocal = (MESH && a.numLights > 0) ? 8 : 0;
    int nSun, nMis;
    float sunMis, skyMis, brdfMis;
    mis_params(k, sf, thin, nLocal, nSun, nMis, sunMis, skyMis, brdfMis);
    if (MESH) {
        Reservoir loc = empty_res();
        LSample locLs = invalid_ls();
        const float locMis = float(nLocal) / nMis;
        for (int i = 0; i < nLocal; ++i) {  // closesthit.cu:350-376
            float src;
            const int li = (int)alias_sample(a.lightAlias, a.numLights, rng.next(), src);
            if (li >= a.numLights) continue;
            const float ux = rng.next(), uy = rng.next();
            const LSample cand = tri_sample(tri_light(a.lights[li]), V2(ux, uy), sf.pos);
            const float blended = mis_weight(sf, cand, src, locMis, brdfMis);
            const float tp = target_pdf(cand, sf);
            const float rr = rng.next();
            if (blended != 0.0f)
                if (stream_sample(loc, (uint32_t)li, V2(ux, uy), rr, tp, 1.0f / blended)) locLs = cand;
        }
        finalize(loc, 1.0f, (float)nMis);
        loc.M = 1;
        w.rLoc[s] = loc;
        w.lLoc0[s] = f4(locLs.position, locLs.solidAnglePdf);
        w.lLoc1[s] = f4(locLs.radiance, (float)locLs.type);
    }
    Reservoir sunRes = empty_res();
    int sunSel = -1;
    if (nSun) {
        float src;
        const int idx = (int)alias_sample(k.sunAlias, k.sunW * k.sunH, rng.next(), src);
        const LSample cand = sun_ls(k, idx);
        const int sx = idx % k.sunW, sy = idx / k.sunW;
        const V2 uv((sx + 0.5f) / float(k.sunW), (sy + 0.5f) / float(k.sunH));
        float blended, tp;
        mis_and_target(sf, cand, src, sunMis, brdfMis, blended, tp);
        const float rr = rng.next();
        if (stream_sample(sunRes, kSunLight, uv, rr, tp, 1.0f / blended)) sunSel = idx;
    }
    finalize(sunRes, 1.0f, (float)nMis);
    sunRes.M = 1;
    Reservoir skyRes = empty_res();
    int skySel = -1;
    {
        float src;
        const float r0 = rng.next(), r1 = rng.next();
        const int idx = (int)alias_sample(k.skyAlias, k.skyW * k.skyH, r0 + r1 / 256.0f, src);
        const LSample cand = sky_ls(k, idx);
        const int sx = idx % k.skyW, sy = idx / k.skyW;
        const V2 uv((sx + 0.5f) / float(k.skyW), (sy + 0.5f) / float(k.skyH));
        float blended, tp;
        mis_and_target(sf, cand, src, skyMis, brdfMis, blended, tp);
        const float rr = rng.next();
        if (stream_sample(skyRes, kSkyLight, uv, rr, tp, 1.0f / blended)) skySel = idx;
    }
    finalize(skyRes, 1.0f, (float)nMis);
    skyRes.M = 1;
    // BRDF candidate direction; its ray is traced by the next k_closest
    {
        const float u0 = rng.next(), u1 = rng.next(), u2 = rng.next(), u3 = rng.next();
        V3 sd, bop;
        float bp;
        disney_sample(u0, u1, u2, u3, sf.normal, sf.geoNormal, wo, sf.albedo, sf.metallic, sf.translucency,
                      sf.roughness, sd, bop, bp);
        const V3 org = spawn_toward(thin, sd, sf.normal, frontPos, backPos);
        // the candidate's direction, w = traced (1) or not (-1); its origin only for the mesh
        // kernels (an emissive triangle's hit point is recomputed from it)
        if (MESH) w.cRayO[s] = f4(org, 0.0f);
        w.cRayD[s] = f4(sd, bp > 0.0f ? 1.0f : -1.0f);
        if (bp > 0.0f) {
            qr.mask = 1u;
            qr.id0 = s;
            qr.o0 = org;
            qr.t0 = 0.0f;
            qr.d0 = sd;
            qr.x0 = kFltMax;
        }
    }
    w.sPos[s] = f4(frontPos, h.t);
    if (thin) w.sBack[s] = f4(backPos, dot(swi, sf.normal) > 0.0f ? 0.0f : 1.0f);
    if (seg > 0) {  // segment 0's are in the G-buffer planes just written
        w.sNrm[s] = f4(sf.normal, sf.roughness);
        w.sAlb[s] = f4(sf.albedo, 0.0f);
    }
    const bool geoDiff = !same_bits(sf.geoNormal, sf.normal);
    if (geoDiff) w.sGeo[s] = f4(sf.geoNormal, 0.0f);
    const int sfl = (sf.metallic ? SF_METAL : 0) | (skipAlbedo ? SF_SKIPALB : 0) | (thin ? SF_THIN : 0) |
                    (geoDiff ? SF_GEO : 0);
    meta.x = (meta.x & 0xFF) | (sfl << 8);
    w.sWo[s] = f4(wo, 0.0f);
    if (a.segments > 1) w.pBop[s] = f4(sbop, terminate ? 1.0f : 0.0f);
    w.cSunSky[s] = make_float4(sunRes.weightSum, sunRes.targetPdf, skyRes.weightSum, skyRes.targetPdf);
    w.nIdx[s] = make_int4(sunSel, skySel, -1, 0);
    meta.x |= F_NEE | (seg == 0 ? F_RESTIR : 0);
    meta.y = rng.idx;
    store_meta(w, s, meta);
}

template <bool MESH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MESH ? 3 : VX_WPE_SHADE))) void k_shade(TraceArgs a, int seg) {
    QRays qr;
    qr.mask = 0u;
    shade_slot<MESH>(a, seg, blockIdx.x * 256 + threadIdx.x, qr);
    block_enqueue(a, 4 * seg + 1, qr);
}

// A sun / sky candidate's reservoir as k_shade left it (stream_sample of one candidate, finalize,
// M = 1): selected (sample index >= 0) -> the light, its sample's uv (the texel centre, quantised as
// stream_sample does), the final weight sum and target pdf; otherwise the empty reservoir with M = 1
// (an unselected candidate keeps target pdf 0, so finalize leaves weight sum 0).
VX_D Reservoir cand_res(uint32_t light, int idx, int mapW, int mapH, float weightSum, float targetPdf) {
    if (idx < 0) return Reservoir{0u, 0u, weightSum, targetPdf, 1.0f};
    const int sx = idx % mapW, sy = idx / mapW;
    const V2 uv((sx + 0.5f) / float(mapW), (sy + 0.5f) / float(mapH));
    return Reservoir{light | kValidBit,
                     (uint32_t)(saturate(uv.x) * 0xffff) | ((uint32_t)(saturate(uv.y) * 0xffff) << 16), weightSum,
                     targetPdf, 1.0f};
}

// BRDF candidate from its traced ray, RIS over {local, sun, sky, BRDF}, visibility ray
template <bool MESH>
VX_D void nee_slot(const TraceArgs &a, int seg, int s, QRays &qr) {
    int px, py;
    if (!slot_pixel(a, s, px, py)) return;
    const WaveBufs &w = a.wb;
    int4 meta = load_meta(w, s);
    if (!(meta.x & F_NEE)) return;
    bool skipAlbedo;
    SurfX sp;
    const SurfS sf = load_surf(a, s, px, py, seg, meta.x, skipAlbedo, &sp);
    const SkyDev &k = a.sky;
    Rng rng{&a.bn, px, py, a.iterationIndex, meta.y};
    const int nLocal = (MESH && a.numLights > 0) ? 8 : 0;
    int nSun, nMis;
    float sunMis, skyMis, brdfMis;
    mis_params(k, sf, sp.thin, nLocal, nSun, nMis, sunMis, skyMis, brdfMis);

    Reservoir localRes = empty_res();
    LSample localLs = invalid_ls();
    if (MESH) {  // the local candidates streamed by k_shade
        localRes = w.rLoc[s];
        const float4 l0 = w.lLoc0[s], l1 = w.lLoc1[s];
        localLs = LSample{xyz(l0), xyz(l1), l0.w, (int)l1.w};
    } else {
        finalize(localRes, 1.0f, (float)nMis);
        localRes.M = 1;
    }
    const int4 idx = w.nIdx[s];
    const float4 css = w.cSunSky[s];
    const Reservoir sunRes = cand_res(kSunLight, idx.x, k.sunW, k.sunH, css.x, css.y);
    const Reservoir skyRes = cand_res(kSkyLight, idx.y, k.skyW, k.skyH, css.z, css.w);
    const LSample sunLs = idx.x >= 0 ? sun_ls(k, idx.x) : invalid_ls();
    const LSample skyLs = idx.y >= 0 ? sky_ls(k, idx.y) : invalid_ls();

    Reservoir brdfRes = empty_res();
    LSample brdfLs = invalid_ls();
    int brdfTex = 0;  // the BRDF candidate's sun / sky map texel
    {
        float lightSrcPdf = 0.0f;
        uint32_t li = kInvalidLight;
        V2 uv(0.0f, 0.0f);
        LSample cand = invalid_ls();
        int candTex = 0;
        const float4 cd = w.cRayD[s];
        if (cd.w >= 0.0f) {
            const V3 sd = xyz(cd);
            // voxel worlds: hit / miss from the distance alone (store_result's tOnly)
            const Hit bh = MESH ? unpack_hit(w.cHit[s], w.cT[s]) : Hit{w.cT[s] != kRayMax ? 1 : 0, 0, 0, 0, 0, 0, 0.0f};
            if (MESH && bh.hit && bh.face == 15) {
                // __closesthit__bsdf_light (closesthit.cu:854-900): an emissive instance's triangle is
                // light (its first light + the mesh's triangle index)
                const int base = a.meshRowLight[bh.x];
                if (nLocal > 0 && a.meshMats[bh.id].emissive && base >= 0) {
                    li = (uint32_t)(base + bh.z);
                    if (li >= (uint32_t)a.numLights) {
                        li = kInvalidLight;
                    } else {
                        const int4 r = a.meshRow[bh.x];
                        const V3 org = xyz(w.cRayO[s]);
                        float t, bu, bv;
                        tri_hit(V3(org.x - (float)r.x, org.y - (float)r.y, org.z - (float)r.z), sd,
                                a.mesh.tri + (size_t)bh.y * 9, 0.0f, INFINITY, 1, t, bu, bv);
                        uv = inverse_tri_sample(bu, bv);
                        cand = tri_sample(tri_light(a.lights[li]), uv, sf.pos);
                        lightSrcPdf = a.lightAlias[li].p;
                    }
                }
            } else if (!bh.hit) {  // __miss__bsdf_light
                if (eq_area_cone_uv(uv, k.sunDir, sd, k.sunCosMax)) {
                    li = kSunLight;
                    int x = (int)(uv.x * k.sunW - 0.5f), y = (int)(uv.y * k.sunH - 0.5f);
                    if (x >= k.sunW) x %= k.sunW;
                    if (x < 0) x = k.sunW - ((-x) % k.sunW);
                    y = clampi(y, 0, k.sunH - 1);
                    const int l = y * k.sunW + x;
                    cand = sun_ls(k, l);
                    cand.position = sd;
                    candTex = l;
                    lightSrcPdf = k.sunAlias[l].p;
                } else {
                    li = kSkyLight;
                    uv = eq_area_sphere_uv(sd);
                    const int x = (int)(uv.x * k.skyW - 0.5f), y = (int)(uv.y * k.skyH - 0.5f);
                    const int l = y * k.skyW + x;
                    cand = sky_ls(k, l);
                    cand.position = sd;
                    candTex = l;
                    lightSrcPdf = k.skyAlias[l].p;
                }
            }
        }
        if (lightSrcPdf != 0.0f) {
            const float misW = (li == kSkyLight) ? skyMis : ((li == kSunLight) ? sunMis : float(nLocal) / nMis);
            float blended, tp;
            mis_and_target(sf, cand, lightSrcPdf, misW, brdfMis, blended, tp);
            const float rr = rng.next();
            if (stream_sample(brdfRes, li, uv, rr, tp, 1.0f / blended)) {
                brdfLs = cand;
                brdfTex = candTex;
            }
        }
    }
    finalize(brdfRes, 1.0f, (float)nMis);
    brdfRes.M = 1;

    Reservoir ris = empty_res();
    combine(ris, localRes, 0.5f, localRes.targetPdf);
    const bool selSun = combine(ris, sunRes, rng.next(), sunRes.targetPdf);
    const bool selSky = combine(ris, skyRes, rng.next(), skyRes.targetPdf);
    const bool selBrdf = combine(ris, brdfRes, rng.next(), brdfRes.targetPdf);
    finalize(ris, 1.0f, 1.0f);
    ris.M = 1;
    const LSample ls = selBrdf ? brdfLs : (selSky ? skyLs : (selSun ? sunLs : localLs));
    const int lsTex = selBrdf ? brdfTex : (selSky ? idx.y : (selSun ? idx.x : 0));
    const bool trace = ls.type != LtInvalid && ris.lightData != 0;
    if (trace) {
        V3 dir;
        float tmax;
        light_ray(ls, sf.pos, 0.0f, dir, tmax);
        qr.mask = 1u;
        qr.id0 = 4 * s;
        qr.o0 = spawn_toward(sp.thin, dir, sf.normal, sp.front, sp.back);
        qr.t0 = 0.0f;
        qr.d0 = dir;
        qr.x0 = tmax;
    }
    w.rRis[s] = make_float4(bits_as_float((int)ris.lightData), bits_as_float((int)ris.uvData), ris.weightSum,
                            ris.targetPdf);
    store_ls(w, s, ls, lsTex);
    meta.y = rng.idx;
    store_meta(w, s, meta);
}

template <bool MESH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MESH ? 1 : VX_WPE_NEE))) void k_nee(TraceArgs a, int seg) {
    QRays qr;
    qr.mask = 0u;
    nee_slot<MESH>(a, seg, blockIdx.x * 256 + threadIdx.x, qr);
    block_enqueue(a, 4 * seg + 2, qr);
}

// visibility of the RIS sample; seg 0: ReSTIR temporal reuse (Restir.h:11-415,
// closesthit.cu:626-851) up to its visibility rays; seg > 0: final shading.
// LoadDIReservoir (Restir.h:48-79): the previous pass's reservoir, its local-light index remapped
// in the pass after a light update (a light that is gone empties it).  Taken literally: an empty
// reservoir (lightData 0) reads as index 0 and is remapped as well.
VX_D Reservoir remap_prev_res(const TraceArgs &a, Reservoir r) {
    if (!a.lightsDirty) return r;
    const uint32_t li = r.lightData & 0x7FFFFFFFu;
    if (li >= 0x7FFFFFFDu || li >= (uint32_t)a.prevNumLights) return r;  // sun / sky, or not a previous light
    const int cur = a.lightRemap[li];
    if (cur < 0 || cur >= a.numLights) return empty_res();
    r.lightData = (r.lightData & 0x80000000u) | (uint32_t)cur;
    return r;
}

// stash: an LDS home for the accepted taps' records ([tap][half][thread], k_restir's workgroup), so
// the bias correction reads them there instead of fetching them again
template <bool MESH>
VX_D void restir_slot(const TraceArgs &a, int seg, int s, QRays &qr, float4 (*stash)[2][256]) {
    int px, py;
    if (!slot_pixel(a, s, px, py)) return;
    const WaveBufs &w = a.wb;
    int4 meta = load_meta(w, s);
    if (!(meta.x & F_NEE)) return;
    // read ahead with the surface below (functions of the pixel and meta.y only): the temporal disks'
    // four random numbers, the previous pass's jitter and the RIS sample's visibility
    float rd0 = bn_rand(a.bn, px, py, a.iterationIndex, meta.y), rd1 = bn_rand(a.bn, px, py, a.iterationIndex, meta.y + 1),
          rd2 = bn_rand(a.bn, px, py, a.iterationIndex, meta.y + 2), rd3 = bn_rand(a.bn, px, py, a.iterationIndex, meta.y + 3);
    float jx = bn_rand(a.bn, px, py, a.iterationIndex - 1, 0), jy = bn_rand(a.bn, px, py, a.iterationIndex - 1, 1);
    // and the next three, for the temporal taps' combine chain
    float rq0 = bn_rand(a.bn, px, py, a.iterationIndex, meta.y + 4), rq1 = bn_rand(a.bn, px, py, a.iterationIndex, meta.y + 5),
          rq2 = bn_rand(a.bn, px, py, a.iterationIndex, meta.y + 6);
    int hit0 = w.oHit[4 * s];
    bool skipAlbedo;
    SurfX sp;
    SurfS sf = load_surf(a, s, px, py, seg, meta.x, skipAlbedo, &sp);
    const bool hasLocal = MESH && a.numLights > 0;
    float4 ris4 = w.rRis[s];
    LSample ls = load_ls(a, s);
    // every read above completes here (unpinned, the compiler sinks them into the branches below,
    // where they follow one another)
    vx_pin(rd0); vx_pin(rd1); vx_pin(rd2); vx_pin(rd3); vx_pin(jx); vx_pin(jy); vx_pin(hit0);
    vx_pin(rq0); vx_pin(rq1); vx_pin(rq2);
    vx_pin(sf.pos); vx_pin(sf.normal); vx_pin(sf.geoNormal); vx_pin(sf.albedo); vx_pin(sf.wo);
    vx_pin(sf.depth); vx_pin(sf.roughness); vx_pin(sp.back); vx_pin(ris4);
    vx_pin(ls.position); vx_pin(ls.radiance); vx_pin(ls.solidAnglePdf);
    Reservoir ris{(uint32_t)float_as_bits(ris4.x), (uint32_t)float_as_bits(ris4.y), ris4.z, ris4.w, 1.0f};
    bool visible = false;
    if (ls.type != LtInvalid && ris.lightData != 0) {
        visible = !hit0;
        if (!visible) { ris.lightData = 0; ris.weightSum = 0; }
    }
    if (!(meta.x & F_RESTIR)) {
        V3 segRad(0.0f);
        if (ls.type != LtInvalid && ris.lightData != 0 && visible) segRad = shade_light(sf, skipAlbedo, ls, ris);
        const float4 b = w.pBop[s];
        seg_end(a, s, px, py, meta, segRad, xyz(b), w.pDir[s].w, b.w != 0.0f, true, false);
        store_meta(w, s, meta);
        return;
    }

    Rng rng{&a.bn, px, py, a.iterationIndex, meta.y};
    Reservoir rr = empty_res();
    combine(rr, ris, 0.5f, ris.targetPdf);
    const CamDev &pc = a.prevCam;
    const V3 prevW = sf.pos;  // + motion (static geometry: 0)
    const V2 puv = pc.dir_to_uv(normalize(prevW - pc.pos));
    const int ppx = (int)(puv.x * pc.res.x), ppy = (int)(puv.y * pc.res.y);
    const V3 dd = prevW - pc.pos;
    const float expDepth = sqrtf(dd.x * dd.x + dd.y * dd.y + dd.z * dd.z);
    // three temporal taps (scalars, not arrays: no runtime-indexed private memory)
    const int ox0 = ppx - px, oy0 = ppy - py;
    int ox1, oy1, ox2, oy2;
    {
        const V2 dsk = restir_disk(rd0, rd1);
        ox1 = ppx - px + (int)dsk.x; oy1 = ppy - py + (int)dsk.y;
    }
    {
        const V2 dsk = restir_disk(rd2, rd3);
        ox2 = (int)dsk.x; oy2 = (int)dsk.y;
    }
    rng.idx += 4;
    const V2 jit(jx, jy);
    unsigned cached = 0;
    int selLoop = -1;
    float tapM0 = 0, tapM1 = 0, tapM2 = 0;
    V3 vd0(0.0f), vd1(0.0f), vd2(0.0f);  // the accepted taps' view directions, for the bias correction
    // the taps' memory reads go out together instead of tap after tap: every tap's record and previous
    // reservoir (a rejected tap's reservoir is read and dropped), then the acceptance tests, then every
    // tap's environment-light entry, then the combine chain in tap order (the same operations on the
    // same values as the loop below)
    float4 tb[3], tn[3];
    Reservoir tr[3];
    bool tin[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int oxi = i == 0 ? ox0 : (i == 1 ? ox1 : ox2), oyi = i == 0 ? oy0 : (i == 1 ? oy1 : oy2);
        const int x = reflect_view(px + oxi, a.W), y = reflect_view(py + oyi, a.H);
        tin[i] = x >= 0 && y >= 0 && x < (int)a.prevCam.res.x && y < (int)a.prevCam.res.y;
        const size_t ti = tin[i] ? (size_t)y * a.W + x : 0;
        tb[i] = a.prev.rec[2 * ti + 1];
        tn[i] = a.prev.rec[2 * ti];
        tr[i] = a.resPrev[ti];
    }
    // (held here: without the pins the compiler sinks each tap's reads into its own branch below,
    // one memory round trip per tap again)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        vx_pin(tb[i]);
        vx_pin(tn[i]);
        vx_pin(tr[i]);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (!tin[i] || tb[i].w == kRayMax) continue;  // the tap is off screen or sky
        const int oxi = i == 0 ? ox0 : (i == 1 ? ox1 : ox2), oyi = i == 0 ? oy0 : (i == 1 ? oy1 : oy2);
        const int x = reflect_view(px + oxi, a.W), y = reflect_view(py + oyi, a.H);
        const V3 vd = a.prevCam.uv_to_dir((V2((float)x, (float)y) + jit) * a.prevCam.invRes);
        SurfS ts;
        rec_surface(a, tn[i], tb[i], vd, ts);
        if (i == 0) vd0 = vd; else if (i == 1) vd1 = vd; else vd2 = vd;
        const bool nOk = dot(sf.normal, ts.geoNormal) >= 0.5f;
        const bool dOk = fabsf(expDepth - ts.depth) <= 0.1f * fmaxf(expDepth, ts.depth);
        const bool rOk = fabsf(sf.roughness - ts.roughness) <= 0.5f * fmaxf(sf.roughness, ts.roughness);
        if (!(nOk && dOk && rOk)) continue;
        cached |= (1u << i);
        stash[i][0][threadIdx.x] = tn[i];
        stash[i][1][threadIdx.x] = tb[i];
    }
    float4 te[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        Reservoir pr = remap_prev_res(a, tr[i]);
        if (isnan(pr.weightSum) || isinf(pr.weightSum)) pr = empty_res();
        if (pr.M > 20.0f) pr.M = 20.0f;
        tr[i] = pr;
        te[i] = env_entry(a.sky, pr);
    }
    const float4 teRis = env_entry(a.sky, ris);  // the combined reservoir's light when no tap is selected
    int nDraw = 0;  // the k-th accepted tap draws rng's k-th next value (rq0..2, read ahead)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (!(cached & (1u << i))) continue;
        Reservoir pr = tr[i];
        if (i == 0) tapM0 = pr.M; else if (i == 1) tapM1 = pr.M; else tapM2 = pr.M;
        float nw = 0.0f;
        LSample cand = invalid_ls();
        if (pr.lightData != 0) {
            if (!light_from_entry(a, cand, pr, sf.pos, hasLocal, te[i])) pr = empty_res();
            nw = target_pdf(cand, sf);
        }
        const float rnd = nDraw == 0 ? rq0 : (nDraw == 1 ? rq1 : rq2);
        ++nDraw;
        if (combine(rr, pr, rnd, nw)) { ls = cand; selLoop = i; }
    }
    rng.idx += nDraw;
    // bias-correction rays: the selected light seen from each accepted tap's surface
    float psv0 = 0, psv1 = 0, psv2 = 0;
    qr.id0 = 4 * s;
    LSample sel = invalid_ls();  // the combined reservoir's light (environment lights: the same for every tap)
    if (rr.lightData != 0)
        light_from_entry(a, sel, rr, sf.pos, hasLocal,
                         pick4(selLoop, te[0], te[1], te[2], teRis));
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (rr.lightData != 0 && (cached & (1u << i))) {
            SurfS ts;
            const V3 vdi = i == 0 ? vd0 : (i == 1 ? vd1 : vd2);
            rec_surface(a, stash[i][0][threadIdx.x], stash[i][1][threadIdx.x], vdi, ts);
            if (MESH && sel.type == LtLocal) light_from_res(a, sel, rr, ts.pos, hasLocal);  // seen from the tap
            const float psv = target_pdf(sel, ts);
            if (i == 0) psv0 = psv; else if (i == 1) psv1 = psv; else psv2 = psv;
            // prevSceneEmpty: OptiX's null prevTopObject -- the ray misses, the sample is visible
            if (psv > 0 && !(i == 0 && i == selLoop) && !a.prevSceneEmpty) {
                qr.mask |= 2u << i;
                const float tmin = 0.01f + 0.01f * ts.depth;
                V3 dir;
                float tmax;
                light_ray(ls, ts.pos, tmin, dir, tmax);
                if (i == 0) { qr.o1 = ts.pos; qr.t1 = tmin; qr.d1 = dir; qr.x1 = tmax; }
                else if (i == 1) { qr.o2 = ts.pos; qr.t2 = tmin; qr.d2 = dir; qr.x2 = tmax; }
                else { qr.o3 = ts.pos; qr.t3 = tmin; qr.d3 = dir; qr.x3 = tmax; }
            }
        }
        w.oHit[4 * s + 1 + i] = 0;
    }
    // final visibility: with no tap selected the sample is the RIS one and the
    // ray equals the RIS visibility ray, whose result is already in oHit[4s]
    if (ls.type != LtInvalid && selLoop >= 0) {
        V3 dir;
        float tmax;
        light_ray(ls, sf.pos, 0.0f, dir, tmax);
        qr.mask |= 1u;
        qr.o0 = spawn_toward(sp.thin, dir, sf.normal, sp.front, sp.back);
        qr.t0 = 0.0f;
        qr.d0 = dir;
        qr.x0 = tmax;
    }
    w.rRR[s] = rr;
    // for k_finish: the taps' target pdfs and M, the selected tap and the accepted-tap mask (the
    // selected light sample is not stored: with a tap selected it is the combined reservoir's light,
    // which k_finish rebuilds from the same operands; else the RIS sample k_nee stored stays)
    w.tapPsv[s] = make_float4(psv0, psv1, psv2, tapM0);
    w.tapM[s] = make_float4(tapM1, tapM2, bits_as_float(selLoop), bits_as_float((int)cached));
    meta.y = rng.idx;
    store_meta(w, s, meta);
}

// WPE: the occupancy bound (1: the compiler's register budget; 4 for small bands, tuning restir_waves)
template <bool MESH, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_restir(TraceArgs a, int seg) {
    __shared__ float4 stash[3][2][256];
    QRays qr;
    qr.mask = 0u;
    const int blk = (a.xcdOrder & 1) ? xcd_panel_block(blockIdx.x, gridDim.x, a.tilesX >> 2) : blockIdx.x;
    restir_slot<MESH>(a, seg, blk * 256 + threadIdx.x, qr, stash);
    block_enqueue(a, 4 * seg + 3, qr);
}

// seg 0: bias-corrected ReSTIR weight, final visibility, shading, reservoir store
VX_D void finish_slot(const TraceArgs &a, int s, int px, int py) {
    const WaveBufs &w = a.wb;
    int4 meta = load_meta(w, s);
    const size_t pi = (size_t)py * a.W + px;
    if (meta.x & F_EMPTY) {
        a.resCur[pi] = empty_res();
        return;
    }
    if (!(meta.x & F_NEE) || !(meta.x & F_RESTIR)) return;
    // every read of the slot's state at once: the surface, the combined reservoir, the taps' record,
    // the four visibility results (one word), the stored light sample and the continuation (pinned
    // below: unpinned, the compiler sinks each read into the branch that uses it)
    const bool one = a.segments == 1;
    Reservoir rr = w.rRR[s];
    float4 psv4 = w.tapPsv[s], m4 = w.tapM[s], ls0 = w.ls0[s];
    int hits = (int)reinterpret_cast<const uint32_t *>(w.oHit)[s];  // oHit[4s .. 4s + 3], low byte first
    // segment 0 (the only one with temporal reuse); travelled and the primary distance: its hit
    // distance (sPos.w).  A one-segment pass ends the path here (k_shade stored no continuation).
    float4 b = one ? make_float4(1.0f, 1.0f, 1.0f, 0.0f) : w.pBop[s];
    float pdf = one ? 1.0f : w.pDir[s].w;
    bool skipAlbedo;
    SurfX sp;
    SurfS sf = load_surf(a, s, px, py, 0, meta.x, skipAlbedo, &sp);
    vx_pin(rr); vx_pin(psv4); vx_pin(m4); vx_pin(ls0); vx_pin(hits); vx_pin(b); vx_pin(pdf);
    vx_pin(sf.pos); vx_pin(sf.normal); vx_pin(sf.geoNormal); vx_pin(sf.albedo); vx_pin(sf.wo);
    vx_pin(sf.depth); vx_pin(sf.roughness); vx_pin(sp.back);
    const int selLoop = float_as_bits(m4.z);
    const unsigned cached = (unsigned)float_as_bits(m4.w);
    // restir_slot's selection: a tap's light (from rr) or the RIS sample; both map entries read together
    const float4 eR = env_entry(a.sky, rr), eS = ls_entry(a.sky, ls0);
    LSample ls = invalid_ls();
    if (selLoop >= 0) light_from_entry(a, ls, rr, sf.pos, a.mesh.nInst > 0 && a.numLights > 0, eR);
    else ls = load_ls_entry(a, s, ls0, eS);
    if (rr.lightData != 0) {
        float piv = rr.targetPdf, piSum = rr.targetPdf * 1;
        for (int i = 0; i < 3; ++i) {
            if ((cached & (1u << i)) == 0) continue;
            float psv = i == 0 ? psv4.x : (i == 1 ? psv4.y : psv4.z);
            const float M = i == 0 ? psv4.w : (i == 1 ? m4.x : m4.y);
            if ((hits >> (8 * (1 + i))) & 0xFF) psv = 0.0f;  // oHit[4s + 1 + i]
            if (selLoop == i) piv = psv;
            piSum += psv * M;
        }
        finalize(rr, piv, piSum);
    }
    bool visible = false;
    if (ls.type != LtInvalid) {
        visible = !(hits & 0xFF);  // oHit[4s]
        if (!visible) { rr.lightData = 0; rr.weightSum = 0; }
    }
    V3 segRad(0.0f);
    if (ls.type != LtInvalid && rr.lightData != 0 && visible) segRad = shade_light(sf, skipAlbedo, ls, rr);
    a.resCur[pi] = rr;
    seg_end(a, s, px, py, meta, segRad, xyz(b), pdf, b.w != 0.0f, true, true, a.texEnabled ? sf.depth : 0.0f, sf.depth);
    store_meta(w, s, meta);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VX_WPE_FINISH))) void k_finish(TraceArgs a) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    int px, py;
    if (!slot_pixel(a, s, px, py)) return;
    finish_slot(a, s, px, py);
    // a one-segment pass ends here: every path of the slot's pixel has ended (in this kernel or in
    // the first half), so its spp accumulation follows (the k_accum launch folded in)
    if (a.accum && a.segments == 1) accum_px(a, (size_t)py * a.W + px);
}

// ----------------------------------------------------------------- instanced meshes
// The mesh pass of a traversal (launched only when the world has instanced meshes):
// a closest-hit ray's voxel result is replaced by a strictly closer mesh triangle (ties stay with
// the voxel face -- the oracle's definition; OptiX leaves the order of equal-t hits unspecified),
// back faces culled (RayGen.cu:52); a visibility ray is occluded by any triangle, either face, in
// [tmin, tmax] (closesthit.cu:616-625).  Mesh hit record: face 15, x = instance row, y = the
// triangle in BLAS leaf order, z = the mesh's triangle index, id = block.
VX_D bool mesh_closest_update(const TraceArgs &a, V3 o, V3 d, float tmax, int4 &hp, float &t) {
    const bool vox = ((hp.w >> 12) & 1) != 0;
    Best b{vox ? t : tmax, 0.0f, 0.0f, -1, -1, -1};
    ScratchStack st;
    mesh_walk<false>(a.mesh, o, d, V3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z), 0.0f, 1, b, st);
    if (b.inst < 0 || (vox && !(b.t < t))) return false;
    hp = make_int4(b.inst, b.leaf, b.tri, 15 | (a.meshRow[b.inst].w << 4) | (1 << 12));
    t = b.t;
    return true;
}
// camera (mode 2) and continuing path rays (mode 0), after k_closest
__global__ __launch_bounds__(256) void k_mesh_slots(TraceArgs a, int mode) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    int px, py;
    if (!slot_pixel(a, s, px, py)) return;
    const WaveBufs &w = a.wb;
    if (mode == 0 && !(w.pMeta[s].x & F_ALIVE)) return;
    int4 hp = w.cHit[s];
    float t = w.cT[s];
    if (mesh_closest_update(a, xyz(w.pPos[s]), xyz(w.pDir[s]), kRayMax, hp, t)) {
        w.cHit[s] = hp;
        w.cT[s] = t;
    }
}
// a ray queue, after its voxel traversal (k_queue + k_resume)
template <bool OCC>
__global__ __launch_bounds__(256) void k_mesh_queue(TraceArgs a, int q) {
    const WaveBufs &w = a.wb;
    const unsigned n = w.qCount[q];
    const unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 ro = w.qO[i], rd = w.qD[i];
    const int id = w.qId[i];
    const V3 o = xyz(ro), d = xyz(rd);
    if (OCC) {
        if (w.oHit[id]) return;
        Best b{rd.w, 0.0f, 0.0f, -1, -1, -1};
        ScratchStack st;
        mesh_walk<true>(a.mesh, o, d, V3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z), ro.w, 0, b, st);
        if (b.inst >= 0) w.oHit[id] = 1;
    } else {
        int4 hp = w.cHit[id];
        float t = w.cT[id];
        if (mesh_closest_update(a, o, d, rd.w, hp, t)) {
            w.cHit[id] = hp;
            w.cT[id] = t;
        }
    }
}

// C2 bring-up mode: primary hit G-buffer + sky, no NEE
__global__ __launch_bounds__(256) void k_primary_gbuffer(TraceArgs a) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    int px, py;
    if (!slot_pixel(a, s, px, py)) return;
    const WaveBufs &w = a.wb;
    const size_t pi = (size_t)py * a.W + px;
    const Hit h = unpack_hit(w.cHit[s], w.cT[s]);
    const V3 o = a.cam.pos, d = camera_ray(a, px, py);  // the camera ray, as k_closest traced it
    if (!h.hit) {
        a.resCur[pi] = empty_res();
        a.cur.albedo[pi] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
        a.cur.material[pi] = (float)0xFFFF;
        a.cur.normalRough[pi] = make_float4(0.0f, -1.0f, 0.0f, 0.0f);
        a.cur.geoNormalThin[pi] = make_float4(0.0f, -1.0f, 0.0f, 0.0f);
        a.cur.matParam[pi] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const V3 e = sky_emission(a.sky, d);
        store_rec_sky(a, pi, kRayMax);
        a.cur.depth[pi] = kRayMax;
        a.illum[pi] = make_float4(e.x, e.y, e.z, kRayMax);
        return;
    }
    V3 fp, bp, ng;
    hit_frame(h, o, d, fp, bp, ng);
    const MatDev &m = a.mats[h.id];
    const V3 alb = max3(V3(m.albedo[0], m.albedo[1], m.albedo[2]), V3(0.001f));
    a.cur.material[pi] = (float)m.materialId;
    a.cur.normalRough[pi] = make_float4(ng.x, ng.y, ng.z, m.roughness);
    a.cur.geoNormalThin[pi] = make_float4(ng.x, ng.y, ng.z, 0.0f);
    a.cur.matParam[pi] = make_float4(m.metallic ? 1.0f : 0.0f, m.translucency, 0.0f, 0.0f);
    a.cur.albedo[pi] = make_float4(alb.x, alb.y, alb.z, 1.0f);
    store_rec(a, pi, ng, m.roughness, m.metallic != 0, alb, h.t);
    if (a.writeMotion) a.motion[pi] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    a.cur.depth[pi] = h.t;
    a.illum[pi] = make_float4(0.0f, 0.0f, 0.0f, h.t);
}

template <bool BOX>
__global__ __launch_bounds__(256) void k_probe(WorldDev w, int n, const float *rays, int *out, float *t, int mode) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float *r = rays + 8 * i;
    const V3 o(r[0], r[1], r[2]), d(r[3], r[4], r[5]);
    int *q = out + 6 * i;
    if (mode & 4) {
        // the straggler path: every iteration goes through dda_save / dda_resume (the state
        // k_queue and k_resume hand over between launches), one iteration per "launch"
        Hit h{0, 0, 0, 0, -1, 0, kRayMax};
        Dda st;
        const bool occ = (mode & 2) != 0;
        const float tmin = occ ? r[6] : 0.0f;
        int rc = occ ? dda_begin<true, BOX>(w, o, d, tmin, r[7], st, h) : dda_begin<false, BOX>(w, o, d, 0.0f, r[7], st, h);
        while (rc == DdaRun) {
            const DdaSaved sv = dda_save(st, i);
            dda_resume<BOX>(w, o, d, tmin, r[7], sv, st);
            rc = occ ? dda_iter<true, BOX, GlobalBricks, true>(w, st, h) : dda_iter<false, BOX, GlobalBricks, true>(w, st, h);
        }
        if (occ) {
            q[0] = rc == DdaEvent ? 1 : 0;
            q[1] = q[2] = q[3] = q[4] = q[5] = 0;
            t[i] = 0.0f;
            return;
        }
        if (rc != DdaEvent) h = Hit{0, 0, 0, 0, -1, 0, kRayMax};
        q[0] = h.hit; q[1] = h.x; q[2] = h.y; q[3] = h.z; q[4] = h.face; q[5] = h.id;
        t[i] = h.t;
        return;
    }
    if (mode == 2) {
        q[0] = dda_occluded<BOX, true>(w, o, d, r[6], r[7]) ? 1 : 0;
        q[1] = q[2] = q[3] = q[4] = q[5] = 0;
        t[i] = 0.0f;
        return;
    }
    const Hit h = dda_closest<BOX, GlobalBricks, true>(w, o, d, r[7]);
    q[0] = h.hit; q[1] = h.x; q[2] = h.y; q[3] = h.z; q[4] = h.face; q[5] = h.id;
    t[i] = h.t;
}

__global__ __launch_bounds__(256) void k_probe_rng(BlueNoiseDev bn, int n, const int *q, float *out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    out[i] = bn_rand(bn, q[4 * i], q[4 * i + 1], q[4 * i + 2], q[4 * i + 3]);
}

// rebuilds a slot's tap records from its planes (after a host write to the planes)
__global__ __launch_bounds__(256) void k_pack_rec(GBuf g, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 nr = g.normalRough[i], al = g.albedo[i], mp = g.matParam[i];
    g.rec[2 * i] = make_float4(nr.x, nr.y, nr.z, bits_as_float(float_as_bits(nr.w) | (mp.x == 1.0f ? (int)0x80000000u : 0)));
    g.rec[2 * i + 1] = make_float4(al.x, al.y, al.z, g.depth[i]);
}

}  // namespace

#ifdef VX_STATS
extern "C" int vxpt_debug_stats(unsigned long long *out64, int reset) {
    hipMemcpyFromSymbol(out64, HIP_SYMBOL(g_stats), sizeof(g_stats), 0, hipMemcpyDeviceToHost);
    hipMemcpyFromSymbol(out64 + 64, HIP_SYMBOL(g_hist), sizeof(g_hist), 0, hipMemcpyDeviceToHost);
    if (reset) {
        static const unsigned long long z[128] = {};
        hipMemcpyToSymbol(HIP_SYMBOL(g_stats), z, sizeof(g_stats), 0, hipMemcpyHostToDevice);
        hipMemcpyToSymbol(HIP_SYMBOL(g_hist), z, sizeof(g_hist), 0, hipMemcpyHostToDevice);
    }
    return 0;
}
#endif

hipError_t launch_pack_rec(const GBuf &g, size_t n, hipStream_t st) {
    hipLaunchKernelGGL(k_pack_rec, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g, n);
    return hipGetLastError();
}

hipError_t launch_probe_rng(const BlueNoiseDev &bn, int n, const int *q, float *out, hipStream_t st) {
    hipLaunchKernelGGL(k_probe_rng, dim3((n + 255) / 256), dim3(256), 0, st, bn, n, q, out);
    return hipGetLastError();
}

hipError_t launch_probe(const WorldDev &w, int n, const float *rays, int *out, float *t, int mode, hipStream_t st) {
    if (w.bbox) hipLaunchKernelGGL(k_probe<true>, dim3((n + 255) / 256), dim3(256), 0, st, w, n, rays, out, t, mode);
    else hipLaunchKernelGGL(k_probe<false>, dim3((n + 255) / 256), dim3(256), 0, st, w, n, rays, out, t, mode);
    return hipGetLastError();
}

namespace {
struct Launcher {
    const TraceArgs &a;
    hipStream_t st;
    dim3 g, b;
    bool mesh, box;
    Launcher(const TraceArgs &a_, hipStream_t st_)
        : a(a_), st(st_), g((a_.nSlots + 255) / 256), b(256), mesh(a_.mesh.nInst > 0), box(a_.world.bbox != nullptr) {}
    // the walks use the empty-box tables when the world has them, else the cubes
    void closest(int mode) {
        if (box && a.ldsBricks) hipLaunchKernelGGL((k_closest<true, true>), g, b, 0, st, a, mode);
        else if (box) hipLaunchKernelGGL((k_closest<true, false>), g, b, 0, st, a, mode);
        else hipLaunchKernelGGL((k_closest<false, false>), g, b, 0, st, a, mode);
    }
    // a ray queue's traversal: iteration-capped pass + straggler continuation (+ the mesh pass).  The
    // stragglers' grid: a fixed number of workgroups per CU (their count is on the device; each wave
    // reads it and strides over its shard), vxpt_tuning.resume_wg_per_cu per CU (the sweep in DESIGN.md)
    template <bool OCC, bool BOX>
    void trav_t(int q, dim3 gq, int shardCap) {
        const dim3 gr(a.numCU * (a.resumeWgPerCU > 0 ? a.resumeWgPerCU : 16));
        hipLaunchKernelGGL((k_queue<OCC, BOX>), gq, b, 0, st, a, q, a.iterCap, shardCap);
        // a path's later segments (queues of segment >= 1) trace what is left of the pass's paths:
        // few rays, so their traversals wait on the longest walks (tuning later_split: after 8 more
        // iterations one lane each, the rest in pieces)
        const bool later = (q >> 2) > 0 && a.laterSplit > 1;
        const int cap2 = later ? 8 : a.iterCap2, G = later ? a.laterSplit : a.resumeSplit;
        if (G > 1 && cap2 == 0) {
            hipLaunchKernelGGL((k_resume_split<OCC, BOX>), gr, b, 0, st, a, q, 1, shardCap, G);
            return;
        }
        hipLaunchKernelGGL((k_resume<OCC, BOX>), gr, b, 0, st, a, q, 1, shardCap, cap2);
        // (tuning iter_cap3: one more capped level, its stragglers compacted again before the last;
        // the straggler states ping-pong, so level 3 reuses the level-1 buffer, consumed by then)
        int last = 2;
        // (not for the later segments' queues: their ladder 8 + pieces; with the third level 4/4-bounce frames
        // 14.25 -> 15.01 ms)
        if (cap2 > 0 && !later && a.iterCap3 > 0) {
            hipLaunchKernelGGL((k_resume<OCC, BOX>), gr, b, 0, st, a, q, 2, shardCap, a.iterCap3);
            last = 3;
            if (a.iterCap4 > 0) {
                hipLaunchKernelGGL((k_resume<OCC, BOX>), gr, b, 0, st, a, q, 3, shardCap, a.iterCap4);
                last = 4;
            }
        }
        if (cap2 > 0 && G > 1)
            hipLaunchKernelGGL((k_resume_split<OCC, BOX>), gr, b, 0, st, a, q, last, shardCap, G);
        else if (cap2 > 0)
            hipLaunchKernelGGL((k_resume<OCC, BOX>), gr, b, 0, st, a, q, last, shardCap, 0);
    }
    void trav(bool occ, int q, int cap) {
        const dim3 gq((cap + 255) / 256);
        const int shardCap = (int)((gq.x + kShards - 1) / kShards) * 256;
        if (occ && box) trav_t<true, true>(q, gq, shardCap);
        else if (occ) trav_t<true, false>(q, gq, shardCap);
        else if (box) trav_t<false, true>(q, gq, shardCap);
        else trav_t<false, false>(q, gq, shardCap);
        if (mesh) {
            if (occ) hipLaunchKernelGGL(k_mesh_queue<true>, gq, b, 0, st, a, q);
            else hipLaunchKernelGGL(k_mesh_queue<false>, gq, b, 0, st, a, q);
        }
    }
    // a segment's shading up to its NEE visibility rays (the shading kernels' mesh variants -- mesh hits,
    // thin films, local lights -- run only with meshes)
    void first_half(int seg) {
        if (mesh) hipLaunchKernelGGL(k_shade<true>, g, b, 0, st, a, seg);
        else hipLaunchKernelGGL(k_shade<false>, g, b, 0, st, a, seg);
        trav(false, 4 * seg + 1, a.nSlots);
        if (mesh) hipLaunchKernelGGL(k_nee<true>, g, b, 0, st, a, seg);
        else hipLaunchKernelGGL(k_nee<false>, g, b, 0, st, a, seg);
        trav(true, 4 * seg + 2, a.nSlots);
    }
    void restir(int seg) {
        const bool w4 = a.restirWaves == 4;
        if (mesh) hipLaunchKernelGGL((w4 ? k_restir<true, 4> : k_restir<true, VX_WPE_RESTIR>), g, b, 0, st, a, seg);
        else hipLaunchKernelGGL((w4 ? k_restir<false, 4> : k_restir<false, VX_WPE_RESTIR>), g, b, 0, st, a, seg);
    }
};
}  // namespace

// A pass's first half: camera rays, segment 0's shading, BRDF-candidate and RIS visibility rays.
// It reads nothing of the previous pass (G-buffer slot, reservoirs): it writes its own slot, its
// state set, and its own radiance plane.
hipError_t launch_trace_front(const TraceArgs &a, hipStream_t st) {
    Launcher L(a, st);
    L.closest(2);
    if (a.primaryOnly) {  // C2 bring-up: the voxel G-buffer only
        hipLaunchKernelGGL(k_primary_gbuffer, L.g, L.b, 0, st, a);
        return hipGetLastError();
    }
    // secondary / visibility rays go through the compacted queues; their counters (4 per segment)
    // are zeroed once per pass, by k_closest above
    if (L.mesh) hipLaunchKernelGGL(k_mesh_slots, L.g, L.b, 0, st, a, 2);
    L.first_half(0);
    return hipGetLastError();
}

// The second half: segment 0's temporal reuse (the first reader of the previous pass's G-buffer and
// reservoirs -- a band's halo rows of them may still be in flight on the exchange stream), its rays,
// k_finish (reservoir store), the later segments, and the spp accumulation.
hipError_t launch_trace_back(const TraceArgs &a, hipStream_t st, hipEvent_t waitBeforeRestir) {
    Launcher L(a, st);
    if (waitBeforeRestir) hipStreamWaitEvent(st, waitBeforeRestir, 0);
    L.restir(0);
    L.trav(true, 3, 4 * a.nSlots);
    hipLaunchKernelGGL(k_finish, L.g, L.b, 0, st, a);
    for (int seg = 1; seg < a.segments; ++seg) {
        L.closest(0);
        if (L.mesh) hipLaunchKernelGGL(k_mesh_slots, L.g, L.b, 0, st, a, 0);
        L.first_half(seg);
        L.restir(seg);
    }
    if (a.accum && a.segments > 1) hipLaunchKernelGGL(k_accum, L.g, L.b, 0, st, a);
    return hipGetLastError();
}

}  // namespace vx
