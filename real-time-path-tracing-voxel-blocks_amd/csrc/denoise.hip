// vxpt -- ReLAX-style diffuse denoiser on gfx950.
//
// Passes and their reference anchors (renderer/denoising/*):
//   firefly  FireflyBoilingFilter (FireflyFilter.h:9-251): detect + filter into a
//            compact list, applied by a second launch so every read sees the
//            pre-filter illumination (the reference's in-place write races).
//   TA       TemporalAccumulation<8,1> (TemporalAccumulation.h:8-449)
//   HF       HistoryFix (HistoryFix.h:6-119)
//   HC       HistoryClamping<8,2> (HistoryClamping.h:6-219)
//   ASmem    AtrousSmem<8,2> (AtrousSmem.h:9-302)
//   Atrous   Atrous (Atrous.h:6-158), x3; the last one also writes the output
//            (BufferCopySky + BufferCopyNonSky, BufferCopy.h:6-116 fused in).
// Buffers are SoA float4/float planes, W*H row-major, 16-B lanes (dwordx4).
// The reference's Float4 operator behaviour (w taken from z) is reproduced
// because the variance / second-moment channel depends on it.
#include "vx_internal.hpp"

#ifdef VX_EXACT_DENOISE
// experiment build (libvxpt_exact.so): the reference's compensated dots and IEEE sqrt/exp in
// every weight, to separate the deliberate numeric deviations from other differences
#define dot_fast dot
#define luminance_fast luminance
#define __expf expf
#define __builtin_amdgcn_sqrtf sqrtf
#endif

namespace vx {
namespace {

constexpr float kRange = 500000.0f;

VX_HD int cl(int v, int n) { return v < 0 ? 0 : (v >= n ? n - 1 : v); }
VX_HD V4 f4(float4 v) { return V4(v.x, v.y, v.z, v.w); }
VX_HD float4 tf(V4 v) { return make_float4(v.x, v.y, v.z, v.w); }
VX_HD V4 ld4(const float4 *b, int W, int H, int x, int y) { return f4(b[(size_t)cl(y, H) * W + cl(x, W)]); }
VX_HD float ld1(const float *b, int W, int H, int x, int y) { return b[(size_t)cl(y, H) * W + cl(x, W)]; }
// 16-bit read of the R32F material plane at byte offset 2x (Load2DUshort1 semantics)
VX_HD float ld_ushort(const float *b, int W, int H, int x, int y) {
    const int ux = clampi(x, 0, 2 * W - 1);
    const uint16_t *row = reinterpret_cast<const uint16_t *>(b + (size_t)cl(y, H) * W);
    return (float)row[ux];
}
VX_HD V3 world_pos(const CamDev &c, int x, int y, float depth) {
    const V2 uv = (V2((float)x, (float)y) + 0.5f) * c.invRes;
    return c.pos + c.uv_to_dir(uv) * depth;
}
VX_HD V3 xyz4(float4 v) { return V3(v.x, v.y, v.z); }
// world position of the (edge-clamped) pixel's hit, from the per-frame plane
VX_HD V3 wp(const DenoiseArgs &a, int x, int y) { return xyz4(a.wpos[(size_t)cl(y, a.H) * a.W + cl(x, a.W)]); }
// the packed plane's value of a pixel: world position of its primary hit and, in w, its 16-bit
// material read (Load2DUshort1 quirk, ld_ushort) for the a-trous / history-fix material tests,
// -1 for sky (no tap weight)
VX_HD float4 wpos_px(const DenoiseArgs &a, int x, int y, float z, float mat16) {
    const V3 p = world_pos(a.cam, x, y, z);
    return make_float4(p.x, p.y, p.z, z > kRange ? -1.0f : mat16);
}
VX_HD float4 wpos_px(const DenoiseArgs &a, int x, int y, float z) {
    return wpos_px(a, x, y, z, ld_ushort(a.material, a.W, a.H, x, y));
}
VX_D float smooth_step10(float x) {  // SmoothStep(1, 0, x)
    // (x - 1) / (0 - 1): dividing by -1 is exact and round-to-nearest is sign
    // symmetric, so this equals 1 - x bit for bit -- without a division per tap
    const float t = saturate(1.0f - x);
    return t * t * (3.0f - 2.0f * t);
}
VX_D float acos_approx(float x) { return sqrtf(2.0f) * sqrtf(saturate(1.0f - x)); }
VX_D float nonexp_w(float x, float px) { return smooth_step10(fabsf(x * px + 0.0f)); }
VX_D float normal_weight_param(float roughness, float af) {
    const float r = saturate(roughness), p = saturate(af);
    const float angle = atanf(r * r * p / (1.0f - p + 1e-6f));
    return 1.0f / fmaxf(angle, 1e-6f);
}
VX_D float plane_w(V3 c, V3 n, V3 s, float thr) { return fabsf(dot(s - c, n)) < thr ? 1.0f : 0.0f; }
// plane_w with the same decision at a third of the cost: an FMA dot with a bound on its distance
// to the compensated one (|fma dot - exact| <= 2u sum|a_i b_i|, |compensated - exact| <= u |exact|);
// only taps within that margin of the threshold evaluate the compensated dot.  NaN/inf fall back.
VX_D float plane_w_fast(V3 c, V3 n, V3 s, float thr) {
    const V3 d = s - c;
    const float f = fabsf(dot_fast(d, n));
    const float mag = fabsf(d.x * n.x) + fabsf(d.y * n.y) + fabsf(d.z * n.z);
    const float e = 4.0e-7f * (mag + thr) + 1.0e-30f;
    if (f + e < thr) return 1.0f;
    if (f - e >= thr) return 0.0f;
    return plane_w(c, n, s, thr);
}
// hardware square root (1 ulp) and exponential for the stencils' continuous weights: the
// IEEE sequences are ~12 and ~16 VALU ops per tap; the weights' error stays far below the
// denoiser's 1e-4 parity tolerance
VX_D float acos_approx_fast(float x) { return sqrtf(2.0f) * __builtin_amdgcn_sqrtf(saturate(1.0f - x)); }

// float4 plane behind a buffer descriptor: 32-bit offsets, hardware range check (a tap outside the
// plane reads 0, and every out-of-frame tap's weight is 0), no clamping or 64-bit address math
struct Plane4 {
    __amdgpu_buffer_rsrc_t r;
    VX_D Plane4(const float4 *p, int n) : r(__builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, n * 16, 0x00020000)) {}
    VX_D V4 operator[](int i) const {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, i * 16, 0, 0);
        return V4(__int_as_float(v[0]), __int_as_float(v[1]), __int_as_float(v[2]), __int_as_float(v[3]));
    }
};
VX_HD V3 rgb_to_ycocg(V3 c) { return V3(0.25f * (c.x + 2.0f * c.y + c.z), c.x - c.z, c.y - 0.5f * (c.x + c.z)); }
VX_HD V3 ycocg_to_rgb(V3 c) { return V3(c.x + 0.5f * (c.y - c.z), c.x + 0.5f * c.z, c.x - 0.5f * (c.y + c.z)); }
VX_D uint32_t seq_hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
    return x;
}
VX_D uint32_t explode(uint32_t x) {
    x = (x | (x << 8)) & 0x00FF00FFu; x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u; x = (x | (x << 1)) & 0x55555555u;
    return x;
}

// ---------------------------------------------------------------- firefly
// 256-thread workgroups over 64x4 pixels; each wave covers two 8x4 tiles (one per 32-lane half of
// the wave).  The same launch writes the packed world-position plane (wpos_px) over rows
// [wy0, wy1) -- the band and the halo rows the later stencils read -- so the filter's own
// neighbour positions come from the depth directly (the same world_pos arithmetic).
// Detected pixels are listed (ffCand) for k_firefly_filter; filtered pixels are listed per 16x16
// tile of the band (ffCount[tile], entries at tile*256):
// k_temporal applies its tile's entries before reading the radiance (or k_firefly_apply does,
// when no temporal pass follows), so every read of this pass sees the pre-filter values (the
// reference's in-place write races).
// The filter of one detected firefly (FireflyFilter.h:131-220), by a whole wave: lane k < 8 fetches
// and tests neighbour k (row-major 3x3 without the centre) in parallel, then every lane combines the
// eight results in the reference's order (the same arithmetic as the loop over neighbours), and
// lane 0 lists the filtered pixel for its 16x16 tile.  The candidate's values are wave-uniform.
VX_D void firefly_filter_wave(const DenoiseArgs &a, int lane, int x, int y, float cd, const Reservoir &r,
                              float nSum, int nCnt) {
    const int W = a.W, H = a.H;
    const size_t i = (size_t)y * W + x;
    const float cw = r.weightSum;
    const float minWeight = 5.0f, wThr = 80.0f, nThr = 0.8f, depthSigma = 0.02f;
    const V4 cc4 = f4(a.illum[i]);
    const float cLum = luminance(cc4.xyz());
    V3 cN = f4(a.normalRough[i]).xyz();
    const float cl_ = length(cN);
    if (cl_ > 0.0f) cN /= cl_; else cN = V3(0.0f, 1.0f, 0.0f);
    const float cMat = a.material[i];
    const V3 cWP = world_pos(a.cam, x, y, cd);
    const float g[3] = {1.0f, 2.0f, 1.0f};
    const float depthScale = fmaxf(fabsf(cd), 1.0f);
    const float nwp = normal_weight_param(1.0f, 0.25f);
    // this lane's neighbour
    const int t = lane < 4 ? lane : lane + 1;
    const int sx = x + t % 3 - 1, sy = y + t / 3 - 1;
    const int inF = lane < 8 && sx >= 0 && sy >= 0 && sx < W && sy < H;
    V4 sc4;
    float tw = 0.0f, score = 0.0f;
    int useTw = 0, cand = 0;
    Reservoir nr = Reservoir{0u, 0u, 0.f, 0.f, 0.f};
    if (inF) {
        const size_t j = (size_t)sy * W + sx;
        sc4 = f4(a.illum[j]);
        const float sd = a.depth[j];
        const V3 sN0 = f4(a.normalRough[j]).xyz();
        const float sMat = a.material[j];
        nr = a.reservoir[j];
        const float gw = g[abs(t % 3 - 1)] * g[abs(t / 3 - 1)];
        do {  // the reference's tests in order; a failed test drops the neighbour from both weights
            if (sd > kRange) break;
            V3 sN = sN0;
            const float sl = length(sN);
            if (sl <= 0.0f) break;
            sN /= sl;
            const float nd = dot(cN, sN);
            if (nd < nThr) break;
            if (fabsf(sMat - cMat) > 0.5f) break;
            const V3 sWP = world_pos(a.cam, sx, sy, sd);
            if (plane_w(cWP, cN, sWP, depthSigma * depthScale) <= 0.0f) break;
            const float nw = nonexp_w(acos_approx(clampf(nd, -1.0f, 1.0f)), nwp);
            const float dw = expf(-fabsf(sd - cd) / (depthScale * depthSigma + 1e-6f));
            const float lw = expf(-fabsf(luminance(sc4.xyz()) - cLum) * a.p.phiL);
            tw = gw * 1.0f * nw * dw * lw;
            useTw = tw > 1e-5f;
            if (nr.lightData != 0 && isfinite(nr.weightSum) && nr.weightSum > 0.0f && nr.weightSum < cw) {
                cand = 1;
                score = fabsf(sd - cd) / (depthScale + 1e-6f) + (1.0f - clampf(nd, 0.0f, 1.0f)) +
                        0.25f * fabsf(nr.weightSum - cw);
            }
        } while (false);
    }
    V4 filt = cc4;
    float filtW = 1.0f;
    V4 fb = cc4 * (g[0] * g[0]);
    float fbW = g[0] * g[0];
    Reservoir best = r;
    float bestScore = 3.402823466e+38f;
    bool repl = false;
#pragma unroll 1
    for (int k = 0; k < 8; ++k) {
        if (!__shfl(inF, k)) continue;
        const int tk = k < 4 ? k : k + 1;
        const float gw = g[abs(tk % 3 - 1)] * g[abs(tk / 3 - 1)];
        const V4 s4(__shfl(sc4.x, k), __shfl(sc4.y, k), __shfl(sc4.z, k), __shfl(sc4.w, k));
        fb += s4 * gw;
        fbW += gw;
        if (__shfl(useTw, k)) {
            const float twk = __shfl(tw, k);
            filt += s4 * twk;
            filtW += twk;
        }
        if (__shfl(cand, k)) {
            const float sk = __shfl(score, k);
            if (sk < bestScore) {
                bestScore = sk;
                best = Reservoir{(uint32_t)__shfl((int)nr.lightData, k), (uint32_t)__shfl((int)nr.uvData, k),
                                 __shfl(nr.weightSum, k), __shfl(nr.targetPdf, k), __shfl(nr.M, k)};
                repl = true;
            }
        }
    }
    if (lane != 0) return;
    V4 outc;
    if (filtW > 0.0f) outc = filt / filtW;
    else if (fbW > 0.0f) outc = fb / fbW;
    else outc = cc4;
    Reservoir dst;
    if (repl) dst = best;
    else {
        dst = r;
        const float avg = (nCnt > 0) ? (nSum / float(nCnt)) : minWeight;
        float tgt = (nCnt > 0) ? (avg * wThr) : minWeight;
        tgt = fmaxf(tgt, minWeight);
        dst.weightSum = fminf(dst.weightSum, tgt);
    }
    const int by = y - a.y0;
    const uint32_t tile = (uint32_t)((by >> 4) * ((W + 15) / 16) + (x >> 4));
    const uint32_t slot = tile * 256u + atomicAdd(a.ffCount + tile, 1u);
    a.ffIndex[slot] = (uint32_t)((by & 15) * 16 + (x & 15));
    a.ffColor[slot] = tf(outc);
    a.ffRes[slot] = dst;
}

// 6 waves/SIMD (80 VGPRs, 12 B/lane of spill in the rare filter): 26.2 -> 23.9 us against the compiler's
// 84 VGPRs at 5; at 8 (64 VGPRs) the spills reach the detection path: 31.9 us
#ifndef VX_WPE_FF
#define VX_WPE_FF 6  // occupancy bound of k_firefly (waves per SIMD; 1 = the compiler's choice)
#endif
template <bool FUSED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VX_WPE_FF))) void k_firefly(DenoiseArgs a, int wy0,
                                                                                                 int wy1, int detect) {
    const int W = a.W, H = a.H;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int l32 = lane & 31;
    // a wave = two 8x4 tiles side by side, a block = 64 x 4 pixels: row segments of 64 pixels
    // (the tiles are the reference's 8x4 ones; the band and wy0 start on 8-row boundaries)
    const int x = blockIdx.x * 64 + wv * 16 + (lane >> 5) * 8 + (l32 & 7);
    const int y = wy0 + blockIdx.y * 4 + (l32 >> 3);
    const bool inb = x < W && y < wy1;
    const size_t i = (size_t)y * W + x;
    const float cd = inb ? a.depth[i] : 0.0f;
    const bool sky = inb && cd > kRange;
    const bool inBand = detect && inb && y >= a.y0 && y < a.y1;
    // the reservoir and the 16-bit material are read beside the depth (not behind the sky test): one
    // memory round trip
    Reservoir r = Reservoir{0u, 0u, 0.f, 0.f, 0.f};
    if (inBand) r = a.reservoir[i];
    const float mat16 = inb ? ld_ushort(a.material, W, H, x, y) : 0.0f;
    if (inb) a.wpos[i] = wpos_px(a, x, y, cd, mat16);
    const bool valid = inBand && !sky && r.lightData != 0 && isfinite(r.weightSum) && r.weightSum > 0.0f;
    float v = valid ? r.weightSum : 0.0f;
    unsigned cnt = valid ? 1u : 0u;
    for (int off = 16; off > 0; off >>= 1) {
        v += __shfl_down(v, off, 32);
        cnt += __shfl_down(cnt, off, 32);
    }
    const float tileSum = __shfl(v, 0, 32);
    const unsigned tileCnt = __shfl(cnt, 0, 32);
    const float cw = r.weightSum;
    const float nSum = tileSum - cw;
    const int nCnt = (int)tileCnt - 1;
    const float minWeight = 5.0f, wThr = 80.0f;
    bool firefly = false;
    if (valid && cw >= minWeight) {
        if (nCnt <= 0) firefly = true;
        else {
            const float avg = nSum / float(nCnt);
            if (avg > 0.0f && cw > avg * wThr) firefly = true;
        }
    }
    if (FUSED) {
        // the wave filters its own detections, one at a time (the filter reads only this pass's
        // inputs, and the tile sums are the wave's)
        unsigned long long m = __ballot(firefly);
        while (m) {
            const int k = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            const int fx = __shfl(x, k), fy = __shfl(y, k);
            const Reservoir fr{(uint32_t)__shfl((int)r.lightData, k), (uint32_t)__shfl((int)r.uvData, k),
                               __shfl(r.weightSum, k), __shfl(r.targetPdf, k), __shfl(r.M, k)};
            firefly_filter_wave(a, lane, fx, fy, __shfl(cd, k), fr, __shfl(nSum, k), __shfl(nCnt, k));
        }
        return;
    }
    // detected pixels are filtered by k_firefly_filter, a wave per pixel: the filter's registers
    // would cut this pass's occupancy (32 -> 84 VGPRs inline)
    if (firefly) a.ffCand[atomicAdd(a.ffCandCount, 1u)] = make_uint4((uint32_t)i, __float_as_uint(nSum), (uint32_t)nCnt, 0u);
}

// the detected fireflies (~100 on the bench scene at 1080p): one wave per pixel, grid-stride
__global__ __launch_bounds__(64) void k_firefly_filter(DenoiseArgs a) {
    const uint32_t n = *a.ffCandCount;
    for (uint32_t s = blockIdx.x; s < n; s += gridDim.x) {
        const uint4 c = a.ffCand[s];
        const size_t i = c.x;
        firefly_filter_wave(a, threadIdx.x, (int)(i % (size_t)a.W), (int)(i / (size_t)a.W), a.depth[i], a.reservoir[i],
                            __uint_as_float(c.y), (int)c.z);
    }
}

// a tile's firefly list entry k: written back to the radiance and reservoir planes
VX_D size_t ff_apply(const DenoiseArgs &a, unsigned tile, unsigned k, float4 &col) {
    const unsigned tilesX = (a.W + 15) / 16, s = tile * 256 + k, p = a.ffIndex[s];
    const size_t i = (size_t)(a.y0 + (tile / tilesX) * 16 + (p >> 4)) * a.W + (tile % tilesX) * 16 + (p & 15);
    col = a.ffColor[s];
    a.illum[i] = col;
    a.reservoir[i] = a.ffRes[s];
    return i;
}

// the lists' consumer when no temporal pass runs (frame 0, temporal accumulation off, or a band
// whose filtered rows travel to its neighbours before the next pass): one workgroup per tile;
// the count is reset for the next frame
__global__ __launch_bounds__(256) void k_firefly_apply(DenoiseArgs a) {
    const unsigned tile = blockIdx.y * ((a.W + 15) / 16) + blockIdx.x;
    if (tile == 0 && threadIdx.x == 0) *a.ffCandCount = 0u;  // k_firefly_filter has finished
    const unsigned n = a.ffCount[tile];
    if (n == 0) return;
    float4 col;
    if (threadIdx.x < n) ff_apply(a, tile, threadIdx.x, col);
    __syncthreads();
    if (threadIdx.x == 0) a.ffCount[tile] = 0u;
}

// ---------------------------------------------------------------- frame 0
__global__ __launch_bounds__(256) void k_frame0(DenoiseArgs a) {
    const size_t i = (size_t)a.y0 * a.W + (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)a.y1 * a.W) return;
    const float4 v = a.illum[i];
    a.prevIllum[i] = v;
    a.prevFast[i] = v;
    a.histLen[i] = 0.0f;
    a.prevHistLen[i] = 0.0f;
}

// XCD-aware 16x16 tiles (k_atrous, the L2-bound stencil): workgroup g runs on XCD g % 8, and XCD k walks
// the k-th vertical strip of tile columns in raster order, so the rows its resident workgroups
// tap stay in its own 4 MiB L2 (round-robin tiles share every halo line between XCDs).  The
// launch grid is grid_xcd(a); false = the grid's padding.  Measured: the 3 a-trous passes
// 57/55/71 -> 49/45/67 us; on the VALU-bound stencils (TA, HC, ASmem) the strips' uneven
// sky/ground mix across XCDs cost more than the L2 gained, so they keep raster tiles.
template <int TS = 16>
VX_D bool xcd_tile(const DenoiseArgs &a, int &tx, int &ty) {
    const int tilesX = (a.W + TS - 1) / TS, tilesY = (a.y1 - a.y0 + TS - 1) / TS;
    const int g = blockIdx.y * gridDim.x + blockIdx.x, k = g % 8, l = g / 8;
    const int sx0 = k * tilesX / 8, sw = (k + 1) * tilesX / 8 - sx0;
    if (sw <= 0 || l >= sw * tilesY) return false;
    tx = sx0 + l % sw;
    ty = l / sw;
    return true;
}

// 4x4-tile supertiles dealt round-robin to the 8 XCDs (workgroup g runs on XCD g % 8): a tile's
// neighbours inside its supertile run on its own XCD, so their shared apron rows and columns stay in
// that XCD's L2, and every XCD gets supertiles from the whole frame (the sky / ground mix stays even).
// Launch grid: grid_st(a).  False = the grid's padding.
template <int TS = 16>
VX_D bool st_tile(const DenoiseArgs &a, int &tx, int &ty) {
    const int tilesX = (a.W + TS - 1) / TS, tilesY = (a.y1 - a.y0 + TS - 1) / TS;
    const int sX = (tilesX + 3) / 4;
    const int g = blockIdx.x, k = g % 8, l = g / 8;
    const int S = (l / 16) * 8 + k, t = l % 16;
    tx = (S % sX) * 4 + (t & 3);
    ty = (S / sX) * 4 + (t >> 2);
    return tx < tilesX && ty < tilesY;
}
// the tile mapping of a stencil kernel: raster (blockIdx) or supertiles (st_tile)
template <bool ST, int TS = 16>
VX_D bool map_tile(const DenoiseArgs &a, int &tx, int &ty) {
    if (ST) return st_tile<TS>(a, tx, ty);
    tx = blockIdx.x;
    ty = blockIdx.y;
    return true;
}

// ---------------------------------------------------------------- TA
// The reprojected history is read from the previous frame's 4x4 tap window whose corner is
// (ox - 1, oy - 1), corners unused: the bicubic filters read its 12 inner taps, the custom bilinear
// filters, the smoothstep normal filter and the history length its central 2x2 -- every position is
// known once the pixel is reprojected.  Tap k of the bicubic order (TemporalAccumulation.h's sample
// order: (x1, y1 - 1), (x1 + 1, y1 - 1), (x1 - 1, y1), ...) sits at window column kBcC[k], row
// kBcR[k]; bilinear tap j (x0 + (j & 1), y0 + (j >> 1)) is bicubic tap bl_tap(j).
struct TaWin {
    int col[4], row[4];  // edge-clamped window columns, and rows times W
    VX_HD TaWin(int W, int H, int ox, int oy) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            col[k] = cl(ox - 1 + k, W);
            row[k] = cl(oy - 1 + k, H) * W;
        }
    }
    VX_HD int bc(int k) const {  // plane index of bicubic tap k
        const int c[12] = {1, 2, 0, 1, 2, 3, 0, 1, 2, 3, 1, 2}, r[12] = {0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3};
        return row[r[k]] + col[c[k]];
    }
};
VX_HD int bl_tap(int j) { return j == 0 ? 3 : (j == 1 ? 4 : (j == 2 ? 7 : 8)); }

// The filters take their taps' values from tap(k) (bicubic tap k, bilinear tap j), already fetched
template <bool kQuirk, class T>
VX_HD V4 bicubic12(const T &tap, int W, int H, V2 uv) {
    const V2 UV(uv.x * (float)W, uv.y * (float)H);
    const float fx = floorf(UV.x - 0.5f), fy = floorf(UV.y - 0.5f);
    const V2 fr = UV - V2(fx + 0.5f, fy + 0.5f), f2 = fr * fr, f3 = f2 * fr;
    const V2 w0 = f2 - 0.5f * (f3 + fr);
    const V2 w1 = 1.5f * f3 - 2.5f * f2 + 1.0f;
    const V2 w3 = 0.5f * (f3 - f2);
    const V2 w2 = 1.0f - w0 - w1 - w3;
    const float wt[12] = {w1.x * w0.y, w2.x * w0.y, w0.x * w1.y, w1.x * w1.y, w2.x * w1.y, w3.x * w1.y,
                          w0.x * w2.y, w1.x * w2.y, w2.x * w2.y, w3.x * w2.y, w1.x * w3.y, w2.x * w3.y};
    V4 out;
    V3 out3(0.0f);
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        sum += wt[k];
        const V4 v = tap(k);
        if (kQuirk) out += v * wt[k];
        else out3 += v.xyz() * wt[k];
    }
    if (kQuirk) { out /= sum; return out; }
    out3 /= sum;
    return V4(out3, 0.0f);
}
VX_HD void bilinear_taps(int W, int H, V2 uv, int &x0, int &y0, float w[4]) {
    const V2 UV(uv.x * (float)W, uv.y * (float)H);
    const float fx = floorf(UV.x - 0.5f), fy = floorf(UV.y - 0.5f);
    const V2 fr = UV - V2(fx + 0.5f, fy + 0.5f);
    const V2 w1 = fr, w0 = 1.0f - fr;
    x0 = (int)fx;
    y0 = (int)fy;
    w[0] = w0.x * w0.y; w[1] = w1.x * w0.y; w[2] = w0.x * w1.y; w[3] = w1.x * w1.y;
}
template <class T>
VX_HD V4 bilinear_custom4(const T &tap, int W, int H, V2 uv, const float cw[4]) {
    int x0, y0;
    float w[4];
    bilinear_taps(W, H, uv, x0, y0, w);
    V4 out;
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float wt = w[k] * cw[k];
        const float weight = (wt < 1e-6f) ? 1e-6f : wt;
        sum += weight;
        out += tap(k) * weight;
    }
    out /= sum;
    return out;
}
// v[k]: the plane at the bilinear taps (x0 + (k & 1), y0 + (k >> 1)), edge-clamped
VX_HD float bilinear_custom1(const float v[4], int W, int H, V2 uv, const float cw[4]) {
    int x0, y0;
    float w[4];
    bilinear_taps(W, H, uv, x0, y0, w);
    float out = 0.0f, sum = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float wt = w[k] * cw[k];
        const float weight = (wt < 1e-6f) ? 1e-6f : wt;
        sum += weight;
        out += v[k] * weight;
    }
    return out / sum;
}
template <class T>
VX_HD V3 bicubic_smoothstep3(const T &tap, int W, int H, V2 uv) {
    const V2 UV(uv.x * (float)W, uv.y * (float)H);
    const float fx = floorf(UV.x - 0.5f), fy = floorf(UV.y - 0.5f);
    const V2 fr = UV - V2(fx + 0.5f, fy + 0.5f), f2 = fr * fr, f3 = f2 * fr;
    const V2 w1 = -2.0f * f3 + 3.0f * f2;
    const V2 w0 = 1.0f - w1;
    const float wt[4] = {w0.x * w0.y, w1.x * w0.y, w0.x * w1.y, w1.x * w1.y};
    V3 out(0.0f);
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // tap k at (x0 + (k & 1), y0 + (k >> 1))
        sum += wt[k];
        out += tap(k) * wt[k];
    }
    out /= sum;
    return out;
}

// The reprojected history of a pixel (TemporalAccumulation.h loadSurfaceMotionBasedPrevData):
// the 12 depth taps' validity, the previous normal's test, the bicubic / custom-bilinear history
// and fast history, and the bilinear history length.  Three round trips, none behind a branch: the
// window's depth, normal and history-length taps; its radiance taps; its fast-history taps (the
// filter the validity chooses reads a subset of the same 12 positions).  The last two stay apart
// (VX_TA_FENCE) so that only one set of 12 taps is in flight in registers.  (A workgroup window of
// the planes staged in LDS was measured slower -- 95 -> 109 us, 137 VGPRs -- and removed, DESIGN.md
// Appendix A.)
#if defined(__HIP_DEVICE_COMPILE__)
#define VX_TA_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define VX_TA_FENCE() do { } while (0)
#endif
// The previous frame's planes at a plane index: plain loads (host tests) or, in the kernel, buffer
// loads with a 32-bit offset (one VGPR per tap address instead of a 64-bit pointer)
struct TaPlanesH {
    const DenoiseArgs *a;
    VX_HD float pz(int i) const { return a->prevDepth[i]; }
    VX_HD V3 pn(int i) const { return xyz4(a->prevNormalRough[i]); }
    VX_HD float ph(int i) const { return a->prevHistLen[i]; }
    VX_HD V3 pi(int i) const { return xyz4(a->prevIllum[i]); }
    VX_HD V3 pf(int i) const { return xyz4(a->prevFast[i]); }
};
VX_D __amdgpu_buffer_rsrc_t rsrc(const void *p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, bytes, 0x00020000);
}
VX_D float ldb1(__amdgpu_buffer_rsrc_t r, int i) { return __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, i * 4, 0, 0)); }
VX_D V3 ldb3(__amdgpu_buffer_rsrc_t r, int i) {  // xyz of a float4 plane
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, i * 16, 0, 0);
    return V3(__int_as_float(v[0]), __int_as_float(v[1]), __int_as_float(v[2]));
}
VX_D V4 ldb4(__amdgpu_buffer_rsrc_t r, int i) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, i * 16, 0, 0);
    return V4(__int_as_float(v[0]), __int_as_float(v[1]), __int_as_float(v[2]), __int_as_float(v[3]));
}
struct TaPlanesD {
    __amdgpu_buffer_rsrc_t z, n, h, i, f;
    VX_D explicit TaPlanesD(const DenoiseArgs &a)
        : z(rsrc(a.prevDepth, a.W * a.H * 4)), n(rsrc(a.prevNormalRough, a.W * a.H * 16)),
          h(rsrc(a.prevHistLen, a.W * a.H * 4)), i(rsrc(a.prevIllum, a.W * a.H * 16)), f(rsrc(a.prevFast, a.W * a.H * 16)) {}
    VX_D float pz(int k) const { return ldb1(z, k); }
    VX_D V3 pn(int k) const { return ldb3(n, k); }
    VX_D float ph(int k) const { return ldb1(h, k); }
    VX_D V3 pi(int k) const { return ldb3(i, k); }
    VX_D V3 pf(int k) const { return ldb3(f, k); }
};
struct TaHist {
    V4 prevI;
    V3 prevF;
    float bicValid, found, quality, hist;
};
template <class P>
VX_HD TaHist ta_history(const P &pl, int W, int H, const Qt &rot, V3 nIn, V2 prevUV, int ox, int oy, float estDepth,
                        const float thrv[4]) {
    const TaWin win(W, H, ox, oy);
    float pz[12], ph[4];
    V3 pn[4];
#pragma unroll
    for (int k = 0; k < 12; ++k) pz[k] = pl.pz(win.bc(k));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int t = win.bc(bl_tap(j));
        pn[j] = pl.pn(t);
        ph[j] = pl.ph(t);
    }
    TaHist r;
    float bicValid = 1.0f;
    float taps[4];
    // the 8 outer taps in the reference's order ((0,-1), (-1,0), (1,-1), (2,0), (-1,1), (0,2), (2,1),
    // (1,2) from (ox, oy)), then the central 2x2
    const int outer[8] = {0, 2, 1, 5, 6, 10, 9, 11};
#pragma unroll
    for (int k = 0; k < 8; ++k) bicValid *= fabsf(pz[outer[k]] - estDepth) > thrv[k >> 1] ? 0.0f : 1.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float v = fabsf(pz[bl_tap(k)] - estDepth) > thrv[k] ? 0.0f : 1.0f;
        bicValid *= v;
        taps[k] = v;
    }
    const V3 pnf = normalize(bicubic_smoothstep3([&](int j) { return pn[j]; }, W, H, prevUV));
    const V3 pnr = normalize(q_rotate(rot, pnf));
    if (dot(nIn, pnr) < 0.0f) {
        taps[0] = taps[1] = taps[2] = taps[3] = 0.0f;
        bicValid = 0.0f;
    }
    const bool useBic = bicValid > 0;
    // the radiance taps: only xyz is read (Float4 * scalar takes w from z, LinearMath.h:866-874)
    V3 pi[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) pi[k] = pl.pi(win.bc(k));
    const auto li = [&](int k) { return V4(pi[k], 0.0f); };
    const auto lib = [&](int j) { return V4(pi[bl_tap(j)], 0.0f); };
    // both filters evaluated and one selected: a branch between them would take the taps' fetches
    // into it (one dependent fetch after another on a wave whose lanes disagree)
    const V4 bicI = bicubic12<true>(li, W, H, prevUV), bilI = bilinear_custom4(lib, W, H, prevUV, taps);
    const V4 prevI = useBic ? bicI : bilI;
    VX_TA_FENCE();
    V3 pf[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) pf[k] = pl.pf(win.bc(k));
    const auto lf = [&](int k) { return V4(pf[k], 0.0f); };
    const auto lfb = [&](int j) { return V4(pf[bl_tap(j)], 0.0f); };
    const V3 bicF = bicubic12<false>(lf, W, H, prevUV).xyz(), bilF = bilinear_custom4(lfb, W, H, prevUV, taps).xyz();
    const V3 prevF = useBic ? bicF : bilF;
    r.prevI = V4(fmaxf(prevI.x, 0.0f), fmaxf(prevI.y, 0.0f), fmaxf(prevI.z, 0.0f), fmaxf(prevI.w, 0.0f));
    r.prevF = max3(prevF, V3(0.0f));
    r.found = (bicValid > 0.0f) ? 2.0f : 1.0f;
    int bx0, by0;
    float bw[4];
    bilinear_taps(W, H, prevUV, bx0, by0, bw);
    r.quality = (bicValid > 0) ? 1.0f : (bw[0] * 1.0f + bw[1] * 1.0f + bw[2] * 1.0f + bw[3] * 1.0f);
    if ((taps[0] * 1.0f + taps[1] * 1.0f + taps[2] * 1.0f + taps[3] * 1.0f) == 0.0f) {
        r.found = 0.0f; r.quality = 0.0f; r.hist = 0.0f;
    } else {
        r.hist = bilinear_custom1(ph, W, H, prevUV, taps);
    }
    r.bicValid = bicValid;
    return r;
}

// The pixel's own inputs and its 3x3 normals: the temporal pass's first memory round trip, fetched
// before anything else (k_temporal issues it ahead of the firefly-list hand-over, the normals staged
// in LDS for the workgroup's tile)
struct TaPix {
    float z;
    V3 cN, avgN, motion, illum;
};
VX_HD TaPix ta_pixel(const DenoiseArgs &a, int x, int y) {
    const int W = a.W, H = a.H;
    const size_t i = (size_t)y * W + x;
    TaPix p;
    p.z = a.depth[i];
    p.cN = f4(a.normalRough[i]).xyz();
    V3 avgN = p.cN;
    for (int ax = -1; ax <= 1; ++ax)
        for (int by = -1; by <= 1; ++by) {
            if (ax == 0 && by == 0) continue;
            avgN += ld4(a.normalRough, W, H, x + ax, y + by).xyz();
        }
    p.avgN = avgN;
    p.motion = f4(a.motion[i]).xyz();
    p.illum = f4(a.illum[i]).xyz();
    return p;
}

// Returns whether the history fix must filter the pixel (HistoryFix.h:20-22:
// non-sky and history <= 4; pixels past the denoising range keep last frame's length).
// p: the pixel's inputs (ta_pixel); ffCol: its firefly-filtered radiance, if any; pl: the previous
// frame's planes (TaPlanesH / TaPlanesD)
template <class P>
VX_HD bool temporal_px(const DenoiseArgs &a, const P &pl, const Qt &rot, int x, int y, const TaPix &p,
                       const float4 *ffCol) {
    const int W = a.W, H = a.H;
    const size_t i = (size_t)y * W + x;
    const float z = p.z;
    if (z > a.p.denoisingRange) return z <= kRange && a.histLen[i] <= 4.0f;
    const CamDev &cam = a.cam, &pc = a.prevCam;
    const V3 cN = p.cN;
    V3 avgN = p.avgN;
    avgN /= 9.0f;
    const V2 pixelUv = (V2((float)x, (float)y) + 0.5f) * V2(a.invW, a.invH);
    const V2 curUV = (V2((float)x, (float)y) + 0.5f) * cam.invRes;
    const V3 view = cam.uv_to_dir(curUV);
    const V3 cWP = cam.pos + view * z;  // world_pos(cam, x, y, z) term for term: the packed plane's value
    const V3 Vv = -normalize(view);
    const float NoV = fabsf(dot(cN, Vv));
    const V3 prevWP = cWP + p.motion;
    const V2 prevUV = pc.dir_to_uv(normalize(prevWP - pc.pos));
    const V3 illum = ffCol ? xyz4(*ffCol) : p.illum;
    const float m1 = luminance(illum), m2 = m1 * m1;
    const V3 camDelta = pc.pos - cam.pos;
    float par1, par2;
    {
        const V2 u1 = pc.dir_to_uv(normalize((prevWP + camDelta) - pc.pos));
        const V2 d1 = (u1 - pixelUv) * V2((float)W, (float)H);
        par1 = sqrtf(d1.x * d1.x + d1.y * d1.y);
        const V2 u2 = cam.dir_to_uv(normalize((prevWP - camDelta) - cam.pos));
        const V2 d2 = (u2 - prevUV) * V2((float)W, (float)H);
        par2 = sqrtf(d2.x * d2.x + d2.y * d2.y);
    }
    const float parMax = fmaxf(par1, par2);
    const float thr = lerpf(a.thrB, a.thrA, 0.0f);
    // loadSurfaceMotionBasedPrevData
    const V3 nIn = normalize(avgN);
    const float estDepth = length(prevWP - pc.pos);
    const V2 ppf(prevUV.x * (float)W, prevUV.y * (float)H);
    const int ox = (int)floorf(ppf.x - 0.5f), oy = (int)floorf(ppf.y - 0.5f);
    const float frustum = (a.frustumK * z) * (float)(W < H ? W : H);
    // TemporalAccumulation.h:82-83: the slope scale is a float (its double quotient rounded to float
    // equals the float quotient: double rounding is innocuous for a division)
    const float slope = 1.0f / lerpf(lerpf(0.05f, 1.0f, NoV), 1.0f, saturate(parMax / 30.0f));
    const float t0 = saturate(thr * slope) * frustum;
    V4 thr4(t0);
    {
        float r[4] = {ox >= 0 ? 1.f : 0.f, oy >= 0 ? 1.f : 0.f, ox + 1 >= 0 ? 1.f : 0.f, oy + 1 >= 0 ? 1.f : 0.f};
        const float cmp[4] = {ox < W ? 1.f : 0.f, oy < H ? 1.f : 0.f, ox + 1 < W ? 1.f : 0.f, oy + 1 < H ? 1.f : 0.f};
        for (int k = 0; k < 4; ++k) r[k] *= cmp[k];
        thr4 *= (V4(r[0], r[2], r[0], r[2]) * V4(r[1], r[1], r[3], r[3]));
    }
    thr4 -= 1e-6f;
    const float thrv[4] = {thr4.x, thr4.y, thr4.z, thr4.w};
    // the quality factor needs no history: computed before the history's round trips, so that
    // none of its inputs stays live across them
    float qf;
    {
        const V3 Vp = normalize(prevWP - pc.pos);
        const float NoVp = fabsf(dot(cN, Vp));
        float sq = (NoVp + 1e-3f) / (NoV + 1e-3f);
        sq *= sq;
        sq *= sq;
        qf = lerpf(0.1f, 1.0f, saturate(sq));
    }
    const TaHist hh = ta_history(pl, W, H, rot, nIn, prevUV, ox, oy, estDepth, thrv);
    const V4 prevI = hh.prevI;
    const V3 prevF = hh.prevF;
    const float found = hh.found;
    float quality = hh.quality, hist = hh.hist;
    hist = hist + 1.0f;
    quality *= qf;
    if (quality < 1.0f) {
        hist *= sqrtf(quality);
        hist = fmaxf(hist, 1.0f);
    }
    hist = fminf(hist, a.p.maxAcc);
    const float alpha = (found > 0) ? fmaxf(a.invAcc1, 1.0f / hist) : 1.0f;
    const float alphaR = (found > 0) ? fmaxf(a.invFast1, 1.0f / hist) : 1.0f;
    const V4 acc = lerp4(prevI, V4(illum, m2), alpha);
    const V3 accR = lerp3(prevF, illum, alphaR);
    a.ping[i] = tf(acc);
    a.pong[i] = make_float4(accR.x, accR.y, accR.z, 0.0f);
    a.histLen[i] = hist;
    return hist <= 4.0f;
}
// the whole temporal step of one pixel with plain loads (tests/native/denoise_driver.hip)
VX_HD bool temporal_px(const DenoiseArgs &a, const Qt &rot, int x, int y, const float4 *ffCol) {
    return temporal_px(a, TaPlanesH{&a}, rot, x, y, ta_pixel(a, x, y), ffCol);
}

// The pixels the history fix must filter (rare once history has built up)
// are listed per 16x16 tile: hfList[tile*256 + k] = pixel index, hfCount[tile]
// = k's; no atomics, and the history-fix launch only works on listed pixels.
// The tile's firefly list (k_firefly) is applied first: its entries go back to the radiance and
// reservoir planes, and the filtered values of the tile's own pixels are handed over in LDS.
// The pixel's own inputs are fetched first, before the tile's firefly-list hand-over (a clamped
// pixel for the grid's padding lanes, so every lane loads unconditionally): the list's round trip and
// the pixel's overlap, and the history taps follow in two more (ta_history).
// 4 waves/SIMD (128 VGPRs, 12 B/lane of spill): 94.3 -> 88.8 us against the compiler's 130 VGPRs at 3
#ifndef VX_WPE_TA
#define VX_WPE_TA 4  // occupancy bound of k_temporal (waves per SIMD; 1 = the compiler's choice)
#endif
template <bool ST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VX_WPE_TA))) void k_temporal(DenoiseArgs a, Qt rot) {
    __shared__ unsigned sTot[4], sFFn, sFFmask[8];
    __shared__ float4 sFF[256];
    int tx, ty;  // supertiles (default) or raster tiles (vxpt_tuning.ta_supertiles = 0)
    if (!map_tile<ST>(a, tx, ty)) return;
    const unsigned tile = ty * ((a.W + 15) / 16) + tx;
    const int W = a.W, H = a.H;
    const int x = tx * 16 + (threadIdx.x & 15), y = a.y0 + ty * 16 + (threadIdx.x >> 4);
    // the pixel's inputs (a clamped pixel for the padding lanes) and the tile's normals with a 1-pixel
    // apron (18x18, edge-clamped like ld4; one slot more for the staging lanes past it), fetched
    // before the firefly-list hand-over below
    constexpr int NT = 18 * 18;
    __shared__ float sN[3][NT + 1];
    const size_t i = (size_t)min(y, a.y1 - 1) * W + min(x, W - 1);
    TaPix px;
    px.z = a.depth[i];
    px.motion = xyz4(a.motion[i]);
    px.illum = xyz4(a.illum[i]);
    V3 nv[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int k = min((int)threadIdx.x + r * 256, NT - 1);
        nv[r] = xyz4(a.normalRough[(size_t)cl(a.y0 + ty * 16 - 1 + k / 18, H) * W + cl(tx * 16 - 1 + k % 18, W)]);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int k = min((int)threadIdx.x + r * 256, NT);
        sN[0][k] = nv[r].x; sN[1][k] = nv[r].y; sN[2][k] = nv[r].z;
    }
    if (threadIdx.x == 0) {
        const unsigned n = a.ffCount[tile];
        sFFn = n;
        if (n) a.ffCount[tile] = 0u;
        if (tile == 0) *a.ffCandCount = 0u;  // k_firefly_filter has finished
    }
    if (threadIdx.x < 8) sFFmask[threadIdx.x] = 0u;
    __syncthreads();
    const unsigned nff = sFFn;
    if (nff) {
        if (threadIdx.x < nff) {
            float4 col;
            ff_apply(a, tile, threadIdx.x, col);
            const unsigned p = a.ffIndex[tile * 256 + threadIdx.x];
            sFF[p] = col;
            atomicOr(&sFFmask[p >> 5], 1u << (p & 31));
        }
        __syncthreads();
    }
    const bool own = nff && ((sFFmask[threadIdx.x >> 5] >> (threadIdx.x & 31)) & 1u);
    {  // the centre normal and the 3x3 sum in ta_pixel's order
        const auto nrm = [&](int dx, int dy) {
            const int k = ((int)(threadIdx.x >> 4) + 1 + dy) * 18 + (int)(threadIdx.x & 15) + 1 + dx;
            return V3(sN[0][k], sN[1][k], sN[2][k]);
        };
        px.cN = nrm(0, 0);
        V3 avgN = px.cN;
        for (int ax = -1; ax <= 1; ++ax)
            for (int by = -1; by <= 1; ++by) {
                if (ax == 0 && by == 0) continue;
                avgN += nrm(ax, by);
            }
        px.avgN = avgN;
    }
    const bool fix = x < a.W && y < a.y1 &&
                     temporal_px(a, TaPlanesD(a), rot, x, y, px, own ? &sFF[threadIdx.x] : nullptr);
    const unsigned long long m = __ballot(fix);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) sTot[wv] = (unsigned)__popcll(m);
    __syncthreads();
    unsigned off = 0;
    for (int k = 0; k < wv; ++k) off += sTot[k];
    if (fix) a.hfList[tile * 256 + off + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)((size_t)y * a.W + x);
    if (threadIdx.x == 0) a.hfCount[tile] = sTot[0] + sTot[1] + sTot[2] + sTot[3];
}

// ---------------------------------------------------------------- HF
VX_D void history_fix_px(const DenoiseArgs &a, int W, int H, int x, int y, size_t i) {
    const float z = a.depth[i], hist = a.histLen[i];
    const float cMat = ld_ushort(a.material, W, H, x, y);
    const V3 cN = f4(a.normalRough[i]).xyz();
    const V3 cWP = wp(a, x, y);
    const float dthr = 0.003f * z;
    V4 sum = f4(a.ping[i]);
    float wsum = 1.0f;
    const float r = exp2f(4.0f - hist) + 1.0f;
    for (int j = -2; j <= 2; ++j)
        for (int k = -2; k <= 2; ++k) {
            const int sx = x + (int)(k * r), sy = y + (int)(j * r);
            const bool inside = sx >= 0 && sy >= 0 && sx < W && sy < H;
            if (k == 0 && j == 0) continue;
            const float sMat = ld_ushort(a.material, W, H, sx, sy);
            const V3 sN = ld4(a.normalRough, W, H, sx, sy).xyz();
            const float sz = ld1(a.depth, W, H, sx, sy);
            const V3 sWP = wp(a, sx, sy);  // out-of-frame taps get weight 0 below
            float w = plane_w(cWP, cN, sWP, dthr);
            w *= powf(fmaxf(0.01f, dot(cN, sN)), 8.0f);
            w = inside ? w : 0;
            w *= (float)(sMat == cMat);
            if (w > 1e-4f) {
                sum += ld4(a.ping, W, H, sx, sy) * w;
                wsum += w;
            }
        }
    a.pong[i] = tf(sum / wsum);
}

// One pixel per 32-lane half-wave: lane t < 25 of the half takes tap t of the 5x5 pattern (t = 12
// is the centre, weight 1), so all 24 sparse taps are fetched at once instead of one dependent
// round trip after another.  The taps' products are then added in the reference's order (centre
// first, then j-major, k-minor: HistoryFix.h's loop) by every lane of the half from shuffles, so
// the sums round exactly as history_fix_px's -- a tree reduction rounds differently.
VX_D void history_fix_wave(const DenoiseArgs &a, int W, int H, int x, int y, size_t i, int lane, bool store) {
    const float z = a.depth[i], hist = a.histLen[i];
    const float cMat = ld_ushort(a.material, W, H, x, y);
    const V3 cN = f4(a.normalRough[i]).xyz();
    const V3 cWP = wp(a, x, y);
    const float dthr = 0.003f * z;
    const float r = exp2f(4.0f - hist) + 1.0f;
    V4 c;            // this lane's tap: ping x weight (the centre: ping, weight 1)
    float cw = 0.0f;  // its weight, 0 when the tap is not taken (w <= 1e-4)
    if (lane < 25) {
        const int j = lane / 5 - 2, k = lane % 5 - 2;
        if (j == 0 && k == 0) {
            c = f4(a.ping[i]);
            cw = 1.0f;
        } else {
            const int sx = x + (int)(k * r), sy = y + (int)(j * r);
            const bool inside = sx >= 0 && sy >= 0 && sx < W && sy < H;
            const float sMat = ld_ushort(a.material, W, H, sx, sy);
            const V3 sN = ld4(a.normalRough, W, H, sx, sy).xyz();
            const V3 sWP = wp(a, sx, sy);
            // the tap's value is fetched beside its weight's inputs (edge-clamped, so always a valid
            // read): one dependent round trip fewer; used only when the weight passes
            const V4 sv = ld4(a.ping, W, H, sx, sy);
            float w = plane_w(cWP, cN, sWP, dthr);
            w *= powf(fmaxf(0.01f, dot(cN, sN)), 8.0f);
            w = inside ? w : 0;
            w *= (float)(sMat == cMat);
            if (w > 1e-4f) {
                c = sv * w;
                cw = w;
            }
        }
    }
    // the taps' values reach every lane of the half through v_readlane (constant lane indices, both
    // halves read, each keeps its own): no LDS-crossbar round trip per tap
    const bool hi = (threadIdx.x & 32u) != 0;
    auto rl = [&](float v, int l) {
        const float lo = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
        const float up = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l + 32));
        return hi ? up : lo;
    };
    V4 sum(rl(c.x, 12), rl(c.y, 12), rl(c.z, 12), rl(c.w, 12));
    float wsum = 1.0f;
#pragma unroll
    for (int t = 0; t < 25; ++t) {
        if (t == 12) continue;
        const float tw = rl(cw, t);
        const V4 tc(rl(c.x, t), rl(c.y, t), rl(c.z, t), rl(c.w, t));
        if (tw > 0.0f) {
            sum += tc;
            wsum += tw;
        }
    }
    if (lane == 0 && store) a.pong[i] = tf(sum / wsum);
}

// One workgroup per 16x16 tile, over the tile's list from k_temporal: a
// sparse list (<= 64 pixels, the steady state) is walked one pixel per wave at
// a time, a dense one (history just reset) gets one lane per pixel.
// blockIdx.z splits a sparse list over gridDim.z workgroups (rounds of 8 pixels dealt round-robin): a
// round is the listed pixel's chain of dependent loads, so a tile's rounds run side by side.
__global__ __launch_bounds__(256) void k_history_fix(DenoiseArgs a) {
    const unsigned tile = blockIdx.y * ((a.W + 15) / 16) + blockIdx.x;
    const unsigned n = a.hfCount[tile];
    const unsigned wv = threadIdx.x >> 6;
    if (n <= 64) {  // sparse (steady state): each half-wave takes every 8th listed pixel, its taps in parallel
        const unsigned half = wv * 2 + ((threadIdx.x >> 5) & 1);
        // wave-uniform trip count; the halves share the readlanes
        for (unsigned k0 = blockIdx.z * 8 + wv * 2; k0 < n; k0 += 8 * gridDim.z) {
            const unsigned k = k0 + (half & 1);
            const bool has = k < n;
            const size_t i = a.hfList[tile * 256 + (has ? k : k0)];
            history_fix_wave(a, a.W, a.H, (int)(i % (size_t)a.W), (int)(i / (size_t)a.W), i, threadIdx.x & 31, has);
        }
        return;
    }
    if (blockIdx.z != 0 || threadIdx.x >= n) return;
    const size_t i = a.hfList[tile * 256 + threadIdx.x];
    history_fix_px(a, a.W, a.H, (int)(i % (size_t)a.W), (int)(i / (size_t)a.W), i);
}

// HistoryClamping's per-pixel step after the 5x5 moments (m1, m2: the fast history's YCoCg; nm1,
// nm2: the radiance), shared by k_history_clamp (moments from its LDS tile) and the host tests
// center: the fast history's YCoCg at the pixel; pi: its temporal history (ping); noisyC: its radiance
VX_HD void history_clamp_px(const DenoiseArgs &a, size_t i, float hist, V3 m1, V3 m2, V3 nm1, float nm2, V3 center,
                            V4 pi, V3 noisyC) {
    m1 /= 25.0f; m2 /= 25.0f; nm1 /= 25.0f; nm2 /= 25.0f;
    const V3 sigma(sqrtf(fmaxf(0.0f, m2.x - m1.x * m1.x)), sqrtf(fmaxf(0.0f, m2.y - m1.y * m1.y)),
                   sqrtf(fmaxf(0.0f, m2.z - m1.z * m1.z)));
    V3 cmin = m1 - 2.0f * sigma, cmax = m1 + 2.0f * sigma;
    // LinearMath.h template min / max on Float3 (x-compare), as component selects (a select of whole
    // vectors went through scratch memory)
    const bool useMin = cmin.x < center.x, useMax = cmax.x > center.x;
    if (a.clampDbg) a.clampDbg[i] = (float)((useMin ? 1 : 0) | (useMax ? 2 : 0) | (hist > 4.0f ? 4 : 0));
    cmin = V3(useMin ? cmin.x : center.x, useMin ? cmin.y : center.y, useMin ? cmin.z : center.z);
    cmax = V3(useMax ? cmax.x : center.x, useMax ? cmax.y : center.y, useMax ? cmax.z : center.z);
    const V3 dY = rgb_to_ycocg(pi.xyz());
    const V3 cY(clampf(dY.x, cmin.x, cmax.x), clampf(dY.y, cmin.y, cmax.y), clampf(dY.z, cmin.z, cmax.z));
    V4 outD(ycocg_to_rgb(cY), pi.w);
    const V3 respC = ycocg_to_rgb(center);
    V4 outR(respC, 0.0f);
    if (hist <= 4.0f) outD.set_xyz(outR.xyz());
    float factor = (cY.x - dY.x) == 0.0f ? 0.0f : saturate((cY.x - dY.x) / (center.x - dY.x));
    // parity hook: bit 8 -- the factor's quotient is ill-conditioned (its denominator within 1e-3 of
    // the fast history's luma, the quotient inside (0, 1)): rounding-level input differences move it
    if (a.clampDbg && hist > 4.0f && factor > 0.0f && factor < 1.0f &&
        fabsf(center.x - dY.x) <= 1e-3f * fmaxf(fabsf(center.x), fabsf(dY.x)))
        a.clampDbg[i] += 8.0f;
    if (hist <= 4.0f) factor = 1.0f;
    float hdl = 10.0f * 0.3f * luminance(abs3(respC - pi.xyz()));
    hdl *= factor;
    if (hist <= 4.0f) hdl = 0.0f;
    const V3 dist = nm1 - respC;
    const float distL = luminance(abs3(dist));
    V3 acc = (distL == 0.0f) ? V3(0.0f) : dist * hdl / distL;
    const float accL = luminance(abs3(acc));
    const float ratio = (accL == 0.0f) ? 0.0f : distL / accL;
    if (ratio < 1.0f) acc *= ratio;
    if (ratio <= 0.0f) acc = V3(0.0f);
    outD.set_xyz(outD.xyz() + acc);
    outR.set_xyz(outR.xyz() + acc);
    const float dL = luminance(pi.xyz()), nL = luminance(nm1);
    const float tSig = 0.5f * sqrtf(fmaxf(0.0f, nm2 - nL * nL));
    const float sSig = 4.5f * sigma.x;
    float reset = 0.5f * fmaxf(0.0f, fabsf(dL - nL) - sSig - tSig) / (1.0e-6f + fmaxf(dL, nL) + sSig + tSig);
    reset = saturate(reset);
    outD.set_xyz(lerp3(outD.xyz(), noisyC, reset));
    outR.set_xyz(lerp3(outR.xyz(), noisyC, reset));
    const float oL = luminance(outD.xyz());
    outD.w += (oL * oL - dL * dL);
    outD.w = fmaxf(0.0f, outD.w);
    a.prevIllum[i] = tf(outD);
    a.prevFast[i] = tf(outR);
    a.prevHistLen[i] = hist;
}

// ---------------------------------------------------------------- HC
// The 5x5 neighbourhood of the 16x16 tile (20x20 with edge clamp) is staged
// once in LDS: YCoCg of the fast history and the noisy radiance.
// Supertiles (st_tile) keep the neighbouring tiles' shared apron in one XCD's L2 (274 -> 200 MB per
// frame, time 49.7 -> 49.3 us against raster tiles; XCD strips were slower, 51 -> 57 us).
template <int TS, bool ST>
__global__ __launch_bounds__(TS * TS) void k_history_clamp(DenoiseArgs a) {
    constexpr int T = TS + 4, N = T * T, NT = TS * TS, R = (N + NT - 1) / NT;
    const int W = a.W, H = a.H;
    const int tx = threadIdx.x % TS, ty = threadIdx.x / TS;
    int btx, bty;
    if (!map_tile<ST, TS>(a, btx, bty)) return;
    const int x0 = btx * TS, y0 = a.y0 + bty * TS;
    const int x = x0 + tx, y = y0 + ty;
    // one slot more than the tile: the staging rounds' lanes past the tile all store into it, so
    // that every staging store is unconditional (a store behind a condition takes its fetch into the
    // branch, behind the other rounds' stores)
    __shared__ float sY[3][N + 1], sR[3][N + 1];
    // one memory round trip: the pixel's own inputs (a clamped pixel for the padding lanes) and every
    // staged tap are fetched before the first is used (the tile's fast history and radiance at the
    // centre come from the staged tile: the same values)
    const size_t i = (size_t)min(y, a.y1 - 1) * W + min(x, W - 1);
    const float z = a.depth[i], hist = a.histLen[i];
    const V4 pi = f4(a.ping[i]);
    float4 pg[R], il[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int k = min((int)threadIdx.x + r * NT, N - 1);
        const size_t j = (size_t)cl(y0 + k / T - 2, H) * W + cl(x0 + k % T - 2, W);
        pg[r] = a.pong[j];
        il[r] = a.illum[j];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int k = min((int)threadIdx.x + r * NT, N);
        const V3 yc = rgb_to_ycocg(xyz4(pg[r]));
        sY[0][k] = yc.x; sY[1][k] = yc.y; sY[2][k] = yc.z;
        sR[0][k] = il[r].x; sR[1][k] = il[r].y; sR[2][k] = il[r].z;
    }
    __syncthreads();
    if (x >= W || y >= a.y1) return;
    if (z > kRange) {
        if (a.clampDbg) a.clampDbg[i] = 0.0f;
        return;
    }
    V3 m1(0.0f), m2(0.0f), nm1(0.0f);
    float nm2 = 0.0f;
    // one column of taps per iteration: fully unrolled, the 25 taps' LDS values were all held in
    // registers (118 VGPRs, 4 waves/SIMD); a column at a time runs at 65 (7 waves), 61 -> 50 us.
    // Precomputing the per-pixel moment terms in the staging loop (3 float4 planes in LDS) was
    // slower (59 us at 44 or 87 VGPRs).
#pragma unroll 1
    for (int dx = -2; dx <= 2; ++dx)
#pragma unroll
        for (int dy = -2; dy <= 2; ++dy) {
            const int k = (ty + 2 + dy) * T + (tx + 2 + dx);
            const V3 s(sY[0][k], sY[1][k], sY[2][k]);
            m1 += s;
            m2 += s * s;
            const V3 nz(sR[0][k], sR[1][k], sR[2][k]);
            const float nl = luminance_fast(nz);
            nm1 += nz;
            nm2 += nl * nl;
        }
    const int kc = (ty + 2) * T + tx + 2;
    history_clamp_px(a, i, hist, m1, m2, nm1, nm2, V3(sY[0][kc], sY[1][kc], sY[2][kc]), pi,
                     V3(sR[0][kc], sR[1][kc], sR[2][kc]));
}

// host restatement of the kernel's moments (the same taps in the same order, read from the planes
// instead of the LDS tile) for the CPU tests (tests/native/denoise_driver.hip)
VX_HD void history_clamp_host(const DenoiseArgs &a, int x, int y) {
    const int W = a.W, H = a.H;
    const size_t i = (size_t)y * W + x;
    if (a.depth[i] > kRange) {
        if (a.clampDbg) a.clampDbg[i] = 0.0f;
        return;
    }
    const float hist = a.histLen[i];
    V3 m1(0.0f), m2(0.0f), nm1(0.0f);
    float nm2 = 0.0f;
    for (int dx = -2; dx <= 2; ++dx)
        for (int dy = -2; dy <= 2; ++dy) {
            const V3 sv = rgb_to_ycocg(ld4(a.pong, W, H, x + dx, y + dy).xyz());
            m1 += sv;
            m2 += sv * sv;
            const V3 nz = ld4(a.illum, W, H, x + dx, y + dy).xyz();
            const float nl = luminance_fast(nz);
            nm1 += nz;
            nm2 += nl * nl;
        }
    history_clamp_px(a, i, hist, m1, m2, nm1, nm2, rgb_to_ycocg(f4(a.pong[i]).xyz()), f4(a.ping[i]), f4(a.illum[i]).xyz());
}

// ---------------------------------------------------------------- A-trous (LDS variant)
// The 16x16 tile's 5x5 neighbourhood (20x20, edge-clamped) of the history,
// normals, material ids and world positions is staged in LDS (AtrousSmem.h
// stages the same tile in shared memory).
// Supertiles (st_tile): 50.4 -> 46.9 us against raster tiles (XCD strips were 51 -> 57); staging
// the depth and recomputing world positions instead of the 16-byte plane was slower (57.8 us).
template <int TS, bool ST>
__global__ __launch_bounds__(TS * TS) void k_atrous_smem(DenoiseArgs a) {
    constexpr int T = TS + 4, N = T * T;
    const int W = a.W, H = a.H;
    const int tx = threadIdx.x % TS, ty = threadIdx.x / TS;
    int btx, bty;
    if (!map_tile<ST, TS>(a, btx, bty)) return;
    const int x0 = btx * TS, y0 = a.y0 + bty * TS;
    const int x = x0 + tx, y = y0 + ty;
    constexpr int NT = TS * TS, R = (N + NT - 1) / NT, NP = N + 1;
    // one slot more than the tile: every staging store is unconditional (k_history_clamp)
    __shared__ float4 sI[NP];
    __shared__ float sNx[NP], sNy[NP], sNz[NP], sM[NP], sPx[NP], sPy[NP], sPz[NP];
    // one memory round trip: the pixel's depth and history length (a clamped pixel for the padding
    // lanes) and every staged tap, fetched before the first is used
    const size_t i = (size_t)min(y, a.y1 - 1) * W + min(x, W - 1);
    const float z = a.depth[i], hist = a.histLen[i];
    float4 vI[R];
    V3 vN[R], vP[R];
    float vM[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int k = min((int)threadIdx.x + r * NT, N - 1);
        const size_t j = (size_t)cl(y0 + k / T - 2, H) * W + cl(x0 + k % T - 2, W);
        vI[r] = a.prevIllum[j];
        vN[r] = xyz4(a.normalRough[j]);
        vM[r] = a.material[j];
        vP[r] = xyz4(a.wpos[j]);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int k = min((int)threadIdx.x + r * NT, N);
        sI[k] = vI[r];
        sNx[k] = vN[r].x; sNy[k] = vN[r].y; sNz[k] = vN[r].z;
        sM[k] = vM[r];
        sPx[k] = vP[r].x; sPy[k] = vP[r].y; sPz[k] = vP[r].z;
    }
    __syncthreads();
    if (x >= W || y >= a.y1) return;
    if (z > 500000.0f) return;
    // the centre's normal, position and material come from the staged tile
    const int kc = (ty + 2) * T + tx + 2;
    const V3 cN(sNx[kc], sNy[kc], sNz[kc]);
    const V3 cWP(sPx[kc], sPy[kc], sPz[kc]);
    const float cMat = sM[kc];
    const float k3[2] = {0.44198f, 0.27901f};
    if (hist >= 3.0f) {
        V4 vs;
        const float kern[4] = {1.0f / 4.0f, 1.0f / 8.0f, 1.0f / 8.0f, 1.0f / 16.0f};
        for (int dx = -1; dx <= 1; ++dx)
            for (int dy = -1; dy <= 1; ++dy)
                vs += f4(sI[(ty + 2 + dy) * T + tx + 2 + dx]) * kern[abs(dx) * 2 + abs(dy)];
        const float vm1 = luminance(vs.xyz());
        const float var = fmaxf(0.0f, vs.w - vm1 * vm1);
        const float cLum = luminance_fast(f4(sI[kc]).xyz());
        const float phiInv = 1.0f / fmaxf(1.0e-4f, a.p.phiL * sqrtf(var));
        const float nwp = normal_weight_param(1.0f, a.p.lobeAngleFraction);
        float sumW = 0.0f;
        V4 sum;
        const float dthr = a.p.depthThreshold * z;
        // a column of taps per iteration (126 -> 64 VGPRs: 4 -> 8 waves/SIMD)
#pragma unroll 1
        for (int cx = -1; cx <= 1; ++cx)
            for (int cy = -1; cy <= 1; ++cy) {
                const int px = x + cx, py = y + cy;
                const bool isC = cx == 0 && cy == 0;
                const bool inside = px >= 0 && py >= 0 && px < W && py < H;
                const float kernel = inside ? k3[abs(cx)] * k3[abs(cy)] : 0.0f;
                const int k = (ty + 2 + cy) * T + tx + 2 + cx;  // = edge-clamped (px, py)
                const V3 sN(sNx[k], sNy[k], sNz[k]);
                const V3 sWP(sPx[k], sPy[k], sPz[k]);
                const float sMat = sM[k];
                float geo = plane_w_fast(cWP, cN, sWP, dthr) * kernel;
                const float nw = nonexp_w(acos_approx_fast(dot_fast(cN, sN)), nwp);
                const V4 si = f4(sI[k]);
                const float lw = fabsf(cLum - luminance_fast(si.xyz())) * phiInv;
                float w = geo * nw * __expf(-lw);
                w = isC ? kernel : w;
                w *= (float)(sMat == cMat);
                sumW += w;
                sum += w * si;
            }
        sumW = fmaxf(sumW, 1e-6f);
        sum /= sumW;
        const float o1 = luminance(sum.xyz());
        a.ping[i] = make_float4(sum.x, sum.y, sum.z, fmaxf(0.0f, sum.w - o1 * o1));
    } else {
        float sw = 0.0f, s1 = 0.0f, s2 = 0.0f;
        V3 si(0.0f);
        const float nwp = normal_weight_param(1.0f, a.p.lobeAngleFraction);
#pragma unroll 1
        for (int cx = -2; cx <= 2; ++cx)
            for (int cy = -2; cy <= 2; ++cy) {
                const int k = (ty + 2 + cy) * T + tx + 2 + cx;
                const V3 sN(sNx[k], sNy[k], sNz[k]);
                const float nw = nonexp_w(acos_approx_fast(dot_fast(cN, sN)), nwp);
                const V4 smp = f4(sI[k]);
                const V3 sill = smp.xyz();
                float w = nw * 1.0f;
                w *= (float)(sM[k] == cMat);
                sw += w;
                si += sill * w;
                s1 += luminance_fast(sill) * w;
                s2 += smp.w * w;
            }
        const float boost = fmaxf(1.0f, 4.0f / (hist + 1.0f));
        sw = fmaxf(sw, 1e-6f);
        si /= sw;
        s1 /= sw;
        s2 /= sw;
        const float var = fmaxf(0.0f, s2 - s1 * s1) * boost;
        a.ping[i] = make_float4(si.x, si.y, si.z, var);
    }
}

// ---------------------------------------------------------------- A-trous
// One pixel of an a-trous pass (Atrous.h); taps come from Src: global planes through buffer
// descriptors (any step, jitter) or an LDS tile with a step-wide apron (steps 2 and 4).  The
// arithmetic is the same code for both.
#ifndef VX_A8_BATCH
#define VX_A8_BATCH 8
#endif
// fetch(k0) fills tP/tN/tV[k0 .. k0 + kBatch - 1] of the 8-tap arrays at every k0 % kBatch == 0
static_assert(VX_A8_BATCH == 0 || (VX_A8_BATCH > 0 && 8 % VX_A8_BATCH == 0), "VX_A8_BATCH must divide 8");
struct GlobalTaps {
    static constexpr int kBatch = VX_A8_BATCH;  // taps fetched together (8: one round trip for all)
    Plane4 pW, pN, pI;
    VX_D V4 wpos(int px, int py, int W) const { return pW[py * W + px]; }
    VX_D V3 nrm(int px, int py, int W) const { return pN[py * W + px].xyz(); }
    VX_D V4 val(int px, int py, int W) const { return pI[py * W + px]; }
};
template <int R, int TS = 16>
struct TileTaps {  // the TSxTS tile at (x0, y0) with an R-pixel apron, zeros outside the frame
    static constexpr int T = TS + 2 * R;
    static constexpr int kBatch = 0;  // LDS taps: read where used
    const float4 *sP, *sI;
    const float *sNx, *sNy, *sNz;
    int x0, y0;
    VX_D int k(int px, int py) const { return (py - y0 + R) * T + (px - x0 + R); }
    VX_D V4 wpos(int px, int py, int) const { return f4(sP[k(px, py)]); }
    VX_D V3 nrm(int px, int py, int) const {
        const int j = k(px, py);
        return V3(sNx[j], sNy[j], sNz[j]);
    }
    VX_D V4 val(int px, int py, int) const { return f4(sI[k(px, py)]); }
};

// z, hist: the pixel's depth and history length, fetched by the caller in its first round trip
template <class Src>
VX_D void atrous_px(const DenoiseArgs &a, const Src &src, float4 *out, unsigned step, unsigned frameIndex, int final,
                    int x, int y, float z, float hist) {
    const int W = a.W, H = a.H;
    const size_t i = (size_t)y * W + x;
    if (z > 500000.0f) {
        if (final) a.output[i] = a.illum[i];  // BufferCopySky
        return;
    }
    // the output's albedo is fetched beside the taps, not behind the result
    const float4 al = final ? a.albedo[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    int ofx = 0, ofy = 0;
    if (step > 4) {
        const uint32_t lin = explode((uint32_t)x) | (explode((uint32_t)y) << 1);
        const uint32_t seed = seq_hash(frameIndex + 0x035F9F29u);
        uint32_t st = seed ^ (seq_hash(lin) + 0x9E3779B9u + (seed << 6) + (seed >> 2));
        st = seq_hash(st);
        const uint32_t u0 = st;
        st = seq_hash(st);
        const uint32_t u1 = st;
        const V2 r(u0 / 4294967295.0f, u1 / 4294967295.0f);
        const V2 o = V2((float)step) * 0.5f * (r - 0.5f);
        ofx = (int)o.x;
        ofy = (int)o.y;
    }
    // every tap's position, normal and value is fetched before the first weight: one memory round
    // trip for the whole stencil (a value read behind its tap's weight test was a second one; the
    // packed tap holds world position + 16-bit material, -1 = sky: weight 0 like the reference's
    // depth test; out-of-frame taps read 0 and get weight 0 below)
    V4 tP[8], tV[8];
    V3 tN[8];
    const auto fetch = [&](int k0) {  // taps k0 .. k0 + kBatch - 1
#pragma unroll
        for (int k = k0; k < k0 + Src::kBatch; ++k) {
            const int t = k < 4 ? k : k + 1, xx = t % 3 - 1, yy = t / 3 - 1;
            const int px = x + ofx + xx * (int)step, py = y + ofy + yy * (int)step;
            tP[k] = src.wpos(px, py, W);
            tN[k] = src.nrm(px, py, W);
            tV[k] = src.val(px, py, W);
        }
    };
    if (Src::kBatch) fetch(0);
    const V4 cP = src.wpos(x, y, W);
    const float cMat = cP.w;
    const V3 cN = src.nrm(x, y, W);
    const V3 cWP = cP.xyz();
    float lobe = a.p.lobeAngleFraction / sqrtf((float)step);
    lobe = lerpf(0.99f, lobe, saturate(hist / 5.0f));
    const V4 c = src.val(x, y, W);
    const float cLum = luminance_fast(c.xyz());
    const float phiInv = 1.0f / fmaxf(1.0e-4f, a.p.phiL * sqrtf(c.w));
    const float nwp = normal_weight_param(1.0f, lobe);
    float sumW = 0.44198f * 0.44198f;
    V4 sum = c * V4(V3(sumW), sumW * sumW);
    const float dthr = a.p.depthThreshold * z;
    const float k3[2] = {0.44198f, 0.27901f};
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // row-major over the 3x3 taps without the centre (Atrous.h order)
        const int t = k < 4 ? k : k + 1, xx = t % 3 - 1, yy = t / 3 - 1;
        const int px = x + ofx + xx * (int)step, py = y + ofy + yy * (int)step;
        const bool inside = px >= 0 && py >= 0 && px < W && py < H;
        const float kernel = k3[abs(xx)] * k3[abs(yy)];
        if (Src::kBatch && k > 0 && k % Src::kBatch == 0) fetch(k);
        if (!Src::kBatch) {
            tP[k] = src.wpos(px, py, W);
            tN[k] = src.nrm(px, py, W);
        }
        const float sMat = tP[k].w;
        float geo = plane_w_fast(cWP, cN, tP[k].xyz(), dthr);
        geo *= kernel;
        geo *= float(inside);
        const float nw = nonexp_w(acos_approx_fast(dot_fast(cN, tN[k])), nwp);
        float w = geo * nw;
        w *= (float)(sMat == cMat);
        if (w > 1e-4f) {
            const V4 sv = Src::kBatch ? tV[k] : src.val(px, py, W);
            float lw = fabsf(cLum - luminance_fast(sv.xyz())) * phiInv;
            lw = fminf(INFINITY, lw);
            w *= __expf(-lw);
            sumW += w;
            sum += V4(V3(w), w * w) * sv;
        }
    }
    const V4 res = sum / V4(V3(sumW), sumW * sumW);
    out[i] = tf(res);
    if (final) a.output[i] = make_float4(res.x * al.x, res.y * al.y, res.z * al.z, 0.0f);
}

#ifndef VX_WPE_A8
#define VX_WPE_A8 1  // occupancy bound of k_atrous (waves per SIMD; 1 = the compiler's choice)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VX_WPE_A8))) void k_atrous(
    DenoiseArgs a, const float4 *in, float4 *out, unsigned step, unsigned frameIndex, int final) {
    int tx, ty;
    if (!xcd_tile(a, tx, ty)) return;
    const int x = tx * 16 + (threadIdx.x & 15), y = a.y0 + ty * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.y1) return;
    const GlobalTaps src{Plane4(a.wpos, a.W * a.H), Plane4(a.normalRough, a.W * a.H), Plane4(in, a.W * a.H)};
    const size_t i = (size_t)y * a.W + x;
    atrous_px(a, src, out, step, frameIndex, final, x, y, a.depth[i], a.histLen[i]);
}

// the tile and its apron staged once in LDS (steps 2 and 4, R = step: 49 -> 36 and 46 -> 36 us)
template <int R, int TS>
__global__ __launch_bounds__(TS * TS) void k_atrous_tile(DenoiseArgs a, const float4 *in, float4 *out,
                                                         unsigned step, unsigned frameIndex, int final) {
    constexpr int T = TileTaps<R, TS>::T, N = T * T, NT = TS * TS, NR = (N + NT - 1) / NT, NP = N + 1;
    // one slot more than the tile: every staging store is unconditional (k_history_clamp)
    __shared__ float4 sP[NP], sI[NP];
    __shared__ float sNx[NP], sNy[NP], sNz[NP];
    int tx, ty;
    if (!xcd_tile<TS>(a, tx, ty)) return;
    const int W = a.W, H = a.H;
    const int x0 = tx * TS, y0 = a.y0 + ty * TS;
    const int x = x0 + (int)(threadIdx.x % TS), y = y0 + (int)(threadIdx.x / TS);
    // one memory round trip: the pixel's depth and history length (a clamped pixel for the padding
    // lanes) and every staged tap (from a clamped position; zero outside the frame), fetched before
    // the first is used
    const size_t i = (size_t)min(y, a.y1 - 1) * W + min(x, W - 1);
    const float z = a.depth[i], hist = a.histLen[i];
    float4 vP[NR], vN[NR], vI[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int k = min((int)threadIdx.x + r * NT, N - 1);
        const size_t j = (size_t)cl(y0 - R + k / T, H) * W + cl(x0 - R + k % T, W);
        vP[r] = a.wpos[j];
        vN[r] = a.normalRough[j];
        vI[r] = in[j];
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int k = min((int)threadIdx.x + r * NT, N);
        const int gx = x0 - R + k % T, gy = y0 - R + k / T;
        const float m = (gx >= 0 && gy >= 0 && gx < W && gy < H) ? 1.0f : 0.0f;
        // zero outside the frame, component by component (a select of whole float4s went through
        // scratch memory); x * 1 and x * 0 are exact for the finite planes
        const auto z4 = [&](float4 v) { return make_float4(m != 0.0f ? v.x : 0.0f, m != 0.0f ? v.y : 0.0f,
                                                            m != 0.0f ? v.z : 0.0f, m != 0.0f ? v.w : 0.0f); };
        sP[k] = z4(vP[r]);
        sI[k] = z4(vI[r]);
        sNx[k] = m != 0.0f ? vN[r].x : 0.0f; sNy[k] = m != 0.0f ? vN[r].y : 0.0f; sNz[k] = m != 0.0f ? vN[r].z : 0.0f;
    }
    __syncthreads();
    if (x >= W || y >= a.y1) return;
    const TileTaps<R, TS> src{sP, sI, sNx, sNy, sNz, x0, y0};
    atrous_px(a, src, out, step, frameIndex, final, x, y, z, hist);
}

__global__ __launch_bounds__(256) void k_copy_output(DenoiseArgs a, const float4 *in) {
    const size_t i = (size_t)a.y0 * a.W + (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)a.y1 * a.W) return;
    if (a.depth[i] > kRange) {
        a.output[i] = a.illum[i];
    } else {
        const float4 v = in[i], al = a.albedo[i];
        a.output[i] = make_float4(v.x * al.x, v.y * al.y, v.z * al.z, 0.0f);
    }
}

// 16x16 tiles over the band rows [y0, y1)
inline dim3 grid16(const DenoiseArgs &a) { return dim3((a.W + 15) / 16, (a.y1 - a.y0 + 15) / 16); }
// xcd_tile<TS>'s grid: 8 strips x the widest strip's tiles
template <int TS = 16>
inline dim3 grid_xcd(const DenoiseArgs &a) {
    const dim3 g((a.W + TS - 1) / TS, (a.y1 - a.y0 + TS - 1) / TS);
    const unsigned per = (g.x + 7) / 8 * g.y;
    return dim3(g.x, (8 * per + g.x - 1) / g.x);
}
inline dim3 grid1d(const DenoiseArgs &a) { return dim3((unsigned)(((size_t)(a.y1 - a.y0) * a.W + 255) / 256)); }

}  // namespace

// world positions over rows [wy0, wy1); with `detect` also the firefly filter over the band (its
// reservoir parity is baked into a.reservoir by the host); with `apply` the filtered pixels are
// written back here rather than by the next k_temporal
hipError_t launch_firefly(const DenoiseArgs &a, int wy0, int wy1, bool detect, bool apply, hipStream_t st) {
    // the detecting wave filters its own fireflies (84 VGPRs, 5 waves/SIMD, for the ~100 pixels of a
    // frame) instead of a second launch: chain 0.3745 -> 0.3709 ms; tuning firefly_fused = 0 keeps
    // k_firefly_filter
    const bool fused = a.tune.ffFused != 0;
    const dim3 g((a.W + 63) / 64, (wy1 - wy0 + 3) / 4);
    if (fused) hipLaunchKernelGGL(k_firefly<true>, g, dim3(256), 0, st, a, wy0, wy1, detect ? 1 : 0);
    else hipLaunchKernelGGL(k_firefly<false>, g, dim3(256), 0, st, a, wy0, wy1, detect ? 1 : 0);
    if (detect && !fused) hipLaunchKernelGGL(k_firefly_filter, dim3(1024), dim3(64), 0, st, a);
    if (detect && apply) hipLaunchKernelGGL(k_firefly_apply, grid16(a), dim3(256), 0, st, a);
    return hipGetLastError();
}
// an empty one-wave kernel: a timing event recorded behind it is stamped once the stream has passed
// every wait before it (vxpt_render_frames' chain start after the cross-stream hand-off)
__global__ __launch_bounds__(64) void k_stream_mark() {}
hipError_t launch_stream_mark(hipStream_t st) {
    hipLaunchKernelGGL(k_stream_mark, dim3(1), dim3(64), 0, st);
    return hipGetLastError();
}
hipError_t launch_frame0_init(const DenoiseArgs &a, hipStream_t st) {
    hipLaunchKernelGGL(k_frame0, grid1d(a), dim3(256), 0, st, a);
    return hipGetLastError();
}
template <int TS = 16>
inline dim3 grid_st(const DenoiseArgs &a) {
    const int tilesX = (a.W + TS - 1) / TS, tilesY = (a.y1 - a.y0 + TS - 1) / TS;
    const int nS = ((tilesX + 3) / 4) * ((tilesY + 3) / 4);
    return dim3((unsigned)((nS + 7) / 8 * 8 * 16));
}
hipError_t launch_temporal(const DenoiseArgs &a, hipStream_t st) {
    const Qt rot = q_rotation_between(a.prevCam.dir, a.cam.dir);
    // supertiles: the taps' history rows stay in the XCD's L2 (351 -> 266 MB per frame, time even);
    // tuning ta_supertiles = 0: raster tiles
    if (a.tune.taSupertiles) hipLaunchKernelGGL((k_temporal<true>), grid_st(a), dim3(256), 0, st, a, rot);
    else hipLaunchKernelGGL((k_temporal<false>), grid16(a), dim3(256), 0, st, a, rot);
    return hipGetLastError();
}
hipError_t launch_history_fix(const DenoiseArgs &a, hipStream_t st) {
    // steady state on the C3 bench: ~3000 listed pixels in ~960 of 8160 tiles, at most ~21 per tile
    // (tools/hf_stats.py); tuning hf_split workgroups per tile
    dim3 g = grid16(a);
    g.z = (unsigned)a.tune.hfSplit;
    hipLaunchKernelGGL(k_history_fix, g, dim3(256), 0, st, a);
    return hipGetLastError();
}
// tile edge of the LDS-staged 5x5 stencils (history clamping, the first a-trous): 32 stages the
// 2-pixel apron at 1.27x the tile's pixels instead of 1.56x (both kernels run at the HBM's rate on
// their fetched bytes)
inline dim3 grid_ts(const DenoiseArgs &a, int ts) { return dim3((a.W + ts - 1) / ts, (a.y1 - a.y0 + ts - 1) / ts); }
hipError_t launch_history_clamp(const DenoiseArgs &a, hipStream_t st) {
    if (a.tune.stencilTile == 32) hipLaunchKernelGGL((k_history_clamp<32, false>), grid_ts(a, 32), dim3(1024), 0, st, a);
    else hipLaunchKernelGGL((k_history_clamp<16, true>), grid_st(a), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_atrous_smem(const DenoiseArgs &a, hipStream_t st) {
    if (a.tune.stencilTile == 32) hipLaunchKernelGGL((k_atrous_smem<32, false>), grid_ts(a, 32), dim3(1024), 0, st, a);
    else hipLaunchKernelGGL((k_atrous_smem<16, true>), grid_st(a), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_atrous(const DenoiseArgs &a, const float4 *in, float4 *out, unsigned step, unsigned frameIndex,
                         bool final, hipStream_t st) {
    // 32x32 tiles (1024 threads, apron load factor 1.27 / 1.56 / 2.64 instead of 1.56 / 2.25 / 5.1)
    // were measured slower for every step: 41 / 41 / 70 us against 36 / 36 / 64 -- the passes are
    // VALU bound on the weights, not on filling the tile
    const int f = final ? 1 : 0;
    if (step == 2)
        hipLaunchKernelGGL((k_atrous_tile<2, 16>), grid_xcd(a), dim3(256), 0, st, a, in, out, step, frameIndex, f);
    else if (step == 4)
        hipLaunchKernelGGL((k_atrous_tile<4, 16>), grid_xcd(a), dim3(256), 0, st, a, in, out, step, frameIndex, f);
    else  // step 8: a 34x34 staged apron for 16x16 pixels was measured slower (71 vs 65 us) than the taps
        hipLaunchKernelGGL(k_atrous, grid_xcd(a), dim3(256), 0, st, a, in, out, step, frameIndex, f);
    return hipGetLastError();
}
hipError_t launch_copy_output(const DenoiseArgs &a, const float4 *in, hipStream_t st) {
    hipLaunchKernelGGL(k_copy_output, grid1d(a), dim3(256), 0, st, a, in);
    return hipGetLastError();
}

}  // namespace vx
