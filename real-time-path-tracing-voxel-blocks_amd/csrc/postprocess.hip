// vxpt -- offline post-processing on gfx950 (PostProcessor::run, PostProcessor.cu:74-122):
// histogram auto-exposure, bloom, lens flare, vignette (PostProcessingPipeline.cu:11-601),
// filmic tone mapping (FilmicToneMapping.h:11-117), crosshair, copy to the frame buffer.
//
// The reference runs one kernel per effect in place on IlluminationOutputBuffer (8 full-frame
// passes, a float atomic per pixel for the histogram, a host round trip for the exposure).  Here
// the chain is three passes and the denoiser output stays intact (parity hook):
//   1. k_lum_bloom  -- 64x16 tile in LDS: the luminance histogram (LDS bins, one global atomic per
//                      non-empty bin and tile), the bloom extract and the horizontal blur -> bloomB
//   2. k_exposure   -- one wave: the reference's histogram scans and exposure adaptation on the
//                      device (state[0] = current average luminance, state[1] = exposure)
//   3. k_compose    -- vertical blur + composite, lens flare, vignette, tone curve, crosshair ->
//                      Float4(sRGB, 0)
// Each stage keeps the reference's per-pixel arithmetic and order; the exchanges through the
// working plane were exact float4 round trips, so fusing them changes no value.
#include "vx_internal.hpp"

namespace vx {
namespace {

constexpr int kBins = 256;
constexpr float kMinLogLum = -8.0f, kMaxLogLum = 4.0f;

VX_D V3 ld3(const float4 *b, int W, int x, int y) {
    const float4 v = b[(size_t)y * W + x];
    return V3(v.x, v.y, v.z);
}
VX_D void st3(float4 *b, int W, int x, int y, V3 c, float w) { b[(size_t)y * W + x] = make_float4(c.x, c.y, c.z, w); }
VX_D V3 clamp3(V3 v, float lo, float hi) { return V3(clampf(v.x, lo, hi), clampf(v.y, lo, hi), clampf(v.z, lo, hi)); }
VX_D float lum_ref(V3 c) { return dot(c, V3(0.2126f, 0.7152f, 0.0722f)); }  // compensated Float3 dot

// ComputeLuminanceHistogramKernel (PostProcessingPipeline.cu:319-350) bin of one pixel
VX_D int hist_bin(float l) {
    const float logLum = log10f(l);
    const float t = clampf((logLum - kMinLogLum) / (kMaxLogLum - kMinLogLum), 0.0f, 1.0f);
    return min((int)(t * kBins), kBins - 1);
}

// BloomExtractBrightPixelsKernel (:12-80), neighbour filter on: c = the pixel, l its luminance,
// n[4] the luminances of the (x-1, x+1, y-1, y+1) neighbours, -inf where outside the image
VX_D V3 bloom_extract(V3 c, float l, const float n[4], float thr) {
    if (!(l > thr)) return V3(0.0f);
    float maxN = 0.0f;
    for (int i = 0; i < 4; i++) maxN = fmaxf(maxN, n[i]);  // fmaxf(m, -inf) = m: a skipped neighbour
    if (maxN < thr * 0.4f) return V3(0.0f);
    return clamp3((c - V3(thr)) * 0.7f, 0.0f, 100.0f);
}

// BloomBlurKernel (:83-125) half width
__host__ __device__ inline int blur_half(const PostParamsDev &p) { return ((int)(p.bloomRadius * 2.0f) + 1) / 2; }

constexpr int TX = 64, TY = 16, kHalo = 8;
constexpr int LW = TX + 2 * kHalo + 2;  // luminance row: blur apron + the extract's x neighbours
constexpr int CW = TX + 2 * kHalo;      // colour / extract row

// Pass 1.  Every input pixel of the tile and its apron is read once; the histogram counts
// only the tile's own pixels.  Counts are integers (< 2^24 per frame), so the u32 totals equal
// the reference's float atomics exactly.
__global__ __launch_bounds__(256) void k_lum_bloom(PostArgs a, int doHist, int doBloom) {
    __shared__ float sL[TY + 2][LW];
    __shared__ float sC[TY][CW][3];
    __shared__ unsigned sH[kBins];
    const int tid = threadIdx.x;
    const int x0 = blockIdx.x * TX, y0 = a.y0 + blockIdx.y * TY;
    const int W = a.W, H = a.H, y1 = a.y1;  // rows [y0, y1) are this band's; y0 - 1 and y1 its halo
    sH[tid] = 0u;
    __syncthreads();
    for (int i = tid; i < (TY + 2) * LW; i += 256) {
        const int ly = i / LW, lx = i - ly * LW;
        const int gy = y0 - 1 + ly, gx = x0 - kHalo - 1 + lx;
        float l = -INFINITY;
        if (gx >= 0 && gx < W && gy >= 0 && gy < H) {
            const V3 c = ld3(a.input, W, gx, gy);
            l = lum_ref(c);
            if (ly >= 1 && ly <= TY && lx >= 1 && lx <= CW && gy < y1) {
                sC[ly - 1][lx - 1][0] = c.x;
                sC[ly - 1][lx - 1][1] = c.y;
                sC[ly - 1][lx - 1][2] = c.z;
                if (doHist && lx > kHalo && lx <= kHalo + TX && !(l < 0.001f)) atomicAdd(&sH[hist_bin(l)], 1u);
            }
        }
        sL[ly][lx] = l;
    }
    __syncthreads();
    if (doHist) {
        const unsigned h = sH[tid];
        if (h) atomicAdd(&a.hist[tid], h);
    }
    if (!doBloom) return;
    const float thr = a.p.bloomThreshold;
    // extract in place at every in-image position (each position reads only its own colour)
    for (int i = tid; i < TY * CW; i += 256) {
        const int ey = i / CW, ex = i - ey * CW;
        const int gx = x0 - kHalo + ex, gy = y0 + ey;
        if (gx < 0 || gx >= W || gy >= y1) continue;
        const int lx = ex + 1, ly = ey + 1;
        const float n[4] = {sL[ly][lx - 1], sL[ly][lx + 1], sL[ly - 1][lx], sL[ly + 1][lx]};
        const V3 e = bloom_extract(V3(sC[ey][ex][0], sC[ey][ex][1], sC[ey][ex][2]), sL[ly][lx], n, thr);
        sC[ey][ex][0] = e.x;
        sC[ey][ex][1] = e.y;
        sC[ey][ex][2] = e.z;
    }
    __syncthreads();
    const int half = blur_half(a.p);  // <= kHalo, checked by the launcher
    for (int i = tid; i < TY * TX; i += 256) {
        const int ey = i / TX, ex = i - ey * TX;
        const int x = x0 + ex, y = y0 + ey;
        if (x >= W || y >= y1) continue;
        V3 r(0.0f);
        float tw = 0.0f;
        for (int k = -half; k <= half; k++) {  // edge-clamped taps; a clamped tap stays in the apron
            const int sx = clampi(x + k, 0, W - 1) - x0 + kHalo;
            r += V3(sC[ey][sx][0], sC[ey][sx][1], sC[ey][sx][2]) * 1.0f;
            tw += 1.0f;
        }
        if (tw > 0.0f) r /= tw;
        st3(a.bloomB, W, x, y, r, 1.0f);
    }
}

// Pass 2: ComputeAverageLuminanceKernel (:353-428) + the host's adaptation and exposure
// (:499-514), one wave.  The bin counts are integers below 2^24, so the total and the running
// sums of the reference's two serial scans are exact in any order: the wave computes them with
// a prefix scan and finds the first bin reaching each percentile with a ballot.  Only the
// weighted log-luminance sum rounds, and lane 0 accumulates it serially in the reference's order.
__global__ __launch_bounds__(64) void k_exposure(PostArgs a) {
    __shared__ float h[kBins];
    const int lane = threadIdx.x;
    float c4[4], run = 0.0f;
    for (int k = 0; k < 4; k++) {  // lane owns bins 4*lane .. 4*lane+3
        c4[k] = (float)a.hist[4 * lane + k];
        a.hist[4 * lane + k] = 0u;
        h[4 * lane + k] = c4[k];
        run += c4[k];
    }
    float incl = run;  // inclusive prefix over lanes
    for (int off = 1; off < 64; off <<= 1) {
        const float v = __shfl_up(incl, off, 64);
        if (lane >= off) incl += v;
    }
    const float total = __shfl(incl, 63, 64);
    const PostParamsDev &p = a.p;
    float avgLum = 0.18f;
    if (total != 0.0f) {
        const float minCount = total * p.histogramMinPercent / 100.0f;
        const float maxCount = total * p.histogramMaxPercent / 100.0f;
        // the first bin whose running sum reaches the count (the serial scan's break)
        int firstMin = kBins, firstMax = kBins;
        float acc = incl - run;
        for (int k = 0; k < 4; k++) {
            acc += c4[k];
            if (acc >= minCount && firstMin == kBins) firstMin = 4 * lane + k;
            if (acc >= maxCount && firstMax == kBins) firstMax = 4 * lane + k;
        }
        for (int off = 32; off >= 1; off >>= 1) {
            firstMin = min(firstMin, __shfl_xor(firstMin, off, 64));
            firstMax = min(firstMax, __shfl_xor(firstMax, off, 64));
        }
        const int minBin = firstMin < kBins ? firstMin : 0;
        const int maxBin = firstMax < kBins ? firstMax : kBins - 1;
        __syncthreads();
        if (lane != 0) return;
        float ws = 0.0f, wt = 0.0f;
#pragma unroll 8
        for (int i = minBin; i <= maxBin; i++) {
            const float binCenter = kMinLogLum + (i + 0.5f) * (kMaxLogLum - kMinLogLum) / kBins;
            ws += h[i] * binCenter;
            wt += h[i];
        }
        if (wt > 0.0f) avgLum = powf(10.0f, ws / wt);
    }
    if (lane != 0) return;
    const float adapt = p.exposureSpeed * a.dtMs;
    const float cur = a.state[0];
    const float next = cur + clampf(adapt, 0.0f, 1.0f) * (avgLum - cur);
    float e = p.targetLuminance / fmaxf(next, 0.001f);
    e *= powf(2.0f, p.exposureCompensation);
    e = clampf(e, powf(2.0f, p.exposureMin), powf(2.0f, p.exposureMax));
    a.state[0] = next;
    a.state[1] = e;
}

// Bloom for radii wider than the LDS apron: extract -> bloomA, horizontal blur -> bloomB
__global__ __launch_bounds__(256) void k_bloom_extract(PostArgs a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = a.y0 + blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.y1) return;
    const V3 c = ld3(a.input, a.W, x, y);
    float n[4];
    const int nx[4] = {x - 1, x + 1, x, x}, ny[4] = {y, y, y - 1, y + 1};
    for (int i = 0; i < 4; i++)
        n[i] = (nx[i] >= 0 && nx[i] < a.W && ny[i] >= 0 && ny[i] < a.H) ? lum_ref(ld3(a.input, a.W, nx[i], ny[i]))
                                                                        : -INFINITY;
    st3(a.bloomA, a.W, x, y, bloom_extract(c, lum_ref(c), n, a.p.bloomThreshold), 1.0f);
}

__global__ __launch_bounds__(256) void k_bloom_blur_h(PostArgs a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = a.y0 + blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.y1) return;
    const int half = blur_half(a.p);
    V3 r(0.0f);
    float tw = 0.0f;
    for (int i = -half; i <= half; i++) {
        r += ld3(a.bloomA, a.W, clampi(x + i, 0, a.W - 1), y) * 1.0f;
        tw += 1.0f;
    }
    if (tw > 0.0f) r /= tw;
    st3(a.bloomB, a.W, x, y, r, 1.0f);
}

// LensFlareKernel (:223-316) for one pixel: the flare added to the pixel
VX_D V3 lens_flare(const PostArgs &a, int x, int y) {
    const PostParamsDev &p = a.p;
    V3 flare(0.0f);
    const V2 uv((float)x / a.W, (float)y / a.H);
    const V2 center(0.5f, 0.5f);
    const float aspect = (float)a.W / (float)a.H;
    const V2 uvA(uv.x * aspect, uv.y), sunA(a.sunU * aspect, a.sunV), cenA(center.x * aspect, center.y);
    const V2 toSun = uvA - sunA;
    const float dist = sqrtf(toSun.x * toSun.x + toSun.y * toSun.y);
    const V2 s2c = cenA - sunA;
    const float axisDistance = sqrtf(s2c.x * s2c.x + s2c.y * s2c.y);
    const float sunSize = fmaxf(p.lensFlareSunSize, 0.0005f);
    const float light = fmaxf(a.sunLuminance, 1.0f);
    if (axisDistance > 0.0001f) {
        const V2 axisDir = s2c / axisDistance;
        if (dist < sunSize) {
            float f = 1.0f - (dist / sunSize);
            f = f * f;
            flare += V3(1.0f, 0.9f, 0.7f) * f * p.lensFlareIntensity * light * 0.1f;
        }
        if (p.lensFlareHaloRadius > 0.0001f) {
            const float h = expf(-dist * dist / (p.lensFlareHaloRadius * p.lensFlareHaloRadius));
            flare += V3(1.0f, 0.8f, 0.6f) * h * p.lensFlareIntensity * light * 0.08f;
        }
        for (int g = 1; g <= p.lensFlareGhostCount; ++g) {
            const float gf = p.lensFlareGhostSpacing * (float)g;
            const float gd = fminf(gf, 1.0f) * axisDistance;
            const V2 gc = sunA + axisDir * gd;
            const V2 tg = uvA - gc;
            const float gdist = sqrtf(tg.x * tg.x + tg.y * tg.y);
            const float gs = 0.02f + (g % 3) * 0.01f;
            const float fall = expf(-gdist * gdist / (gs * gs));
            const int m = g % 4;
            const V3 tint = m == 0 ? V3(1.0f, 0.7f, 0.3f) : (m == 1 ? V3(0.8f, 1.0f, 0.5f)
                            : (m == 2 ? V3(0.6f, 0.8f, 1.0f) : V3(1.0f, 0.6f, 0.8f)));
            const float gi = p.lensFlareIntensity * light * 0.04f *
                             (1.0f - (float)g / fmaxf((float)p.lensFlareGhostCount, 1.0f));
            flare += tint * fall * gi;
        }
        if (p.lensFlareDistortion > 0.0f) {
            const float start = fmaxf(sunSize * 1.5f, 0.02f);
            const float fade = clampf((dist - start) / 0.5f, 0.0f, 1.0f);
            const float strength = p.lensFlareDistortion * p.lensFlareIntensity * light * 0.02f;
            const float fall = (1.0f / (1.0f + dist * 6.0f)) * fade * fade;
            flare += V3(strength, 0.0f, -strength) * fall;
        }
    }
    return flare;
}

// VignetteKernel (:151-185) factor
VX_D float vignette(const PostParamsDev &p, int W, int H, int x, int y) {
    const float nx = (float)(2 * x - W) / (float)W, ny = (float)(2 * y - H) / (float)H;
    const float d = sqrtf(nx * nx + ny * ny);
    const float t = clampf((d - p.vignetteRadius) / p.vignetteSmoothness, 0.0f, 1.0f);
    const float sm = t * t * (3.0f - 2.0f * t);
    float v = 1.0f - sm;
    v = 1.0f - p.vignetteStrength * (1.0f - v);
    return clampf(v, 0.0f, 1.0f);
}

VX_D V3 aces(V3 x) {  // FilmicToneMapping.h:12-20
    const float A = 2.51f, B = 0.03f, C = 2.43f, D = 0.59f, E = 0.14f;
    return clamp3(x * (A * x + V3(B)) / (x * (C * x + V3(D)) + V3(E)), 0.0f, 1.0f);
}
VX_D V3 uncharted2(V3 x) {  // :23-32
    const float A = 0.15f, B = 0.50f, C = 0.10f, D = 0.20f, E = 0.02f, F = 0.30f;
    return ((x * (A * x + V3(C * B)) + V3(D * E)) / (x * (A * x + V3(B)) + V3(D * F))) - V3(E / F);
}
VX_D float srgb(float c) { return (c <= 0.0031308f) ? 12.92f * c : 1.055f * powf(c, 1.0f / 2.4f) - 0.055f; }

// Pass 3: vertical blur + BloomCompositeKernel (:128-148), LensFlareKernel (its sun-visibility
// test, IsSunVisible :208-221 -- depth at the sun pixel >= RayMaxLowerBound -- read on the device),
// VignetteKernel, FilmicToneMapping (:58-117), DrawCrosshair (PostProcessor.cu:14-46),
// CopyToInteropBuffer (:48-63).  64-wide rows: the vertical taps are coalesced row reads.
__global__ __launch_bounds__(256) void k_compose(PostArgs a, int flare) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = a.y0 + blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= a.W || y >= a.y1) return;
    const PostParamsDev &p = a.p;
    V3 c = ld3(a.input, a.W, x, y);
    if (p.enableBloom) {
        const int half = blur_half(p);
        V3 r(0.0f);
        float tw = 0.0f;
        for (int i = -half; i <= half; i++) {
            r += ld3(a.bloomB, a.W, x, clampi(y + i, 0, a.H - 1)) * 1.0f;
            tw += 1.0f;
        }
        if (tw > 0.0f) r /= tw;
        c = c + r * p.bloomIntensity;
    }
    if (flare && a.hist[kBins] != 0u) c = c + lens_flare(a, x, y);  // the sun pixel is sky (k_sun_flag)
    if (p.enableVignette) c *= vignette(p, a.W, a.H, x, y);
    c *= p.enableAutoExposure ? a.state[1] : p.manualExposure;
    V3 t;
    if (p.curve == 1) {
        const float Wp = p.whitePoint;
        const V3 ws = V3(1.0f) / uncharted2(V3(Wp));
        t = uncharted2(c * 2.0f) * ws;
    } else if (p.curve == 2) {
        const V3 num = c * (V3(1.0f) + (c / (p.whitePoint * p.whitePoint)));
        t = num / (V3(1.0f) + c);
    } else {
        t = aces(c);
    }
    t = clamp3(t, 0.0f, 1.0f);
    if (p.contrast != 1.0f)  // pow(x, 1) = x exactly
        t = V3(powf(t.x, p.contrast), powf(t.y, p.contrast), powf(t.z, p.contrast));
    const float l = lum_ref(t);
    t = V3(l) + p.saturation * (t - V3(l));
    t = clamp3(t * p.gain + V3(p.lift), 0.0f, 1.0f);
    t = V3(srgb(t.x), srgb(t.y), srgb(t.z));
    if (p.crosshair) {
        const int cx = a.W / 2, cy = a.H / 2;
        if ((abs(y - cy) <= 1 && abs(x - cx) <= 10) || (abs(x - cx) <= 1 && abs(y - cy) <= 10)) t = V3(1.0f);
    }
    a.frame[(size_t)y * a.W + x] = make_float4(t.x, t.y, t.z, 0.0f);
}

// The lens flare's sun test (depth of the sun's pixel is sky) as a flag beside the histogram,
// written by the band that owns the pixel (0 elsewhere), so that a band all-reduce of the
// histogram carries it to every band
__global__ void k_sun_flag(PostArgs a) {
    const bool own = a.sunPy >= a.y0 && a.sunPy < a.y1;
    a.hist[kBins] = (own && a.depth[(size_t)a.sunPy * a.W + a.sunPx] >= 1.0e26f) ? 1u : 0u;
}

}  // namespace

int post_bloom_half(const PostArgs &a) { return a.p.enableBloom ? blur_half(a.p) : 0; }

// HBM traffic per pixel with bloom on: pass 1 reads 16 B (+ apron) and writes 16 B of bloomB,
// pass 3 reads 16 B input + 16 B bloomB (+ taps from cache) and writes 16 B: 80 B per pixel.
// Phase 1: histogram + bloom of the band's rows (reads input rows y0 - 1 .. y1) and the sun flag;
// phase 2 (after a banded frame's histogram all-reduce and bloomB halo): exposure + compose.
hipError_t launch_post_phase1(const PostArgs &a, hipStream_t st) {
    const int rows = a.y1 - a.y0;
    const bool lds = blur_half(a.p) <= kHalo;
    const int hist = a.p.enableAutoExposure ? 1 : 0, bloomLds = a.p.enableBloom && lds ? 1 : 0;
    if (hist || bloomLds)
        hipLaunchKernelGGL(k_lum_bloom, dim3((a.W + TX - 1) / TX, (rows + TY - 1) / TY), dim3(256), 0, st, a, hist,
                           bloomLds);
    if (a.p.enableBloom && !lds) {
        const dim3 g((a.W + 15) / 16, (rows + 15) / 16);
        hipLaunchKernelGGL(k_bloom_extract, g, dim3(256), 0, st, a);
        hipLaunchKernelGGL(k_bloom_blur_h, g, dim3(256), 0, st, a);
    }
    if (a.p.enableLensFlare && a.sunOnScreen) hipLaunchKernelGGL(k_sun_flag, dim3(1), dim3(1), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_post_phase2(const PostArgs &a, hipStream_t st) {
    if (a.p.enableAutoExposure) hipLaunchKernelGGL(k_exposure, dim3(1), dim3(64), 0, st, a);
    hipLaunchKernelGGL(k_compose, dim3((a.W + 63) / 64, (a.y1 - a.y0 + 3) / 4), dim3(256), 0, st, a,
                       a.p.enableLensFlare && a.sunOnScreen ? 1 : 0);
    return hipGetLastError();
}
hipError_t launch_postprocess(const PostArgs &a, hipStream_t st) {
    if (hipError_t e = launch_post_phase1(a, st)) return e;
    return launch_post_phase2(a, st);
}

}  // namespace vx
