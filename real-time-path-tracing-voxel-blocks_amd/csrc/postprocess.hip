// vxpt -- offline post-processing on gfx950 (PostProcessor::run, PostProcessor.cu:74-122):
// histogram auto-exposure, bloom, lens flare, vignette (PostProcessingPipeline.cu:11-601),
// filmic tone mapping (FilmicToneMapping.h:11-117), crosshair, copy to the frame buffer.
//
// The reference works in place on IlluminationOutputBuffer; here the denoiser
// output stays intact (parity hook) and the chain runs on a working plane,
// ending in the frame plane (Float4(colour, 0), CopyToInteropBuffer).  The
// auto-exposure state (current average luminance) lives on the device, so the
// reference's host round trip (cudaMemcpy of the average, PostProcessingPipeline.cu:495-514)
// becomes a one-thread kernel and the frame needs no host synchronisation.
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

// ComputeLuminanceHistogramKernel (PostProcessingPipeline.cu:319-350): counts are exact (< 2^24)
__global__ __launch_bounds__(256) void k_histogram(PostArgs a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.H) return;
    const float l = lum_ref(ld3(a.work, a.W, x, y));
    if (l < 0.001f) return;
    const float logLum = log10f(l);
    const float t = clampf((logLum - kMinLogLum) / (kMaxLogLum - kMinLogLum), 0.0f, 1.0f);
    const int bin = min((int)(t * kBins), kBins - 1);
    atomicAdd(&a.hist[bin], 1.0f);
}

// ComputeAverageLuminanceKernel (:353-428) + the host's adaptation and exposure
// (:499-514), one thread; state[0] = current average luminance, state[1] = exposure
__global__ void k_exposure(PostArgs a) {
    const float *h = a.hist;
    const PostParamsDev &p = a.p;
    float total = 0.0f;
    for (int i = 0; i < kBins; i++) total += h[i];
    float avgLum = 0.18f;
    if (total != 0.0f) {
        const float minCount = total * p.histogramMinPercent / 100.0f;
        const float maxCount = total * p.histogramMaxPercent / 100.0f;
        float acc = 0.0f;
        int minBin = 0, maxBin = kBins - 1;
        for (int i = 0; i < kBins; i++) {
            acc += h[i];
            if (acc >= minCount) { minBin = i; break; }
        }
        acc = 0.0f;
        for (int i = 0; i < kBins; i++) {
            acc += h[i];
            if (acc >= maxCount) { maxBin = i; break; }
        }
        float ws = 0.0f, wt = 0.0f;
        for (int i = minBin; i <= maxBin; i++) {
            const float binCenter = kMinLogLum + (i + 0.5f) * (kMaxLogLum - kMinLogLum) / kBins;
            ws += h[i] * binCenter;
            wt += h[i];
        }
        if (wt > 0.0f) avgLum = powf(10.0f, ws / wt);
    }
    const float adapt = p.exposureSpeed * a.dtMs;
    const float cur = a.state[0];
    const float next = cur + clampf(adapt, 0.0f, 1.0f) * (avgLum - cur);
    float e = p.targetLuminance / fmaxf(next, 0.001f);
    e *= powf(2.0f, p.exposureCompensation);
    e = clampf(e, powf(2.0f, p.exposureMin), powf(2.0f, p.exposureMax));
    a.state[0] = next;
    a.state[1] = e;
}

// BloomExtractBrightPixelsKernel (:12-80), neighbour filter on
__global__ __launch_bounds__(256) void k_bloom_extract(PostArgs a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.H) return;
    const float thr = a.p.bloomThreshold;
    V3 c = ld3(a.work, a.W, x, y);
    if (lum_ref(c) > thr) {
        float maxN = 0.0f;
        const int nx[4] = {x - 1, x + 1, x, x}, ny[4] = {y, y, y - 1, y + 1};
        for (int i = 0; i < 4; i++)
            if (nx[i] >= 0 && nx[i] < a.W && ny[i] >= 0 && ny[i] < a.H)
                maxN = fmaxf(maxN, lum_ref(ld3(a.work, a.W, nx[i], ny[i])));
        if (maxN < thr * 0.4f) c = V3(0.0f);
        else c = clamp3((c - V3(thr)) * 0.7f, 0.0f, 100.0f);
    } else {
        c = V3(0.0f);
    }
    st3(a.bloomA, a.W, x, y, c, 1.0f);
}

// BloomBlurKernel (:83-125): box blur along one axis, edge-clamped
__global__ __launch_bounds__(256) void k_bloom_blur(PostArgs a, const float4 *in, float4 *out, int dx, int dy) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.H) return;
    const int half = ((int)(a.p.bloomRadius * 2.0f) + 1) / 2;
    V3 r(0.0f);
    float tw = 0.0f;
    for (int i = -half; i <= half; i++) {
        const int sx = clampi(x + dx * i, 0, a.W - 1), sy = clampi(y + dy * i, 0, a.H - 1);
        r += ld3(in, a.W, sx, sy) * 1.0f;
        tw += 1.0f;
    }
    if (tw > 0.0f) r /= tw;
    st3(out, a.W, x, y, r, 1.0f);
}

// BloomCompositeKernel (:128-148)
__global__ __launch_bounds__(256) void k_bloom_composite(PostArgs a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.H) return;
    const V3 c = ld3(a.work, a.W, x, y) + ld3(a.bloomA, a.W, x, y) * a.p.bloomIntensity;
    st3(a.work, a.W, x, y, c, 1.0f);
}

// LensFlareKernel (:223-316); the sun-visibility test of the host (IsSunVisible,
// :208-221: depth at the sun pixel >= RayMaxLowerBound) is read here on the device
__global__ __launch_bounds__(256) void k_lens_flare(PostArgs a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.H) return;
    if (!(a.depth[(size_t)a.sunPy * a.W + a.sunPx] >= 1.0e26f)) return;
    const PostParamsDev &p = a.p;
    const V3 orig = ld3(a.work, a.W, x, y);
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
    st3(a.work, a.W, x, y, orig + flare, 1.0f);
}

// VignetteKernel (:151-185)
__global__ __launch_bounds__(256) void k_vignette(PostArgs a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.H) return;
    const PostParamsDev &p = a.p;
    V3 c = ld3(a.work, a.W, x, y);
    const float nx = (float)(2 * x - a.W) / (float)a.W, ny = (float)(2 * y - a.H) / (float)a.H;
    const float d = sqrtf(nx * nx + ny * ny);
    const float t = clampf((d - p.vignetteRadius) / p.vignetteSmoothness, 0.0f, 1.0f);
    const float sm = t * t * (3.0f - 2.0f * t);
    float v = 1.0f - sm;
    v = 1.0f - p.vignetteStrength * (1.0f - v);
    v = clampf(v, 0.0f, 1.0f);
    c *= v;
    st3(a.work, a.W, x, y, c, 1.0f);
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

// FilmicToneMapping (:58-117) + DrawCrosshair (PostProcessor.cu:14-46) +
// CopyToInteropBuffer (:48-63)
__global__ __launch_bounds__(256) void k_tonemap(PostArgs a) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= a.W || y >= a.H) return;
    const PostParamsDev &p = a.p;
    V3 c = ld3(a.work, a.W, x, y);
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

inline dim3 grid(const PostArgs &a) { return dim3((a.W + 15) / 16, (a.H + 15) / 16); }

}  // namespace

hipError_t launch_postprocess(const PostArgs &a, hipStream_t st) {
    const dim3 g = grid(a), b(256);
    hipMemcpyAsync(a.work, a.input, (size_t)a.W * a.H * sizeof(float4), hipMemcpyDeviceToDevice, st);
    if (a.p.enableAutoExposure) {
        hipMemsetAsync(a.hist, 0, kBins * sizeof(float), st);
        hipLaunchKernelGGL(k_histogram, g, b, 0, st, a);
        hipLaunchKernelGGL(k_exposure, dim3(1), dim3(1), 0, st, a);
    }
    if (a.p.enableBloom) {
        hipLaunchKernelGGL(k_bloom_extract, g, b, 0, st, a);
        hipLaunchKernelGGL(k_bloom_blur, g, b, 0, st, a, a.bloomA, a.bloomB, 1, 0);
        hipLaunchKernelGGL(k_bloom_blur, g, b, 0, st, a, a.bloomB, a.bloomA, 0, 1);
        hipLaunchKernelGGL(k_bloom_composite, g, b, 0, st, a);
    }
    if (a.p.enableLensFlare && a.sunOnScreen) hipLaunchKernelGGL(k_lens_flare, g, b, 0, st, a);
    if (a.p.enableVignette) hipLaunchKernelGGL(k_vignette, g, b, 0, st, a);
    hipLaunchKernelGGL(k_tonemap, g, b, 0, st, a);
    return hipGetLastError();
}

}  // namespace vx
