// ORACLE (test infrastructure only) -- CPU restatement of the reference's
// offline post-processing (PostProcessor::run, renderer/postprocessing/PostProcessor.cu:74-122):
//   auto-exposure  ComputeLuminanceHistogramKernel / ComputeAverageLuminanceKernel
//                  (PostProcessingPipeline.cu:319-428) + the host adaptation (:499-514)
//   bloom          BloomExtractBrightPixelsKernel / BloomBlurKernel / BloomCompositeKernel (:12-148)
//   lens flare     LensFlareKernel (:223-316), IsSunVisible (:208-221)
//   vignette       VignetteKernel (:151-185)
//   tone mapping   FilmicToneMapping (FilmicToneMapping.h:58-117)
//   crosshair      DrawCrosshair (PostProcessor.cu:14-46), CopyToInteropBuffer (:48-63)
// Every pass is a sequential loop over pixels in the reference's per-pixel
// arithmetic; the histogram counts are exact, so the parallel order of the
// reference's atomics does not matter.
#include <cmath>
#include <cstdlib>
#include <vector>

#include "orc_math.h"

using namespace orc;

namespace {

struct PostParams {  // ToneMappingParams + PostProcessingPipelineParams (GlobalSettings.h:10-186)
    float manualExposure;
    int curve;
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

F3 aces(F3 x) {
    const float a = 2.51f, b = 0.03f, c = 2.43f, d = 0.59f, e = 0.14f;
    return clamp3f(x * (a * x + b) / (x * (c * x + d) + e), F3(0.0f), F3(1.0f));
}
F3 uncharted2(F3 x) {
    const float A = 0.15f, B = 0.50f, C = 0.10f, D = 0.20f, E = 0.02f, F = 0.30f;
    return ((x * (A * x + C * B) + D * E) / (x * (A * x + B) + D * F)) - E / F;
}
float srgb(float c) { return (c <= 0.0031308f) ? 12.92f * c : 1.055f * std::pow(c, 1.0f / 2.4f) - 0.055f; }

}  // namespace

extern "C" void orc_postprocess(int W, int H, const float *in, const float *depth, const void *params,
                                float *state, float dtMs, int sunOnScreen, int sunPx, int sunPy, float sunU,
                                float sunV, float sunLuminance, float *out) {
    const PostParams &p = *static_cast<const PostParams *>(params);
    const size_t n = (size_t)W * H;
    std::vector<F3> col(n), bloomA(n), bloomB(n);
    for (size_t i = 0; i < n; i++) col[i] = F3(in[4 * i], in[4 * i + 1], in[4 * i + 2]);
    auto at = [&](std::vector<F3> &b, int x, int y) -> F3 & { return b[(size_t)y * W + x]; };
    float exposure = p.manualExposure;
    if (p.enableAutoExposure) {
        float hist[256] = {};
        for (size_t i = 0; i < n; i++) {
            const float l = luminance(col[i]);
            if (l < 0.001f) continue;
            const float t = clampf((std::log10(l) - (-8.0f)) / (4.0f - (-8.0f)), 0.0f, 1.0f);
            const int bin = mymin((int)(t * 256), 255);
            hist[bin] += 1.0f;
        }
        float total = 0.0f;
        for (int i = 0; i < 256; i++) total += hist[i];
        float avg = 0.18f;
        if (total != 0.0f) {
            const float minCount = total * p.histogramMinPercent / 100.0f;
            const float maxCount = total * p.histogramMaxPercent / 100.0f;
            float acc = 0.0f;
            int minBin = 0, maxBin = 255;
            for (int i = 0; i < 256; i++) {
                acc += hist[i];
                if (acc >= minCount) { minBin = i; break; }
            }
            acc = 0.0f;
            for (int i = 0; i < 256; i++) {
                acc += hist[i];
                if (acc >= maxCount) { maxBin = i; break; }
            }
            float ws = 0.0f, wt = 0.0f;
            for (int i = minBin; i <= maxBin; i++) {
                const float bc = -8.0f + (i + 0.5f) * (4.0f - (-8.0f)) / 256;
                ws += hist[i] * bc;
                wt += hist[i];
            }
            if (wt > 0.0f) avg = std::pow(10.0f, ws / wt);
        }
        state[0] = lerpf(state[0], avg, clampf(p.exposureSpeed * dtMs, 0.0f, 1.0f));
        exposure = p.targetLuminance / std::fmax(state[0], 0.001f);
        exposure *= std::pow(2.0f, p.exposureCompensation);
        exposure = clampf(exposure, std::pow(2.0f, p.exposureMin), std::pow(2.0f, p.exposureMax));
        state[1] = exposure;
    }
    if (p.enableBloom) {
        const float thr = p.bloomThreshold;
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) {
                F3 c = at(col, x, y);
                if (luminance(c) > thr) {
                    float maxN = 0.0f;
                    const int nx[4] = {x - 1, x + 1, x, x}, ny[4] = {y, y, y - 1, y + 1};
                    for (int i = 0; i < 4; i++)
                        if (nx[i] >= 0 && nx[i] < W && ny[i] >= 0 && ny[i] < H)
                            maxN = std::fmax(maxN, luminance(at(col, nx[i], ny[i])));
                    c = maxN < thr * 0.4f ? F3(0.0f) : clamp3f((c - F3(thr)) * 0.7f, F3(0.0f), F3(100.0f));
                } else {
                    c = F3(0.0f);
                }
                at(bloomA, x, y) = c;
            }
        const int half = ((int)(p.bloomRadius * 2.0f) + 1) / 2;
        for (int pass = 0; pass < 2; pass++) {
            std::vector<F3> &src = pass == 0 ? bloomA : bloomB, &dst = pass == 0 ? bloomB : bloomA;
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++) {
                    F3 r(0.0f);
                    float tw = 0.0f;
                    for (int i = -half; i <= half; i++) {
                        const int sx = clampi(x + (pass == 0 ? i : 0), 0, W - 1), sy = clampi(y + (pass == 1 ? i : 0), 0, H - 1);
                        r += at(src, sx, sy) * 1.0f;
                        tw += 1.0f;
                    }
                    if (tw > 0.0f) r /= tw;
                    at(dst, x, y) = r;
                }
        }
        for (size_t i = 0; i < n; i++) col[i] = col[i] + bloomA[i] * p.bloomIntensity;
    }
    if (p.enableLensFlare && sunOnScreen && depth[(size_t)sunPy * W + sunPx] >= 1.0e26f) {
        const float aspect = (float)W / (float)H;
        const F2 sunA(sunU * aspect, sunV), cenA(0.5f * aspect, 0.5f);
        const F2 s2c = cenA - sunA;
        const float axisDistance = std::sqrt(s2c.x * s2c.x + s2c.y * s2c.y);
        const float sunSize = std::fmax(p.lensFlareSunSize, 0.0005f), light = std::fmax(sunLuminance, 1.0f);
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) {
                F3 flare(0.0f);
                const F2 uv((float)x / W, (float)y / H);
                const F2 uvA(uv.x * aspect, uv.y);
                const F2 ts = uvA - sunA;
                const float dist = std::sqrt(ts.x * ts.x + ts.y * ts.y);
                if (axisDistance > 0.0001f) {
                    const F2 axisDir = s2c / axisDistance;
                    if (dist < sunSize) {
                        float f = 1.0f - (dist / sunSize);
                        f = f * f;
                        flare += F3(1.0f, 0.9f, 0.7f) * f * p.lensFlareIntensity * light * 0.1f;
                    }
                    if (p.lensFlareHaloRadius > 0.0001f) {
                        const float h = std::exp(-dist * dist / (p.lensFlareHaloRadius * p.lensFlareHaloRadius));
                        flare += F3(1.0f, 0.8f, 0.6f) * h * p.lensFlareIntensity * light * 0.08f;
                    }
                    for (int g = 1; g <= p.lensFlareGhostCount; ++g) {
                        const float gd = std::fmin(p.lensFlareGhostSpacing * (float)g, 1.0f) * axisDistance;
                        const F2 gc = sunA + axisDir * gd;
                        const F2 tg = uvA - gc;
                        const float gdist = std::sqrt(tg.x * tg.x + tg.y * tg.y);
                        const float gs = 0.02f + (g % 3) * 0.01f;
                        const float fall = std::exp(-gdist * gdist / (gs * gs));
                        F3 tint;
                        switch (g % 4) {
                            case 0: tint = F3(1.0f, 0.7f, 0.3f); break;
                            case 1: tint = F3(0.8f, 1.0f, 0.5f); break;
                            case 2: tint = F3(0.6f, 0.8f, 1.0f); break;
                            default: tint = F3(1.0f, 0.6f, 0.8f); break;
                        }
                        const float gi = p.lensFlareIntensity * light * 0.04f *
                                         (1.0f - (float)g / std::fmax((float)p.lensFlareGhostCount, 1.0f));
                        flare += tint * fall * gi;
                    }
                    if (p.lensFlareDistortion > 0.0f) {
                        const float start = std::fmax(sunSize * 1.5f, 0.02f);
                        const float fade = clampf((dist - start) / 0.5f, 0.0f, 1.0f);
                        const float strength = p.lensFlareDistortion * p.lensFlareIntensity * light * 0.02f;
                        const float fall = (1.0f / (1.0f + dist * 6.0f)) * fade * fade;
                        flare += F3(strength, 0.0f, -strength) * fall;
                    }
                }
                at(col, x, y) = at(col, x, y) + flare;
            }
    }
    if (p.enableVignette)
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) {
                const float fx = (2.0f * x - W) / (float)W, fy = (2.0f * y - H) / (float)H;
                const float d = std::sqrt(fx * fx + fy * fy);
                const float t = clampf((d - p.vignetteRadius) / p.vignetteSmoothness, 0.0f, 1.0f);
                float v = 1.0f - t * t * (3.0f - 2.0f * t);
                v = clampf(1.0f - p.vignetteStrength * (1.0f - v), 0.0f, 1.0f);
                at(col, x, y) = at(col, x, y) * v;
            }
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            F3 c = at(col, x, y) * (p.enableAutoExposure ? exposure : p.manualExposure);
            F3 t;
            if (p.curve == 1) {
                const F3 ws = F3(1.0f) / uncharted2(F3(p.whitePoint));
                t = uncharted2(c * 2.0f) * ws;
            } else if (p.curve == 2) {
                t = (c * (1.0f + (c / (p.whitePoint * p.whitePoint)))) / (1.0f + c);
            } else {
                t = aces(c);
            }
            t = clamp3f(t, F3(0.0f), F3(1.0f));
            t = F3(std::pow(t.x, p.contrast), std::pow(t.y, p.contrast), std::pow(t.z, p.contrast));
            const float l = luminance(t);
            t = lerp3(F3(l), t, p.saturation);
            t = clamp3f(t * p.gain + p.lift, F3(0.0f), F3(1.0f));
            t = F3(srgb(t.x), srgb(t.y), srgb(t.z));
            if (p.crosshair) {
                const int cx = W / 2, cy = H / 2;
                if ((std::abs(y - cy) <= 1 && std::abs(x - cx) <= 10) || (std::abs(x - cx) <= 1 && std::abs(y - cy) <= 10))
                    t = F3(1.0f);
            }
            float *o = out + 4 * ((size_t)y * W + x);
            o[0] = t.x; o[1] = t.y; o[2] = t.z; o[3] = 0.0f;
        }
}
