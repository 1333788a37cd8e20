// ORACLE (test infrastructure only): restatement of renderer/sky/Sky.cu and
// the CPU alias-table build of renderer/shaders/AliasTable.cu.
#include "orc_sky.h"

#include <cstdio>
#include <queue>
#include <string>

namespace orc {

static bool read_f32(const std::string &p, std::vector<float> &v, size_t n) {
    FILE *f = std::fopen(p.c_str(), "rb");
    if (!f) return false;
    v.resize(n);
    size_t got = std::fread(v.data(), 4, n, f);
    std::fclose(f);
    return got == n;
}

bool Sky::load_tables(const char *dir) {
    std::string d(dir);
    return read_f32(d + "/sky_datasets.f32", tSky, 540) && read_f32(d + "/sky_datasets_rad.f32", tSkyRad, 60) &&
           read_f32(d + "/solar_datasets.f32", tSolar, 1800) && read_f32(d + "/limb_darkening.f32", tLimb, 60);
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
        float p = w[i] / sum;
        prob[i] = p;
        scaled[i] = p * n;
    }
    std::queue<int> small, large;
    for (unsigned i = 0; i < n; ++i) (scaled[i] < 1.0f ? small : large).push((int)i);
    while (!small.empty() && !large.empty()) {
        int s = small.front(); small.pop();
        int l = large.front(); large.pop();
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

namespace {
// SpectrumToXyz (Sky.cu:85-131)
const float kCieX[10] = {2.372527e-02f, 1.955480e+00f, 1.074553e+01f, 5.056697e+00f, 4.698190e+00f,
                         2.391135e+01f, 3.798705e+01f, 1.929414e+01f, 2.970610e+00f, 2.092986e-01f};
const float kCieY[10] = {6.813859e-04f, 6.771017e-02f, 1.171193e+00f, 6.997765e+00f, 2.666710e+01f,
                         3.758372e+01f, 2.503930e+01f, 8.150395e+00f, 1.098635e+00f, 7.563256e-02f};
const float kCieZ[10] = {1.119121e-01f, 9.441195e+00f, 5.597921e+01f, 3.589996e+01f, 5.070894e+00f,
                         3.523189e-01f, 3.422707e-02f, 2.539118e-03f, 7.836666e-06f, 0.000000e+00f};
inline F3 spectrum_xyz(int c) {
    constexpr float kCieYIntegral = 106.856895f;
    return F3(kCieX[c], kCieY[c], kCieZ[c]) / kCieYIntegral;
}
inline F3 xyz_to_srgb(const F3 &xyz) {  // util/ColorSpace.h:18-29
    const M3 m(3.2404542f, -1.5371385f, -0.4985314f, -0.9692660f, 1.8760108f, 0.0415560f, 0.0556434f, -0.2040259f,
               1.0572252f);
    return m * xyz;
}
float fit6(const float *M, float t, int i, int stride) {  // Sky.cu:19-47
    return (std::pow(1.0f - t, 5.0f) * M[i] + 5.0f * std::pow(1.0f - t, 4.0f) * t * M[i + stride] +
            10.0f * std::pow(1.0f - t, 3.0f) * std::pow(t, 2.0f) * M[i + 2 * stride] +
            10.0f * std::pow(1.0f - t, 2.0f) * std::pow(t, 3.0f) * M[i + 3 * stride] +
            5.0f * (1.0f - t) * std::pow(t, 4.0f) * M[i + 4 * stride] + std::pow(t, 5.0f) * M[i + 5 * stride]);
}

struct SkyState { float cfg[90]; float rad[10]; };

F3 sky_radiance(const SkyState &s, const F3 &rd, const F3 &sunDir) {  // Sky.cu:133-173
    float theta = std::acos(rd.y);
    float gamma = std::acos(clampf(dot(rd, sunDir), -1, 1));
    F3 xyz(0);
    for (int ch = 0; ch < 10; ++ch) {
        const float *c = s.cfg + ch * 9;
        const float expM = std::exp(c[4] * gamma);
        const float rayM = std::cos(gamma) * std::cos(gamma);
        const float mieM = (1.0f + std::cos(gamma) * std::cos(gamma)) /
                           std::pow((1.0f + c[8] * c[8] - 2.0f * c[8] * std::cos(gamma)), 1.5f);
        const float zenith = std::sqrt(std::cos(theta));
        // `cos(theta) + 0.01` promotes the first factor to binary64
        const double f1 = 1.0f + (double)c[0] * std::exp((double)c[1] / ((double)std::cos(theta) + 0.01));
        const float f2 = c[2] + c[3] * expM + c[5] * rayM + c[6] * mieM + c[7] * zenith;
        float ri = (float)(f1 * (double)f2);
        float radiance = ri * s.rad[ch];
        xyz += radiance * spectrum_xyz(ch);
    }
    return xyz_to_srgb(xyz);
}

F3 sun_radiance(const Sky &sk, const F3 &rd, const F3 &sunDir) {  // Sky.cu:175-257
    float gamma = std::acos(clampf(dot(rd, sunDir), -1, 1));
    float elevation = (kPi / 2.0f) - std::acos(sunDir.y);
    const float sunAngle = 0.51f;
    const float solarRadius = sunAngle * kPi / 180.0f / 2.0f;
    const float scale = 1.0f / ((sunAngle / 0.51f) * (sunAngle / 0.51f));
    F3 xyz(0);
    float srs = std::sin(solarRadius);
    float ar2 = 1.0f / (srs * srs);
    float sg = std::sin(gamma);
    float sc2 = 1.0f - ar2 * sg * sg;
    if (sc2 < 0.0f) sc2 = 0.0f;
    float sampleCos = std::sqrt(sc2);
    if (sampleCos == 0.0f) return F3(0.0f);
    for (int ch = 0; ch < 10; ++ch) {
        const int pieces = 45, order = 4;
        int pos = (int)(std::pow((float)(2.0 * (double)elevation / (double)kPi), (float)(1.0 / 3.0)) * pieces);
        if (pos > 44) pos = 44;
        const float breakX = (float)((double)std::pow(((float)pos / (float)pieces), 3.0f) * ((double)kPi * 0.5));
        const float *coefs = sk.tSolar.data() + ch * 180 + (order * (pos + 1) - 1);
        float res = 0.0f;
        const float x = elevation - breakX;
        float xe = 1.0f;
        for (int i = 0; i < order; ++i) {
            res += xe * *coefs--;
            xe *= x;
        }
        float direct = res;
        const float *ld = sk.tLimb.data() + ch * 6;
        float dark = ld[0] + ld[1] * sampleCos + ld[2] * std::pow(sampleCos, 2.0f) + ld[3] * std::pow(sampleCos, 3.0f) +
                     ld[4] * std::pow(sampleCos, 4.0f) + ld[5] * std::pow(sampleCos, 5.0f);
        direct *= dark * scale;
        xyz += direct * spectrum_xyz(ch);
    }
    return xyz_to_srgb(xyz);
}
}  // namespace

void Sky::build(float timeOfDay, float axisAngle, float axisRotate, float brightness) {
    // sun direction (Sky.cu:363-368)
    F3 axis(1.0f, std::cos(axisAngle * kPiOver180), std::sin(axisAngle * kPiOver180));
    axis *= F3(std::sin(axisRotate * kPiOver180), 1.0f, std::cos(axisRotate * kPiOver180));
    axis = normalize(axis);
    const float angle = std::fmod(timeOfDay * kPi, kTwoPi);
    sunDir = rotate3f(axis, angle, cross(F3(0, 1, 0), axis)).normalized();

    // updateSkyState (Sky.cu:57-83)
    SkyState st;
    float elevation = (kPi / 2.0f) - std::acos(sunDir.y);
    float se = std::pow(elevation / (kPi / 2.0f), (1.0f / 3.0f));
    for (int ch = 0; ch < 10; ++ch) {
        for (int i = 0; i < 9; ++i) st.cfg[ch * 9 + i] = fit6(tSky.data() + ch * 54, se, i, 9);
        st.rad[ch] = fit6(tSkyRad.data() + ch * 6, se, 0, 1);
    }

    sky.assign((size_t)skyW * skyH * 4, 0.0f);
    sun.assign((size_t)sunW * sunH * 4, 0.0f);
    std::vector<float> skyPdf((size_t)skyW * skyH, 0.0f), sunPdf((size_t)sunW * sunH, 0.0f);
    const int half = skyH / 2;
    // kernel Sky (Sky.cu:259-280): upper hemisphere rows half..skyH-1
    for (int y = 0; y < half; ++y)
        for (int x = 0; x < skyW; ++x) {
            float u = ((float)x + 0.5f) / (float)skyW;
            float v = ((float)y + 0.5f) / (float)half;
            int yy = y + half;
            F3 rd = equal_area_hemisphere_dir(u, v);
            F3 c = sky_radiance(st, rd, sunDir) * brightness;
            c = max3f(c, F3(0.0f));
            size_t i = (size_t)skyW * yy + x;
            sky[i * 4 + 0] = c.x; sky[i * 4 + 1] = c.y; sky[i * 4 + 2] = c.z; sky[i * 4 + 3] = 0.0f;
            skyPdf[i] = luminance(c);
        }
    double upper = 0.0;
    for (size_t i = (size_t)skyW * half; i < (size_t)skyW * skyH; ++i) upper += (double)skyPdf[i];
    const float sumUpper = (float)upper;
    // kernel SkyLowerHemisphere (Sky.cu:282-303)
    for (int y = 0; y < half; ++y)
        for (int x = 0; x < skyW; ++x) {
            float v = ((float)y + 0.5f) / (float)half - 1.0f;
            F3 mist(sumUpper / (float)(skyW * skyH));
            float blend = clampf((v + 0.4f) * (1.0f / 0.5f));
            size_t j = (size_t)skyW * half + x;
            F3 em(sky[j * 4 + 0], sky[j * 4 + 1], sky[j * 4 + 2]);
            F3 c = smoothstep3f(mist, em, blend);
            size_t i = (size_t)skyW * y + x;
            sky[i * 4 + 0] = c.x; sky[i * 4 + 1] = c.y; sky[i * 4 + 2] = c.z; sky[i * 4 + 3] = 0.0f;
            skyPdf[i] = luminance(c);
        }
    skyAlias = build_alias(skyPdf, skySum);
    // kernel SkySun (Sky.cu:305-327)
    const float cosMax = std::cos(0.51f * kPi / 180.0f / 2.0f);
    for (int y = 0; y < sunH; ++y)
        for (int x = 0; x < sunW; ++x) {
            float u = ((float)x + 0.5f) / (float)sunW;
            float v = ((float)y + 0.5f) / (float)sunH;
            F3 rd = equal_area_cone_dir(sunDir, u, v, cosMax);
            F3 c = sun_radiance(*this, rd, sunDir) * brightness;
            c = max3f(c, F3(0.0f));
            size_t i = (size_t)sunW * y + x;
            sun[i * 4 + 0] = c.x; sun[i * 4 + 1] = c.y; sun[i * 4 + 2] = c.z; sun[i * 4 + 3] = 0.0f;
            sunPdf[i] = luminance(c);
        }
    sunAlias = build_alias(sunPdf, sunSum);
}

}  // namespace orc
