// vxpt -- spectral sky / sun precompute on gfx950.
// Behaviour of renderer/sky/Sky.cu:133-327 (Hosek-style 10-channel fit,
// limb-darkened sun).  Runs once per sky change; the 1024x512 map and the
// 32x32 sun map stay resident in HBM (8 MiB + 16 KiB) for the trace kernel.
#include "vx_internal.hpp"

namespace vx {
namespace {

__constant__ float cCieX[10] = {2.372527e-02f, 1.955480e+00f, 1.074553e+01f, 5.056697e+00f, 4.698190e+00f,
                                2.391135e+01f, 3.798705e+01f, 1.929414e+01f, 2.970610e+00f, 2.092986e-01f};
__constant__ float cCieY[10] = {6.813859e-04f, 6.771017e-02f, 1.171193e+00f, 6.997765e+00f, 2.666710e+01f,
                                3.758372e+01f, 2.503930e+01f, 8.150395e+00f, 1.098635e+00f, 7.563256e-02f};
__constant__ float cCieZ[10] = {1.119121e-01f, 9.441195e+00f, 5.597921e+01f, 3.589996e+01f, 5.070894e+00f,
                                3.523189e-01f, 3.422707e-02f, 2.539118e-03f, 7.836666e-06f, 0.000000e+00f};

VX_D V3 cie(int c) { return V3(cCieX[c], cCieY[c], cCieZ[c]) / 106.856895f; }
VX_D V3 xyz_to_srgb(V3 v) {
    const M3 m = m3_rows(3.2404542f, -1.5371385f, -0.4985314f, -0.9692660f, 1.8760108f, 0.0415560f, 0.0556434f,
                         -0.2040259f, 1.0572252f);
    return m3_apply(m, v);
}

struct SkyConsts { float cfg[90]; float rad[10]; };

VX_D V3 sky_radiance(const SkyConsts &s, V3 rd, V3 sunDir) {
    float theta = acosf(rd.y);
    float gamma = acosf(clampf(dot(rd, sunDir), -1, 1));
    V3 xyz(0.0f);
    for (int ch = 0; ch < 10; ++ch) {
        const float *c = s.cfg + ch * 9;
        const float cg = cosf(gamma);
        const float expM = expf(c[4] * gamma);
        const float rayM = cg * cg;
        const float mieM = (1.0f + cg * cg) / powf((1.0f + c[8] * c[8] - 2.0f * c[8] * cg), 1.5f);
        const float ct = cosf(theta);
        const float zenith = sqrtf(ct);
        // the reference's `cos(theta) + 0.01` promotes this factor to binary64
        const double f1 = 1.0f + (double)c[0] * exp((double)c[1] / ((double)ct + 0.01));
        const float f2 = c[2] + c[3] * expM + c[5] * rayM + c[6] * mieM + c[7] * zenith;
        const float radiance = (float)(f1 * (double)f2) * s.rad[ch];
        xyz += radiance * cie(ch);
    }
    return xyz_to_srgb(xyz);
}

VX_D V3 sun_radiance(const float *solar, const float *limb, V3 rd, V3 sunDir) {
    float gamma = acosf(clampf(dot(rd, sunDir), -1, 1));
    float elevation = (kPi / 2.0f) - acosf(sunDir.y);
    const float sunAngle = 0.51f;
    const float solarRadius = sunAngle * kPi / 180.0f / 2.0f;
    const float scale = 1.0f / ((sunAngle / 0.51f) * (sunAngle / 0.51f));
    float srs = sinf(solarRadius);
    float ar2 = 1.0f / (srs * srs);
    float sg = sinf(gamma);
    float sc2 = 1.0f - ar2 * sg * sg;
    if (sc2 < 0.0f) sc2 = 0.0f;
    float sampleCos = sqrtf(sc2);
    if (sampleCos == 0.0f) return V3(0.0f);
    int pos = (int)(powf((float)(2.0 * (double)elevation / (double)kPi), (float)(1.0 / 3.0)) * 45);
    if (pos > 44) pos = 44;
    const float breakX = (float)((double)powf(((float)pos / 45.0f), 3.0f) * ((double)kPi * 0.5));
    const float x = elevation - breakX;
    V3 xyz(0.0f);
    for (int ch = 0; ch < 10; ++ch) {
        const float *coefs = solar + ch * 180 + (4 * (pos + 1) - 1);
        float res = 0.0f, xe = 1.0f;
        for (int i = 0; i < 4; ++i) {
            res += xe * coefs[-i];
            xe *= x;
        }
        const float *ld = limb + ch * 6;
        float dark = ld[0] + ld[1] * sampleCos + ld[2] * powf(sampleCos, 2.0f) + ld[3] * powf(sampleCos, 3.0f) +
                     ld[4] * powf(sampleCos, 4.0f) + ld[5] * powf(sampleCos, 5.0f);
        float direct = res;
        direct *= dark * scale;
        xyz += direct * cie(ch);
    }
    return xyz_to_srgb(xyz);
}

__global__ __launch_bounds__(256) void k_sky_upper(SkyConsts s, V3 sunDir, float brightness, float4 *sky,
                                                    float *pdf, int W, int H) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int half = H / 2;
    if (x >= W || y >= half) return;
    const float u = ((float)x + 0.5f) / (float)W;
    const float v = ((float)y + 0.5f) / (float)half;
    const float r = sqrtf(1.0f - v * v);
    const float phi = kTwoPi * u;
    const V3 rd(r * cosf(phi), v, r * sinf(phi));  // EqualAreaHemisphereMap
    V3 c = sky_radiance(s, rd, sunDir) * brightness;
    c = max3(c, V3(0.0f));
    const size_t i = (size_t)W * (y + half) + x;
    sky[i] = make_float4(c.x, c.y, c.z, 0.0f);
    pdf[i] = luminance(c);
}

__global__ __launch_bounds__(256) void k_sun(const float *solar, const float *limb, V3 sunDir, float brightness,
                                             float4 *sun, float *pdf, int W, int H) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= W * H) return;
    const int x = i % W, y = i / W;
    const float u = ((float)x + 0.5f) / (float)W, v = ((float)y + 0.5f) / (float)H;
    const V3 rd = eq_area_cone_dir(sunDir, u, v, cosf(0.51f * kPi / 180.0f / 2.0f));
    V3 c = sun_radiance(solar, limb, rd, sunDir) * brightness;
    c = max3(c, V3(0.0f));
    sun[i] = make_float4(c.x, c.y, c.z, 0.0f);
    pdf[i] = luminance(c);
}

__global__ __launch_bounds__(256) void k_sky_lower(float4 *sky, float *pdf, int W, int H, float sumUpper) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int half = H / 2;
    if (x >= W || y >= half) return;
    const float v = ((float)y + 0.5f) / (float)half - 1.0f;
    const V3 mist(sumUpper / (float)(W * H));
    const float blend = clampf((v + 0.4f) * (1.0f / 0.5f));
    const float4 e = sky[(size_t)W * half + x];
    const V3 em(e.x, e.y, e.z);
    const V3 c = mist + (blend * blend * (3.0f - 2.0f * blend)) * (em - mist);  // smoothstep3f
    const size_t i = (size_t)W * y + x;
    sky[i] = make_float4(c.x, c.y, c.z, 0.0f);
    pdf[i] = luminance(c);
}

}  // namespace

hipError_t launch_sky(const float *cfg90, const float *rad10, const float *solar, const float *limb, V3 sunDir,
                      float brightness, float4 *sky, float4 *sun, float *skyPdf, float *sunPdf, int skyW, int skyH,
                      int sunW, int sunH, hipStream_t st) {
    SkyConsts s;
    for (int i = 0; i < 90; ++i) s.cfg[i] = cfg90[i];
    for (int i = 0; i < 10; ++i) s.rad[i] = rad10[i];
    dim3 g((skyW + 63) / 64, (skyH / 2 + 3) / 4);
    hipLaunchKernelGGL(k_sky_upper, g, dim3(256), 0, st, s, sunDir, brightness, sky, skyPdf, skyW, skyH);
    hipLaunchKernelGGL(k_sun, dim3((sunW * sunH + 255) / 256), dim3(256), 0, st, solar, limb, sunDir, brightness, sun,
                       sunPdf, sunW, sunH);
    return hipGetLastError();
}

hipError_t launch_sky_lower(float4 *sky, float *skyPdf, int skyW, int skyH, float sumUpper, hipStream_t st) {
    dim3 g((skyW + 63) / 64, (skyH / 2 + 3) / 4);
    hipLaunchKernelGGL(k_sky_lower, g, dim3(256), 0, st, sky, skyPdf, skyW, skyH, sumUpper);
    return hipGetLastError();
}

}  // namespace vx
