// ORACLE (test infrastructure only): restatement of the per-pixel path loop
// renderer/shaders/RayGen.cu, hit/miss programs closesthit.cu / miss.cu,
// Disney BSDF (Bsdf.h:371-617), ReSTIR-DI (Restir.h), with the OptiX traversal
// replaced by the voxel DDA contract (orc_scene.h).
#include "orc_trace.h"

#include <cmath>
#include <utility>

namespace orc {

void Frame::alloc(int w, int h) {
    W = w; H = h;
    size_t n = (size_t)w * h;
    for (auto *v : {&illum, &normalRough, &geoNormalThin, &albedo, &matParam, &motion, &prevNormalRough,
                    &prevGeoNormalThin, &prevAlbedo, &prevMatParam, &ping, &pong, &prevIllum, &prevFast, &output})
        v->assign(n, F4(0.0f));
    for (auto *v : {&depth, &material, &prevDepth, &prevMaterial, &histLen, &prevHistLen, &clampBits}) v->assign(n, 0.0f);
    reservoir.assign(2 * n, Reservoir{});
}

namespace {

constexpr uint32_t kValidBit = 0x80000000u, kIndexMask = 0x7FFFFFFFu;
constexpr uint32_t kInvalidLight = 0x7FFFFFFFu, kSkyLight = 0x7FFFFFFEu, kSunLight = 0x7FFFFFFDu;
enum { LtInvalid = 0, LtSky = 1, LtSun = 2, LtLocal = 3 };
constexpr float kRoughThresh = 0.00001f, kTranslThresh = 0.001f;
constexpr float kMinPdf = 1e-5f, kMaxThroughput = 32.0f, kMinLobe = 0.05f;

struct LightSample { F3 position, radiance; float solidAnglePdf = 0; int type = LtInvalid; };
struct State { F3 normal, geoNormal, albedo, wo; float roughness = 0; bool metallic = false; float translucency = 0; };
struct Surf { F3 pos; float depth = 0; bool thin = false; int materialId = 0; State st; };

// ------------------------------------------------------------ Disney BSDF
F3 clamp_throughput(const F3 &v) {  // Bsdf.h:12-22
    float l = luminance(v), a = std::fabs(l);
    if (a > kMaxThroughput && a > 0.0f) return v * (kMaxThroughput / a);
    return v;
}
float disney_diffuse_fresnel(float cwo, float cwi, float r) {
    float energyBias = lerpf(0.0f, 0.5f, r);
    float energyFactor = lerpf(1.0f, 1.0f / 1.51f, r);
    float fd90 = energyBias + 2.0f * r * cwi * cwi;
    float f0 = 1.0f;
    float ls = f0 + (fd90 - f0) * pow5(1.0f - cwo);
    float vs = f0 + (fd90 - f0) * pow5(1.0f - cwi);
    return ls * vs * energyFactor;
}
float gtr2(float ch, float sh, float sp, float cp, float ax, float ay) {
    float ax2 = ax * ax, ay2 = ay * ay;
    float s = (cp * cp) / ax2 + (sp * sp) / ay2;
    float t = sh * sh * s + ch * ch;
    return 1.0f / (kPi * ax * ay * t * t);
}
float smith_g(float c, float a) {
    float a2 = a * a, c2 = c * c;
    return 2.0f / (1.0f + std::sqrt(1.0f + a2 * (1.0f - c2) / c2));
}
void spec_reflect_sample(const F3 &n, const F3 &ng, const F3 &wo, const F3 &albedo, F3 &wi, F3 &bop, float &pdf) {
    wi = reflect3f(-wo, n);
    if (dot(wi, n) <= 0.0f || dot(wi, ng) <= 0.0f) { bop = F3(0.0f); pdf = 0.0f; return; }
    bop = albedo; pdf = 1.0f;
}
float fresnel_dielectric(float et, float cosIn) {
    const float cosi = std::fabs(cosIn);
    float sint = 1.0f - cosi * cosi;
    sint = (0.0f < sint) ? std::sqrt(sint) / et : 0.0f;
    if (1.0f < sint) return 1.0f;
    float cost = 1.0f - sint * sint;
    cost = (0.0f < cost) ? std::sqrt(cost) : 0.0f;
    const float ec = et * cosi, et2 = et * cost;
    const float rPerp = (cosi - et2) / (cosi + et2);
    const float rPar = (ec - cost) / (ec + cost);
    const float r = (rPar * rPar + rPerp * rPerp) * 0.5f;
    return r <= 1.0f ? r : 1.0f;
}
bool refract3(F3 &r, const F3 &i, const F3 &n, float ior) {  // LinearMath.h:1483-1513
    F3 nn = n;
    float neg = dot(i, nn), eta;
    if (neg > 0.0f) { eta = ior; nn = -n; neg = -neg; } else eta = 1.f / ior;
    const float k = 1.f - eta * eta * (1.f - neg * neg);
    if (k < 0.0f) { r = F3(0.f); return false; }
    r = normalize(eta * i - (eta * neg + std::sqrt(k)) * nn);
    return true;
}
void spec_refl_trans_sample(float u, const F3 &n, const F3 &ng, const F3 &wo, const F3 &albedo, F3 &wi, F3 &bop,
                            float &pdf, bool &trans) {
    const float ior = 1.4f;
    const bool front = dot(wo, ng) > 0.0f;
    const float eta = front ? ior / 1.0f : 1.0f / ior;
    F3 wr = reflect3f(-wo, n), wt;
    float R = 1.0f;
    if (refract3(wt, -wo, n, eta)) R = fresnel_dielectric(eta, dot(wo, n));
    if (u <= R) { wi = wr; pdf = R; } else { wi = wt; pdf = 1.0f - R; trans = true; }
    bop = albedo / pdf;
}

void disney_sample(const F4 &u, const F3 &n, const F3 &ng, const F3 &wo, const F3 &albedo, bool metallic,
                   float translucency, float roughness, F3 &wi, F3 &bop, float &pdf, bool &trans) {
    if (roughness < kRoughThresh) {  // Bsdf.h:403-425
        trans = false;
        if (translucency < kTranslThresh) {
            spec_reflect_sample(n, ng, wo, albedo, wi, bop, pdf);
            pdf = std::fmax(pdf, kMinPdf);
            bop = clamp_throughput(bop);
        } else if (translucency > 1.0f - kTranslThresh) {
            spec_refl_trans_sample(u.x, n, ng, wo, albedo, wi, bop, pdf, trans);
            pdf = std::fmax(pdf, kMinPdf);
            bop = clamp_throughput(bop);
        } else {
            bop = F3(0.0f); pdf = 0.0f;
        }
        return;
    }
    trans = false;
    const float specParam = 0.5f;
    const float metalness = metallic ? 1.0f : 0.0f;
    float alpha = std::fmax(roughness * roughness, kRoughThresh);
    float cwo = std::fmax(kSafeCos, dot(n, wo));
    float lum = 0.299f * albedo.x + 0.587f * albedo.y + 0.114f * albedo.z;
    F3 tint = lum > 0.0f ? albedo / lum : F3(1.0f);
    F3 specColor = lerp3(F3(1.0f), tint, 0.0f);
    F3 C0 = lerp3(0.08f * specParam * specColor, albedo, metalness);
    F3 F = C0 + (F3(1.0f) - C0) * pow5(1.0f - cwo);
    float avgF = (F.x + F.y + F.z) / 3.0f;
    float sw = avgF, dw = (1.0f - metalness) * (1.0f - avgF), tw = sw + dw;
    if (tw < kSafeCos) { bop = F3(0.0f); pdf = 0.0f; return; }
    float sp = sw / tw;
    if (dw > kSafeCos && sw > kSafeCos) sp = clampf(sp, kMinLobe, 1.0f - kMinLobe);
    sp = clampf(sp, 0.0f, 1.0f);
    float dp = std::fmax(0.0f, 1.0f - sp);
    if (u.w < sp) {
        float ct = std::sqrt((1.0f - u.x) / (1.0f + (alpha * alpha - 1.0f) * u.x));
        ct = clampf(ct, kSafeCos, 1.0f);
        float st = std::sqrt(std::fmax(0.0f, 1.0f - ct * ct));
        float phi = kTwoPi * u.y;
        F3 wh(st * std::cos(phi), st * std::sin(phi), ct);
        align_vector(n, wh);
        wi = normalize(reflect3f(-wo, wh));
        if (dot(wi, n) <= 0.0f || dot(wi, ng) <= 0.0f) { bop = F3(0.0f); pdf = 0.0f; return; }
        float cwi = dot(wi, n);
        float cwh = std::fmax(kSafeCos, std::fabs(dot(wh, n)));
        float cwowh = std::fmax(kSafeCos, std::fabs(dot(wo, wh)));
        float swh = std::sqrt(std::fmax(0.0f, 1.0f - cwh * cwh));
        float D = gtr2(cwh, swh, 0.0f, 1.0f, alpha, alpha);
        F3 Fs = C0 + (F3(1.0f) - C0) * pow5(1.0f - cwowh);
        float G = smith_g(cwo, alpha) * smith_g(cwi, alpha);
        F3 brdf = Fs * D * G / (4.0f * cwo * cwi);
        float mpdf = D * cwh / (4.0f * cwowh);
        mpdf = std::fmax(mpdf, kMinPdf);
        float wsp = std::fmax(sp, kMinPdf);
        pdf = mpdf * wsp;
        pdf = std::fmax(pdf, kMinPdf);
        bop = clamp_throughput(brdf * cwi / pdf);
    } else {
        float ct = std::sqrt(u.x);
        float st = std::sqrt(std::fmax(0.0f, 1.0f - ct * ct));
        float phi = kTwoPi * u.y;
        wi = F3(st * std::cos(phi), st * std::sin(phi), ct);
        align_vector(n, wi);
        if (dot(wi, ng) <= 0.0f) { bop = F3(0.0f); pdf = 0.0f; return; }
        float cwi = std::fmax(kSafeCos, dot(wi, n));
        float fl = disney_diffuse_fresnel(cwo, cwi, roughness);
        F3 db = albedo * (1.0f - metalness) * fl / kPi;
        float dpdf = cwi / kPi;
        dpdf = std::fmax(dpdf, kMinPdf);
        float wdp = std::fmax(dp, kMinPdf);
        pdf = dpdf * wdp;
        pdf = std::fmax(pdf, kMinPdf);
        bop = clamp_throughput(db * cwi / pdf);
    }
}

void disney_eval(const F3 &n, const F3 &ng, const F3 &wi, const F3 &wo, const F3 &albedo, bool metallic,
                 float /*translucency*/, float roughness, F3 &bsdf, float &pdf) {  // Bsdf.h:539-617
    bsdf = F3(0.0f);
    if (roughness < kRoughThresh) { pdf = 0.0f; return; }
    if (dot(wo, n) <= 0.0f || dot(wi, n) <= 0.0f || dot(wo, ng) <= 0.0f || dot(wi, ng) <= 0.0f) { pdf = 0.0f; return; }
    const float specParam = 0.5f;
    const float metalness = metallic ? 1.0f : 0.0f;
    float alpha = std::fmax(roughness * roughness, kRoughThresh);
    float cwo = dot(wo, n), cwi = dot(wi, n);
    F3 wh = normalize(wi + wo);
    float cwh = std::fmax(kSafeCos, std::fabs(dot(wh, n)));
    float cwowh = std::fmax(kSafeCos, std::fabs(dot(wo, wh)));
    float lum = 0.299f * albedo.x + 0.587f * albedo.y + 0.114f * albedo.z;
    F3 tint = lum > 0.0f ? albedo / lum : F3(1.0f);
    F3 specColor = lerp3(F3(1.0f), tint, 0.0f);
    F3 C0 = lerp3(0.08f * specParam * specColor, albedo, metalness);
    F3 F = C0 + (F3(1.0f) - C0) * pow5(1.0f - cwowh);
    F3 diffuse(0.0f);
    if (!metallic) {
        float fl = disney_diffuse_fresnel(cwo, cwi, roughness);
        diffuse = albedo * (1.0f - metalness) * fl / kPi;
    }
    float s2 = std::fmax(0.0f, 1.0f - cwh * cwh);
    float swh = std::sqrt(s2);
    float D = gtr2(cwh, swh, 0.0f, 1.0f, alpha, alpha);
    float G = smith_g(cwo, alpha) * smith_g(cwi, alpha);
    F3 spec = F * D * G / (4.0f * cwo * cwi);
    bsdf = clamp_throughput(diffuse + spec);
    float avgF = (F.x + F.y + F.z) / 3.0f;
    float sw = avgF, dw = (1.0f - metalness) * (1.0f - avgF), tw = sw + dw;
    if (tw < kSafeCos) { pdf = 0.0f; return; }
    float sp = sw / tw;
    if (dw > kSafeCos && sw > kSafeCos) sp = clampf(sp, kMinLobe, 1.0f - kMinLobe);
    sp = clampf(sp, 0.0f, 1.0f);
    float dp = std::fmax(0.0f, 1.0f - sp);
    float dpdf = std::fmax(cwi / kPi, kMinPdf);
    float spdf = std::fmax(D * cwh / (4.0f * cwowh), kMinPdf);
    float wsp = std::fmax(sp, kMinPdf), wdp = std::fmax(dp, kMinPdf);
    pdf = dpdf * wdp + spdf * wsp;
    pdf = std::fmax(pdf, kMinPdf);
}

// ------------------------------------------------------------ per-pixel ctx
struct Px {
    const Scene &s;
    Frame &f;
    int px, py, it;
    int randIdx = 0;
    float rnd() { return s.bn.rand(px, py, it, randIdx++); }
    F2 rnd2() { float a = rnd(); float b = rnd(); return F2(a, b); }  // left-to-right argument order
    F4 rnd4() { float a = rnd(), b = rnd(), c = rnd(), d = rnd(); return F4(a, b, c, d); }
    float rnd16() { F2 u = rnd2(); return u.x + u.y / 256.0f; }
    size_t idx() const { return (size_t)py * f.W + px; }
};

const float kSunCosMax() { static const float v = std::cos(0.51f * kPi / 180.0f / 2.0f); return v; }

F3 load_sky(const Sky &k, int x, int y) {
    size_t i = (size_t)y * k.skyW + x;
    return F3(k.sky[i * 4], k.sky[i * 4 + 1], k.sky[i * 4 + 2]);
}
F3 load_sun(const Sky &k, int x, int y) {
    x = clampi(x, 0, k.sunW - 1); y = clampi(y, 0, k.sunH - 1);  // surface clamp
    size_t i = (size_t)y * k.sunW + x;
    return F3(k.sun[i * 4], k.sun[i * 4 + 1], k.sun[i * 4 + 2]);
}

LightSample sun_sample(const Scene &s, int idx) {  // Restir.h:221-253
    const Sky &k = s.sky;
    int sx = idx % k.sunW, sy = idx / k.sunW;
    F2 uv((sx + 0.5f) / float(k.sunW), (sy + 0.5f) / float(k.sunH));
    const float cm = kSunCosMax();
    LightSample ls;
    ls.solidAnglePdf = (k.sunW * k.sunH) / (kTwoPi * (1.0f - cm));
    ls.position = equal_area_cone_dir(k.sunDir, uv.x, uv.y, cm);
    ls.radiance = load_sun(k, sx, sy);
    ls.type = LtSun;
    return ls;
}
LightSample sky_sample(const Scene &s, int idx) {  // Restir.h:256-283
    const Sky &k = s.sky;
    int sx = idx % k.skyW, sy = idx / k.skyW;
    F2 uv((sx + 0.5f) / float(k.skyW), (sy + 0.5f) / float(k.skyH));
    LightSample ls;
    ls.solidAnglePdf = (k.skyW * k.skyH) / (4.0f * kPi);
    ls.position = equal_area_sphere_dir(uv.x, uv.y);
    ls.radiance = load_sky(k, sx, sy);
    ls.type = LtSky;
    return ls;
}

// TriangleLight::calcSample (Light.h:54-82): SampleTriangle (LinearMath.h:2048-2056), PdfAtoW
LightSample tri_sample(const TriLight &t, F2 uv, const F3 &viewer) {
    const float sx = std::sqrt(uv.x);
    const F3 bary(1.0f - sx, sx * (1.0f - uv.y), sx * uv.y);
    LightSample r;
    r.position = t.base + t.edge1 * bary.y + t.edge2 * bary.z;
    F3 L = r.position - viewer;
    const float Ld = length(L);
    L /= Ld;
    const float areaPdf = 1.0f / t.area;
    const float cosT = saturate(dot(L, -t.normal));
    r.solidAnglePdf = areaPdf * (Ld * Ld) / cosT;
    r.radiance = t.radiance;
    r.type = LtLocal;
    return r;
}
F2 inverse_tri_sample(float u, float v) {  // InverseTriangleSample (LinearMath.h:2059-2064)
    const F3 b(1.0f - u - v, u, v);
    const float sx = 1 - b.x;
    return F2(sx * sx, b.z / sx);
}
// the direction a light sample is seen in from p (closesthit.cu:610, 738, 794, 829)
F3 light_dir(const LightSample &ls, const F3 &p) { return ls.type == LtLocal ? normalize(ls.position - p) : ls.position; }

float target_pdf(const LightSample &ls, const Surf &sf) {  // Restir.h:194-211
    if (ls.solidAnglePdf <= 0 || ls.type == LtInvalid) return 0.0f;
    F3 wi = light_dir(ls, sf.pos);
    F3 fr; float pdf;
    disney_eval(sf.st.normal, sf.st.geoNormal, wi, sf.st.wo, sf.st.albedo, sf.st.metallic, sf.st.translucency,
                sf.st.roughness, fr, pdf);
    F3 refl = ls.radiance * fr * std::fabs(dot(wi, sf.st.normal)) / ls.solidAnglePdf;
    return luminance(refl);
}

float brdf_pdf(const Surf &sf, const F3 &wi) {
    F3 fr; float pdf;
    disney_eval(sf.st.normal, sf.st.geoNormal, wi, sf.st.wo, sf.st.albedo, sf.st.metallic, sf.st.translucency,
                sf.st.roughness, fr, pdf);
    return pdf;
}

float mis_weight(const Surf &sf, const LightSample &ls, float selPdf, float lightMis, bool env, float brdfMis) {
    float sa = ls.solidAnglePdf;  // Restir.h:286-328, brdfCutoff == 0
    if (brdfMis == 0.0f || sa <= 0.0f || std::isinf(sa) || std::isnan(sa)) return lightMis * selPdf;
    F3 dir = ls.position;
    if (ls.type == LtLocal) {
        const F3 toLight = ls.position - sf.pos;
        const float dist = length(toLight);
        dir = toLight / dist;
    }
    float bp = brdf_pdf(sf, dir);  // brdfCutoff 0: the distance test never drops it
    (void)env;
    float src = selPdf * sa;
    float blended = lightMis * src + brdfMis * bp;
    return blended / sa;
}

bool stream_sample(Reservoir &r, uint32_t light, F2 uv, float rnd, float target, float invSrc) {
    float w = target * invSrc;
    r.M += 1;
    r.weightSum += w;
    bool sel = (rnd * r.weightSum < w);
    if (sel) {
        r.lightData = light | kValidBit;
        r.uvData = (uint32_t)(saturate(uv.x) * 0xffff) | ((uint32_t)(saturate(uv.y) * 0xffff) << 16);
        r.targetPdf = target;
    }
    return sel;
}
bool combine(Reservoir &r, const Reservoir &n, float rnd, float target) {  // Restir.h:114-161
    float w = target * (n.weightSum * n.M);
    r.M += n.M;
    r.weightSum += w;
    bool sel = (rnd * r.weightSum < w);
    if (sel) { r.lightData = n.lightData; r.uvData = n.uvData; r.targetPdf = target; }
    return sel;
}
void finalize(Reservoir &r, float num, float den) {
    float d = r.targetPdf * den;
    r.weightSum = (d == 0.0f) ? 0.0f : (r.weightSum * num) / d;
}

bool light_from_reservoir(const Scene &s, LightSample &ls, const Reservoir &r, const Surf &sf,
                          bool hasLocal) {  // Restir.h:383-415
    uint32_t li = r.lightData & kIndexMask;
    F2 uv = F2((float)(r.uvData & 0xffff), (float)(r.uvData >> 16)) / float(0xffff);
    const Sky &k = s.sky;
    if (li == kSkyLight) {
        int x = clampi(int(uv.x * k.skyW), 0, k.skyW - 1), y = clampi(int(uv.y * k.skyH), 0, k.skyH - 1);
        ls = sky_sample(s, y * k.skyW + x);
    } else if (li == kSunLight) {
        int x = clampi(int(uv.x * k.sunW), 0, k.sunW - 1), y = clampi(int(uv.y * k.sunH), 0, k.sunH - 1);
        ls = sun_sample(s, y * k.sunW + x);
    } else if (hasLocal && li < (uint32_t)s.mesh.numLights) {
        ls = tri_sample(tri_light(s.mesh, (int)li), uv, sf.pos);
        return true;
    }
    return li < kInvalidLight;
}

int reflect_into_view(int p, int n) {  // ClampSamplePositionIntoView (Restir.h:330-346)
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - p - 1;
    return p;
}

bool prev_surface(Px &c, Surf &sf, int x, int y) {  // GetPrevSurface (Restir.h:348-381)
    const Camera &pc = c.s.prevCam;
    if (x < 0 || y < 0 || x >= (int)pc.res.x || y >= (int)pc.res.y) return false;
    size_t i = (size_t)y * c.f.W + x;
    sf.depth = c.f.prevDepth[i];
    if (sf.depth == kRayMax) return false;
    F4 nr = c.f.prevNormalRough[i], gt = c.f.prevGeoNormalThin[i], mp = c.f.prevMatParam[i];
    float mat = c.f.prevMaterial[i];
    // randPrev uses the *current* pixel's launch index and iterationIndex-1
    float j0 = c.s.bn.rand(c.px, c.py, c.it - 1, 0), j1 = c.s.bn.rand(c.px, c.py, c.it - 1, 1);
    F2 uv = (F2((float)x, (float)y) + F2(j0, j1)) * pc.invRes;
    F3 vd = pc.uv_to_dir(uv);
    sf.pos = pc.pos + vd * sf.depth;
    sf.thin = (gt.w == 1.0f);
    sf.materialId = (int)mat;
    sf.st.wo = -vd;
    sf.st.normal = nr.xyz();
    sf.st.geoNormal = gt.xyz();
    sf.st.albedo = c.f.prevAlbedo[i].xyz();
    sf.st.roughness = nr.w;
    sf.st.metallic = (mp.x == 1.0f);
    sf.st.translucency = mp.y;
    return true;
}

struct Ray {
    F3 pos, wo, wi, radiance, bsdfOverPdf;
    float distance = kRayMax, pdf = 0;
    float travelled = 0;  // sum of hit distances: ray cone width = spread * travelled (closesthit.cu:195)
    unsigned depth = 0;
    bool hitFirstDiffuse = false, terminate = false, curDiffuse = false, lastDiffuse = false;
};

void store_reservoir(Px &c, const Reservoir &r) {
    size_t p = c.idx() + (size_t)(c.it % 2) * c.f.W * c.f.H;
    c.f.reservoir[p] = r;
}
// LoadDIReservoir (Restir.h:48-79): in the pass after a light update the previous pass's local-light
// indices go through the update's remap; a light that is gone empties the reservoir.  Taken
// literally: an empty reservoir (lightData 0) reads as index 0 and is remapped as well.
Reservoir load_prev_reservoir(Px &c, int x, int y) {
    size_t p = (size_t)x + (size_t)y * c.f.W + (size_t)((c.it + 1) % 2) * c.f.W * c.f.H;
    Reservoir r = c.f.reservoir[p];
    const Scene &s = c.s;
    if (!s.lightsDirty) return r;
    const uint32_t li = r.lightData & 0x7FFFFFFFu;
    if (li >= 0x7FFFFFFDu) return r;  // sun / sky: unchanged
    if (s.prevNumLights > 0 && li < (uint32_t)s.prevNumLights) {
        const int cur = s.lightRemap[li];
        if (cur < 0 || cur >= s.mesh.numLights) return Reservoir{};
        r.lightData = (r.lightData & 0x80000000u) | (uint32_t)cur;
    }
    return r;
}

// Closest hit over the voxel faces and the instanced meshes (one IAS in the reference): a mesh
// hit replaces the voxel hit only when strictly closer (ties go to the voxel face).
struct AnyHit { Hit vox; MeshHit mesh; bool isMesh = false, hit = false; float t = kRayMax; };
AnyHit closest_any(const Scene &s, const F3 &o, const F3 &d, float tmax) {
    AnyHit a;
    a.vox = dda_closest(s.world, o, d, tmax);
    a.hit = a.vox.hit;
    a.t = a.vox.hit ? a.vox.t : kRayMax;
    if (!s.mesh.inst.empty()) {
        const MeshHit m = mesh_closest_hit(s.mesh, o, d, a.vox.hit ? a.vox.t : tmax);
        if (m.hit && (!a.vox.hit || m.t < a.vox.t)) { a.mesh = m; a.isMesh = true; a.hit = true; a.t = m.t; }
    }
    return a;
}
// visibility (mask 0xFE: every voxel face and every mesh triangle, either side)
bool occluded_any(const Scene &s, const F3 &o, const F3 &d, float tmin, float tmax) {
    if (dda_occluded(s.world, o, d, tmin, tmax)) return true;
    return !s.mesh.inst.empty() && mesh_any_hit(s.mesh, o, d, tmin, tmax);
}
// a visibility ray toward a light sample (closesthit.cu:606-633): local lights stop 0.01 short
bool light_occluded(const Scene &s, const F3 &org, const LightSample &ls, const F3 &p, float extra) {
    const F3 sd = light_dir(ls, p);
    const float tmax = ls.type == LtLocal ? length(ls.position - p) - 0.01f - extra : kRayMax;
    return occluded_any(s, org, sd, extra, tmax);
}

void on_miss(Px &c, Ray &rd) {  // miss.cu:9-82
    const Sky &k = c.s.sky;
    if (rd.depth == 0) {
        store_reservoir(c, Reservoir{});
        size_t i = c.idx();
        c.f.albedo[i] = F4(1.0f);
        c.f.material[i] = (float)0xFFFF;
        c.f.normalRough[i] = F4(0.0f, -1.0f, 0.0f, 0.0f);
        c.f.geoNormalThin[i] = F4(0.0f, -1.0f, 0.0f, 0.0f);
        c.f.matParam[i] = F4(0.0f);
    }
    F3 emission(0);
    F2 uv = equal_area_sphere_uv(rd.wi);
    {  // SampleBicubicSmoothStep + BoundaryFuncRepeatXClampY (Sampler.h:653-698, 255-280)
        F2 UV(uv.x * (float)k.skyW, uv.y * (float)k.skyH);
        F2 tc(std::floor(UV.x - 0.5f) + 0.5f, std::floor(UV.y - 0.5f) + 0.5f);
        F2 fr = UV - tc;
        F2 f2 = fr * fr, f3 = f2 * fr;
        F2 w1 = -2.0f * f3 + 3.0f * f2;
        F2 w0 = 1.0f - w1;
        int tx0 = (int)std::floor(UV.x - 0.5f), ty0 = (int)std::floor(UV.y - 0.5f);
        int sx[4] = {tx0, tx0 + 1, tx0, tx0 + 1}, sy[4] = {ty0, ty0, ty0 + 1, ty0 + 1};
        float wt[4] = {w0.x * w0.y, w1.x * w0.y, w0.x * w1.y, w1.x * w1.y};
        F3 out(0.0f);
        float sum = 0;
        for (int i = 0; i < 4; ++i) {
            int x = sx[i], y = sy[i];
            if (x >= k.skyW) x %= k.skyW;
            if (x < 0) x = k.skyW - (-x) % k.skyW;
            if (y >= k.skyH) y = k.skyH - 1;
            if (y < 0) y = 0;
            sum += wt[i];
            out += load_sky(k, x, y) * wt[i];
        }
        out /= sum;
        emission += out;
    }
    if (equal_area_cone_uv(uv, k.sunDir, rd.wi, kSunCosMax())) {
        int x = (int)(uv.x * k.sunW), y = (int)(uv.y * k.sunH);
        if (x >= k.sunW) x %= k.sunW;
        if (x < 0) x = k.sunW - (-x) % k.sunW;
        emission += load_sun(k, x, y);
    }
    rd.radiance = emission;
    rd.distance = kRayMax;
    rd.terminate = true;
}

// tex2DLod on an RGBA8 mip chain (TextureManager.cu:228-246: wrap, linear, linear mip, unorm,
// lod clamped to [0, maxLod]) with float filter weights
struct TexSample { float r, g, b, a; };
TexSample texel(const Scene &s, const Texture &t, int l, int x, int y) {
    const int S = t.size >> l;
    const uint8_t *p = s.texels.data() + 4 * ((size_t)t.off[l] + (size_t)(y * S + x));
    return {p[0] / 255.0f, p[1] / 255.0f, p[2] / 255.0f, p[3] / 255.0f};
}
int wrap_i(int i, int S) {
    const int m = i % S;
    return m < 0 ? m + S : m;
}
TexSample tex_bilinear(const Scene &s, const Texture &t, int l, float u, float v) {
    const int S = t.size >> l;
    const float x = u * (float)S - 0.5f, y = v * (float)S - 0.5f;
    const float fx = std::floor(x), fy = std::floor(y);
    const float ax = x - fx, ay = y - fy;
    const int x0 = wrap_i((int)fx, S), x1 = wrap_i((int)fx + 1, S), y0 = wrap_i((int)fy, S), y1 = wrap_i((int)fy + 1, S);
    const TexSample a = texel(s, t, l, x0, y0), b = texel(s, t, l, x1, y0), c = texel(s, t, l, x0, y1),
                    d = texel(s, t, l, x1, y1);
    const float w00 = (1.0f - ax) * (1.0f - ay), w10 = ax * (1.0f - ay), w01 = (1.0f - ax) * ay, w11 = ax * ay;
    return {a.r * w00 + b.r * w10 + c.r * w01 + d.r * w11, a.g * w00 + b.g * w10 + c.g * w01 + d.g * w11,
            a.b * w00 + b.b * w10 + c.b * w01 + d.b * w11, a.a * w00 + b.a * w10 + c.a * w01 + d.a * w11};
}
TexSample tex_lod(const Scene &s, int id, float u, float v, float lod) {
    const Texture &t = s.textures[id];
    lod = std::fmin(std::fmax(lod, 0.0f), (float)t.maxLod);
    const int l0 = (int)std::floor(lod);
    const float fl = lod - (float)l0;
    const TexSample c0 = tex_bilinear(s, t, l0, u, v);
    if (!(fl > 0.0f)) return c0;
    const TexSample c1 = tex_bilinear(s, t, std::min(l0 + 1, t.maxLod), u, v);
    return {c0.r * (1.0f - fl) + c1.r * fl, c0.g * (1.0f - fl) + c1.g * fl, c0.b * (1.0f - fl) + c1.b * fl,
            c0.a * (1.0f - fl) + c1.a * fl};
}
// Camera::getRayConeWidth (Camera.h:133-149)
float ray_cone_spread(const Camera &cam, int px, int py) {
    const F2 pc = (F2((float)px, (float)py) + 0.5f) - cam.res / 2.0f;
    const F2 po(std::copysign(0.5f, pc.x), std::copysign(0.5f, pc.y));
    const F2 uvN = (pc - po) * cam.invRes * 2.0f, uvF = (pc + po) * cam.invRes * 2.0f;
    const F2 pN = uvN * cam.tanHalfFov, pF = uvF * cam.tanHalfFov;
    return std::atan(std::sqrt(pF.x * pF.x + pF.y * pF.y)) - std::atan(std::sqrt(pN.x * pN.x + pN.y * pN.y));
}

void on_hit(Px &c, Ray &rd, const AnyHit &ah) {  // closesthit.cu:10-852
    const Scene &s = c.s;
    Frame &f = c.f;
    const size_t pi = c.idx();
    rd.distance = ah.t;
    F3 frontPos, backPos, geoNormal;
    int block;
    if (!ah.isMesh) {
        const Hit &h = ah.vox;
        // hit point on the face plane (OptiX barycentric reconstruction is not reproducible)
        F3 hp = rd.pos + rd.wi * h.t;
        const int axis = (h.face < 2) ? 1 : (h.face < 4 ? 0 : 2);
        const int cell = axis == 0 ? h.x : (axis == 1 ? h.y : h.z);
        const bool high = (h.face == 0 || h.face == 3 || h.face == 4);
        hp[axis] = (float)(cell + (high ? 1 : 0));
        safe_spawn(h, hp, frontPos, backPos, geoNormal);
        block = h.id;
    } else {
        mesh_spawn(s.mesh, ah.mesh, frontPos, backPos, geoNormal);
        block = s.mesh.inst[ah.mesh.row].block;
    }
    F3 motionWS = frontPos - frontPos;  // static geometry
    if (rd.depth == 0) f.motion[pi] = F4(motionWS, 0.0f);
    rd.pos = frontPos;
    bool hitFront = dot(rd.wo, geoNormal) > 0.0f;
    const Material &m = s.mats[block];
    if (m.isEmissive) {  // closesthit.cu:107-122
        if (!rd.hitFirstDiffuse) {
            rd.radiance = m.albedo;
            if (rd.depth == 0) {
                f.albedo[pi] = F4(1.0f);
                f.material[pi] = (float)0xFFFF;
                f.normalRough[pi] = F4(0.0f, -1.0f, 0.0f, 0.0f);
                f.geoNormalThin[pi] = F4(0.0f, -1.0f, 0.0f, 0.0f);
                f.matParam[pi] = F4(0.0f);
            }
        }
        rd.terminate = true;
        return;
    }
    if (m.isThinfilm && !hitFront) {  // closesthit.cu:124-133: the normal faces the incoming ray
        geoNormal = -geoNormal;
        hitFront = true;
        std::swap(frontPos, backPos);
    }
    State st;
    st.geoNormal = geoNormal;
    st.wo = rd.wo;
    st.metallic = m.metallic;
    if (!s.textures.empty()) {  // closesthit.cu:167-254
        rd.travelled += ah.t;
        const float cone = ray_cone_spread(s.cam, c.px, c.py) * rd.travelled;
        F2 tc(0.0f, 0.0f);
        const F3 p = rd.pos;  // the front position before the thin-film swap
        if (m.worldGridUV) {
            if (std::fabs(geoNormal.x) > 0.9f) tc = F2(std::fmod(p.z, m.uvScale), std::fmod(p.y, m.uvScale));
            else if (std::fabs(geoNormal.y) > 0.9f) tc = F2(std::fmod(p.x, m.uvScale), std::fmod(p.z, m.uvScale));
            else if (std::fabs(geoNormal.z) > 0.9f) tc = F2(std::fmod(p.x, m.uvScale), std::fmod(p.y, m.uvScale));
        } else if (ah.isMesh) {
            tc = mesh_texcoord(s.mesh, ah.mesh);
        }
        tc = tc / m.uvScale;
        const float mip0 = std::sqrt(1024.0f * 1024.0f + 1024.0f * 1024.0f);
        const float lod = std::log2(cone / mymax(dot(geoNormal, rd.wo), 0.2f) / m.uvScale * 2.0f * mip0) - 3.0f;
        st.albedo = m.albedo;
        if (m.tex[0] >= 0) {
            const TexSample t = tex_lod(s, m.tex[0], tc.x, tc.y, lod);
            st.albedo = st.albedo * F3(t.r, t.g, t.b);
        }
        st.albedo = max3f(st.albedo, F3(0.001f));
        st.roughness = m.roughness;
        if (m.tex[2] >= 0) st.roughness = tex_lod(s, m.tex[2], tc.x, tc.y, lod).r;
        if (m.tex[3] >= 0) st.metallic = tex_lod(s, m.tex[3], tc.x, tc.y, lod).r > 0.5f;
        if (m.tex[1] >= 0) {
            const TexSample t = tex_lod(s, m.tex[1], tc.x, tc.y, lod);
            F3 n = normalize(F3(t.r, t.g, t.b) - 0.5f);
            n.x = -n.x;
            n.y = -n.y;
            align_vector(geoNormal, n);
            st.normal = n;
        } else {
            st.normal = st.geoNormal;
        }
    } else {
        st.albedo = max3f(m.albedo, F3(0.001f));
        st.roughness = m.roughness;
        st.normal = st.geoNormal;
    }
    if (rd.hitFirstDiffuse) st.roughness = mymin(st.roughness * 2.0f + 0.1f, 1.0f);
    bool isDiffuse = st.roughness > kRoughThresh;
    st.translucency = m.translucency;
    st.normal = lerp3(st.geoNormal, st.normal, 0.2f);
    rd.curDiffuse = isDiffuse;
    if (rd.depth == 0) {
        f.material[pi] = (float)m.materialId;
        f.normalRough[pi] = F4(st.normal, st.roughness);
        f.geoNormalThin[pi] = F4(st.normal, m.isThinfilm ? 1.0f : 0.0f);
        f.matParam[pi] = F4(st.metallic ? 1.0f : 0.0f, st.translucency, 0.0f, 0.0f);
    }
    F3 sWi, sBop;
    float sPdf;
    bool trans = false;
    F4 u4 = c.rnd4();
    disney_sample(u4, st.normal, st.geoNormal, st.wo, st.albedo, st.metallic, st.translucency, st.roughness, sWi, sBop,
                  sPdf, trans);
    if (sPdf <= 0.0f) rd.terminate = true;
    rd.pos = m.isThinfilm ? (dot(sWi, st.normal) > 0.0f ? frontPos : backPos) : frontPos;  // closesthit.cu:288
    rd.wi = sWi;
    rd.bsdfOverPdf = sBop;
    rd.pdf = sPdf;
    bool skipAlbedo = false;
    if (rd.depth == 0) {
        rd.hitFirstDiffuse = true;
        f.albedo[pi] = F4(st.albedo, 1.0f);
        skipAlbedo = true;
    }
    const bool restir = rd.depth == 0;
    if (!isDiffuse) {
        if (restir) store_reservoir(c, Reservoir{});
        return;
    }
    Surf sf;
    sf.st = st;
    sf.materialId = m.materialId;
    sf.pos = rd.pos;
    sf.depth = rd.distance;
    sf.thin = m.isThinfilm;

    const Sky &k = s.sky;
    LightSample lightSample;
    Reservoir ris;
    const bool skipSun = !sf.thin && (dot(st.normal, k.sunDir) < 0.0f || dot(st.geoNormal, k.sunDir) < 0.0f);
    const int nLocal = s.mesh.numLights > 0 ? 8 : 0, nSun = skipSun ? 0 : 1, nSky = 1, nBrdf = 1;
    // a ray leaving the surface toward `dir` starts on the side it leaves from (thin films,
    // closesthit.cu:457, 614, 799)
    auto spawn = [&](const F3 &dir) { return sf.thin ? (dot(dir, st.normal) > 0.0f ? frontPos : backPos) : frontPos; };
    const int nMis = nLocal + nSun + nSky + nBrdf;
    const float sunMis = float(nSun) / nMis, skyMis = float(nSky) / nMis, brdfMis = float(nBrdf) / nMis;
    const float localMis = float(nLocal) / nMis;

    Reservoir localRes;
    LightSample localSample;
    for (int i = 0; i < nLocal; ++i) {  // closesthit.cu:350-376
        float srcPdf;
        const int li = (int)alias_sample(s.mesh.lightAlias, c.rnd(), srcPdf);
        if (li >= s.mesh.numLights) continue;
        const F2 uv = c.rnd2();
        const LightSample cand = tri_sample(tri_light(s.mesh, li), uv, sf.pos);
        const float blended = mis_weight(sf, cand, srcPdf, localMis, false, brdfMis);
        const float tp = target_pdf(cand, sf);
        const float rr = c.rnd();
        if (blended != 0.0f)
            if (stream_sample(localRes, (uint32_t)li, uv, rr, tp, 1.0f / blended)) localSample = cand;
    }
    finalize(localRes, 1.0f, (float)nMis);
    localRes.M = 1;

    Reservoir sunRes;
    LightSample sunLs;
    for (int i = 0; i < nSun; ++i) {
        float srcPdf;
        int idx = (int)alias_sample(k.sunAlias, c.rnd(), srcPdf);
        LightSample cand = sun_sample(s, idx);
        int sx = idx % k.sunW, sy = idx / k.sunW;
        F2 uv((sx + 0.5f) / float(k.sunW), (sy + 0.5f) / float(k.sunH));
        float blended = mis_weight(sf, cand, srcPdf, sunMis, true, brdfMis);
        float tp = target_pdf(cand, sf);
        float rr = c.rnd();
        if (stream_sample(sunRes, kSunLight, uv, rr, tp, 1.0f / blended)) sunLs = cand;
    }
    finalize(sunRes, 1.0f, (float)nMis);
    sunRes.M = 1;

    Reservoir skyRes;
    LightSample skyLs;
    for (int i = 0; i < nSky; ++i) {
        float srcPdf;
        int idx = (int)alias_sample(k.skyAlias, c.rnd16(), srcPdf);
        LightSample cand = sky_sample(s, idx);
        int sx = idx % k.skyW, sy = idx / k.skyW;
        F2 uv((sx + 0.5f) / float(k.skyW), (sy + 0.5f) / float(k.skyH));
        float blended = mis_weight(sf, cand, srcPdf, skyMis, true, brdfMis);
        float tp = target_pdf(cand, sf);
        float rr = c.rnd();
        if (stream_sample(skyRes, kSkyLight, uv, rr, tp, 1.0f / blended)) skyLs = cand;
    }
    finalize(skyRes, 1.0f, (float)nMis);
    skyRes.M = 1;

    Reservoir brdfRes;
    LightSample brdfLs;
    for (int i = 0; i < nBrdf; ++i) {
        float lightSrcPdf = 0.0f;
        uint32_t li = kInvalidLight;
        F2 uv(0, 0);
        LightSample cand;
        F3 sd;
        float bp;
        bool tr = false;
        F4 u = c.rnd4();
        F3 bop;
        disney_sample(u, st.normal, st.geoNormal, st.wo, st.albedo, st.metallic, st.translucency, st.roughness, sd,
                      bop, bp, tr);
        if (bp > 0.0f) {
            const AnyHit bh = closest_any(s, spawn(sd), sd, FLT_MAX);
            if (bh.isMesh && nLocal > 0) {  // __closesthit__bsdf_light (closesthit.cu:854-900)
                const MeshInstance &mi = s.mesh.inst[bh.mesh.row];
                if (s.mats[mi.block].isEmissive && mi.lightBase >= 0) {
                    li = (uint32_t)(mi.lightBase + bh.mesh.tri);
                    if (li >= (uint32_t)s.mesh.numLights) {
                        li = kInvalidLight;
                    } else {
                        uv = inverse_tri_sample(bh.mesh.u, bh.mesh.v);
                        cand = tri_sample(tri_light(s.mesh, (int)li), uv, sf.pos);
                        lightSrcPdf = s.mesh.lightAlias[li].p;
                    }
                }
            } else if (!bh.hit) {
                if (equal_area_cone_uv(uv, k.sunDir, sd, kSunCosMax())) {
                    li = kSunLight;
                    int x = (int)(uv.x * k.sunW - 0.5f), y = (int)(uv.y * k.sunH - 0.5f);
                    if (x >= k.sunW) x %= k.sunW;
                    if (x < 0) x = k.sunW - ((-x) % k.sunW);
                    y = clampi(y, 0, k.sunH - 1);
                    int idx = y * k.sunW + x;
                    cand = sun_sample(s, idx);
                    cand.position = sd;
                    lightSrcPdf = k.sunAlias[idx].p;
                } else {
                    li = kSkyLight;
                    uv = equal_area_sphere_uv(sd);
                    int x = (int)(uv.x * k.skyW - 0.5f), y = (int)(uv.y * k.skyH - 0.5f);
                    // clamp2i result discarded in the reference (closesthit.cu:508)
                    int idx = y * k.skyW + x;
                    cand = sky_sample(s, idx);
                    cand.position = sd;
                    lightSrcPdf = k.skyAlias[idx].p;
                }
            }
        }
        if (lightSrcPdf == 0.0f) continue;
        float tp = target_pdf(cand, sf);
        bool env = li == kSkyLight || li == kSunLight;
        float misW = (li == kSkyLight) ? skyMis : ((li == kSunLight) ? sunMis : localMis);
        float blended = mis_weight(sf, cand, lightSrcPdf, misW, env, brdfMis);
        float rr = c.rnd();
        if (stream_sample(brdfRes, li, uv, rr, tp, 1.0f / blended)) brdfLs = cand;
    }
    finalize(brdfRes, 1.0f, (float)nMis);
    brdfRes.M = 1;

    combine(ris, localRes, 0.5f, localRes.targetPdf);
    float r1 = c.rnd();
    bool selSun = combine(ris, sunRes, r1, sunRes.targetPdf);
    float r2 = c.rnd();
    bool selSky = combine(ris, skyRes, r2, skyRes.targetPdf);
    float r3 = c.rnd();
    bool selBrdf = combine(ris, brdfRes, r3, brdfRes.targetPdf);
    finalize(ris, 1.0f, 1.0f);
    ris.M = 1;
    if (selBrdf) lightSample = brdfLs;
    else if (selSky) lightSample = skyLs;
    else if (selSun) lightSample = sunLs;
    else lightSample = localSample;

    bool visible = false;
    if (lightSample.type != LtInvalid && ris.lightData != 0) {
        visible = !light_occluded(s, spawn(light_dir(lightSample, sf.pos)), lightSample, sf.pos, 0.0f);
        if (!visible) { ris.lightData = 0; ris.weightSum = 0; }
    }

    Reservoir rr;
    if (restir) {
        combine(rr, ris, 0.5f, ris.targetPdf);
        const Camera &pc = s.prevCam;
        F3 cur = sf.pos;
        F3 prevW = cur + motionWS;
        F2 puv = pc.dir_to_uv(normalize(prevW - pc.pos));
        int ppx = (int)(puv.x * pc.res.x), ppy = (int)(puv.y * pc.res.y);
        F3 dd = prevW - pc.pos;
        float expDepth = std::sqrt(dd.x * dd.x + dd.y * dd.y + dd.z * dd.z);
        int off[3][2];
        off[0][0] = ppx - c.px; off[0][1] = ppy - c.py;
        F2 d1 = concentric_disk(c.rnd2()) * 64.0f;
        off[1][0] = ppx - c.px + (int)d1.x; off[1][1] = ppy - c.py + (int)d1.y;
        F2 d2 = concentric_disk(c.rnd2()) * 64.0f;
        off[2][0] = (int)d2.x; off[2][1] = (int)d2.y;
        unsigned cached = 0;
        int selLoop = -1;
        const float mCap = 20.0f;
        for (int i = 0; i < 3; ++i) {
            int x = reflect_into_view(c.px + off[i][0], f.W), y = reflect_into_view(c.py + off[i][1], f.H);
            Surf ts;
            if (!prev_surface(c, ts, x, y)) continue;
            bool nOk = dot(sf.st.normal, ts.st.geoNormal) >= 0.5f;
            bool dOk = std::fabs(expDepth - ts.depth) <= 0.1f * mymax(expDepth, ts.depth);
            bool rOk = std::fabs(sf.st.roughness - ts.st.roughness) <= 0.5f * mymax(sf.st.roughness, ts.st.roughness);
            if (!(nOk && dOk && rOk)) continue;
            cached |= (1u << i);
            Reservoir pr = load_prev_reservoir(c, x, y);
            if (std::isnan(pr.weightSum) || std::isinf(pr.weightSum)) pr = Reservoir{};
            if (pr.M > mCap) pr.M = mCap;
            float nw = 0;
            LightSample cand;
            if (pr.lightData != 0) {
                if (!light_from_reservoir(s, cand, pr, sf, nLocal > 0)) pr = Reservoir{};
                nw = target_pdf(cand, sf);
            }
            float rn = c.rnd();
            if (combine(rr, pr, rn, nw)) { lightSample = cand; selLoop = i; }
        }
        if (rr.lightData != 0) {
            float piv = rr.targetPdf, piSum = rr.targetPdf * 1;
            for (int i = 0; i < 3; ++i) {
                if ((cached & (1u << i)) == 0) continue;
                int x = reflect_into_view(c.px + off[i][0], f.W), y = reflect_into_view(c.py + off[i][1], f.H);
                Surf ts;
                prev_surface(c, ts, x, y);
                LightSample sel;
                light_from_reservoir(s, sel, rr, ts, nLocal > 0);
                float ps = target_pdf(sel, ts);
                if (ps > 0 && !(i == 0 && i == selLoop) && !s.prevSceneEmpty) {
                    const float extra = 0.01f + 0.01f * ts.depth;
                    if (light_occluded(s, ts.pos, lightSample, ts.pos, extra)) ps = 0.0f;
                }
                Reservoir pr = load_prev_reservoir(c, x, y);
                if (std::isnan(pr.weightSum) || std::isinf(pr.weightSum)) pr = Reservoir{};
                if (pr.M > mCap) pr.M = mCap;
                if (selLoop == i) piv = ps;
                piSum += ps * pr.M;
            }
            finalize(rr, piv, piSum);
        }
        if (lightSample.type != LtInvalid) {
            visible = !light_occluded(s, spawn(light_dir(lightSample, sf.pos)), lightSample, sf.pos, 0.0f);
            if (!visible) { rr.lightData = 0; rr.weightSum = 0; }
        }
    }
    const Reservoir &shade = restir ? rr : ris;
    if (lightSample.type != LtInvalid && shade.lightData != 0 && visible) {
        F3 sd = light_dir(lightSample, sf.pos);
        F3 alb = skipAlbedo ? F3(1.0f) : st.albedo;
        F3 bsdf; float pdf;
        disney_eval(st.normal, st.geoNormal, sd, st.wo, alb, st.metallic, st.translucency, st.roughness, bsdf, pdf);
        float cosT = std::fmax(0.0f, dot(sd, st.normal));
        F3 L = bsdf * cosT * lightSample.radiance * shade.weightSum / lightSample.solidAnglePdf;
        rd.radiance += L;
    }
    if (restir) store_reservoir(c, rr);
}

bool trace_next(Px &c, Ray &rd, F3 &radiance, F3 &throughput) {  // RayGen.cu:8-100
    rd.bsdfOverPdf = F3(1.0f);
    rd.pdf = 0.0f;
    rd.radiance = F3(0.0f);
    rd.wo = -rd.wi;
    rd.distance = kRayMax;
    rd.terminate = false;
    rd.lastDiffuse = rd.curDiffuse;
    rd.curDiffuse = false;
    const AnyHit h = closest_any(c.s, rd.pos, rd.wi, kRayMax);
    if (h.hit) on_hit(c, rd, h);
    else on_miss(c, rd);
    radiance += throughput * rd.radiance;
    if (rd.terminate || rd.pdf <= 0.0f || is_null(rd.bsdfOverPdf)) return false;
    throughput *= rd.bsdfOverPdf;
    return true;
}

void primary_only(Px &c) {
    // C2 bring-up: primary DDA + sky miss + G-buffer of the first hit, no NEE.
    const Scene &s = c.s;
    F2 j = c.rnd2();
    F2 uv = (F2((float)c.px, (float)c.py) + j) * s.cam.invRes;
    Ray rd;
    rd.pos = s.cam.pos;
    rd.wi = s.cam.uv_to_dir(uv);
    rd.wo = -rd.wi;
    Hit h = dda_closest(s.world, rd.pos, rd.wi, kRayMax);
    size_t pi = c.idx();
    if (!h.hit) {
        on_miss(c, rd);
        c.f.depth[pi] = kRayMax;
        c.f.illum[pi] = F4(rd.radiance, kRayMax);
        return;
    }
    F3 hp = rd.pos + rd.wi * h.t;
    const int axis = (h.face < 2) ? 1 : (h.face < 4 ? 0 : 2);
    const int cell = axis == 0 ? h.x : (axis == 1 ? h.y : h.z);
    hp[axis] = (float)(cell + ((h.face == 0 || h.face == 3 || h.face == 4) ? 1 : 0));
    F3 fp, bp, ng;
    safe_spawn(h, hp, fp, bp, ng);
    const Material &m = s.mats[h.id];
    F3 alb = max3f(m.albedo, F3(0.001f));
    c.f.material[pi] = (float)m.materialId;
    c.f.normalRough[pi] = F4(ng, m.roughness);
    c.f.geoNormalThin[pi] = F4(ng, 0.0f);
    c.f.matParam[pi] = F4(m.metallic ? 1.0f : 0.0f, m.translucency, 0.0f, 0.0f);
    c.f.albedo[pi] = F4(alb, 1.0f);
    c.f.motion[pi] = F4(0.0f);
    c.f.depth[pi] = h.t;
    c.f.illum[pi] = F4(F3(0.0f), h.t);
}

}  // namespace

void trace_frame(const Scene &s, Frame &f, int it, int y0, int y1, bool primaryOnlyMode) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < f.W; ++x) {
            Px c{s, f, x, y, it};
            if (primaryOnlyMode) { primary_only(c); continue; }
            // __raygen__pathtracer (RayGen.cu:102-182)
            F2 j = c.rnd2();
            F2 uv = (F2((float)x, (float)y) + j) * s.cam.invRes;
            F3 dir = s.cam.uv_to_dir(uv);
            Ray rd;
            rd.pos = s.cam.pos;
            rd.wi = dir;
            F3 radiance(0.0f), throughput(1.0f);
            bool done = false;
            float primaryDist = kRayMax;
            int total = 0, diffuse = 0;
            while (!done) {
                done = !trace_next(c, rd, radiance, throughput);
                ++total;
                if (rd.curDiffuse) ++diffuse;
                if (total == s.totalBounceLimit || diffuse == s.diffuseBounceLimit) done = true;
                if (rd.depth == 0) primaryDist = rd.distance;
                ++rd.depth;
            }
            if (std::isnan(radiance.x) || std::isnan(radiance.y) || std::isnan(radiance.z)) radiance = F3(0.5f);
            size_t i = (size_t)y * f.W + x;
            f.depth[i] = primaryDist;
            f.illum[i] = F4(radiance, primaryDist);
        }
}

void post_trace_copies(Frame &f) {
    f.prevGeoNormalThin = f.geoNormalThin;
    f.prevAlbedo = f.albedo;
    f.prevMatParam = f.matParam;
}

}  // namespace orc
