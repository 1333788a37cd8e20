// ORACLE (test infrastructure only): restatement of the ReLAX-style denoiser,
// renderer/denoising/{Denoiser.cu, FireflyFilter.h, BufferCopy.h,
// TemporalAccumulation.h, HistoryFix.h, HistoryClamping.h, AtrousSmem.h,
// Atrous.h, DenoiserCommon.h}.
//
// Defined semantics where the reference is undefined or racy:
//   * FireflyBoilingFilter reduces over the whole 8x4 tile with sky / out of
//     bounds lanes contributing 0, in the __shfl_down tree order
//     (FireflyFilter.h:51-65); neighbour reads see pre-filter values.
//   * Load2DUshort1 on the R32F material surface (HistoryFix.h:61,87,
//     Atrous.h:47,110) reads 16 bits at byte offset 2*x: the low half of the
//     float at x>>1 for even x, the high half for odd x; the byte coordinate
//     clamps to [0, 4W-2], the row to [0, H-1].
//   * surface reads clamp to the edge (Sampler.h:134-188).
#include <cstring>
#include "orc_trace.h"

namespace orc {
namespace {

constexpr float kRange = 500000.0f;

inline int cl(int v, int n) { return v < 0 ? 0 : (v >= n ? n - 1 : v); }
inline F4 ld4(const std::vector<F4> &b, const Frame &f, int x, int y) { return b[(size_t)cl(y, f.H) * f.W + cl(x, f.W)]; }
inline float ld1(const std::vector<float> &b, const Frame &f, int x, int y) {
    return b[(size_t)cl(y, f.H) * f.W + cl(x, f.W)];
}
inline float ld_ushort(const std::vector<float> &b, const Frame &f, int x, int y) {
    long bx = 2L * x;
    if (bx < 0) bx = 0;
    if (bx > 4L * f.W - 2) bx = 4L * f.W - 2;
    uint32_t bits;
    std::memcpy(&bits, &b[(size_t)cl(y, f.H) * f.W + (bx >> 2)], 4);
    return (float)((((bx >> 1) & 1) ? (bits >> 16) : bits) & 0xFFFFu);
}
inline F3 world_pos(const Camera &c, int x, int y, float depth) {  // DenoiserCommon.h:272-279
    F2 uv = (F2((float)x, (float)y) + 0.5f) * c.invRes;
    return c.pos + c.uv_to_dir(uv) * depth;
}
inline float linear_step(float a, float b, float x) { return saturate((x - a) / (b - a)); }
inline float smooth_step(float a, float b, float x) { float t = linear_step(a, b, x); return t * t * (3.0f - 2.0f * t); }
inline float acos_approx(float x) { return std::sqrt(2.0f) * std::sqrt(saturate(1.0f - x)); }
inline float nonexp_weight(float x, float px, float py) { return smooth_step(1.0f, 0.0f, std::fabs(x * px + py)); }
inline float normal_weight_param(float roughness, float angleFraction) {
    float r = saturate(roughness), p = saturate(angleFraction);
    float tanHalf = r * r * p / (1.0f - p + 1e-6f);
    float angle = std::atan(tanHalf);
    return 1.0f / mymax(angle, 1e-6f);
}
inline float plane_weight(const F3 &c, const F3 &n, const F3 &s, float thr) {
    return std::fabs(dot(s - c, n)) < thr ? 1.0f : 0.0f;
}
inline F3 rgb_to_ycocg(const F3 &c) { return F3(0.25f * (c.x + 2.0f * c.y + c.z), c.x - c.z, c.y - 0.5f * (c.x + c.z)); }
inline F3 ycocg_to_rgb(const F3 &c) { return F3(c.x + 0.5f * (c.y - c.z), c.x + 0.5f * c.z, c.x - 0.5f * (c.y + c.z)); }

// hash RNG (DenoiserCommon.h:407-511)
inline uint32_t seq_hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
    return x;
}
inline uint32_t explode(uint32_t x) {
    x = (x | (x << 8)) & 0x00FF00FFu; x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u; x = (x | (x << 1)) & 0x55555555u;
    return x;
}
inline uint32_t rng_init(uint32_t px, uint32_t py, uint32_t frame) {
    uint32_t lin = explode(px) | (explode(py) << 1);
    uint32_t seed = seq_hash(frame + 0x035F9F29u);
    return seed ^ (seq_hash(lin) + 0x9E3779B9u + (seed << 6) + (seed >> 2));
}

// Catmull-Rom 12-tap (Sampler.h:576-650) on float4 with the Float4 operator quirks
template <bool kQuirkyF4>
F4 bicubic12(const std::vector<F4> &b, const Frame &f, F2 uv) {
    F2 UV(uv.x * (float)f.W, uv.y * (float)f.H);
    F2 tc(std::floor(UV.x - 0.5f) + 0.5f, std::floor(UV.y - 0.5f) + 0.5f);
    F2 fr = UV - tc, f2 = fr * fr, f3 = f2 * fr;
    F2 w0 = f2 - 0.5f * (f3 + fr);
    F2 w1 = 1.5f * f3 - 2.5f * f2 + 1.0f;
    F2 w3 = 0.5f * (f3 - f2);
    F2 w2 = 1.0f - w0 - w1 - w3;
    int x1 = (int)std::floor(UV.x - 0.5f), y1 = (int)std::floor(UV.y - 0.5f);
    int x0 = x1 - 1, x2 = x1 + 1, x3 = x1 + 2, y0 = y1 - 1, y2 = y1 + 1, y3 = y1 + 2;
    const int sx[12] = {x1, x2, x0, x1, x2, x3, x0, x1, x2, x3, x1, x2};
    const int sy[12] = {y0, y0, y1, y1, y1, y1, y2, y2, y2, y2, y3, y3};
    const float wt[12] = {w1.x * w0.y, w2.x * w0.y, w0.x * w1.y, w1.x * w1.y, w2.x * w1.y, w3.x * w1.y,
                          w0.x * w2.y, w1.x * w2.y, w2.x * w2.y, w3.x * w2.y, w1.x * w3.y, w2.x * w3.y};
    F4 out(0.0f);
    F3 out3(0.0f);
    float sum = 0;
    for (int i = 0; i < 12; ++i) {
        sum += wt[i];
        F4 v = ld4(b, f, sx[i], sy[i]);
        if (kQuirkyF4) out += v * wt[i];
        else out3 += v.xyz() * wt[i];
    }
    if (kQuirkyF4) { out /= sum; return out; }
    out3 /= sum;
    return F4(out3, 0.0f);
}

F3 bicubic_smoothstep3(const std::vector<F4> &b, const Frame &f, F2 uv) {  // BoundaryFuncClamp
    F2 UV(uv.x * (float)f.W, uv.y * (float)f.H);
    F2 tc(std::floor(UV.x - 0.5f) + 0.5f, std::floor(UV.y - 0.5f) + 0.5f);
    F2 fr = UV - tc, f2 = fr * fr, f3 = f2 * fr;
    F2 w1 = -2.0f * f3 + 3.0f * f2;
    F2 w0 = 1.0f - w1;
    int x0 = (int)std::floor(UV.x - 0.5f), y0 = (int)std::floor(UV.y - 0.5f);
    const int sx[4] = {x0, x0 + 1, x0, x0 + 1}, sy[4] = {y0, y0, y0 + 1, y0 + 1};
    const float wt[4] = {w0.x * w0.y, w1.x * w0.y, w0.x * w1.y, w1.x * w1.y};
    F3 out(0.0f);
    float sum = 0;
    for (int i = 0; i < 4; ++i) {
        sum += wt[i];
        out += ld4(b, f, sx[i], sy[i]).xyz() * wt[i];
    }
    out /= sum;
    return out;
}

void bilinear_taps(const Frame &f, F2 uv, int &x0, int &y0, float w[4]) {
    F2 UV(uv.x * (float)f.W, uv.y * (float)f.H);
    F2 tc(std::floor(UV.x - 0.5f) + 0.5f, std::floor(UV.y - 0.5f) + 0.5f);
    F2 fr = UV - tc;
    F2 w1 = fr, w0 = 1.0f - fr;
    x0 = (int)std::floor(UV.x - 0.5f);
    y0 = (int)std::floor(UV.y - 0.5f);
    w[0] = w0.x * w0.y; w[1] = w1.x * w0.y; w[2] = w0.x * w1.y; w[3] = w1.x * w1.y;
}
F4 bilinear_custom4(const std::vector<F4> &b, const Frame &f, F2 uv, const F4 &cw) {  // Sampler.h:452-498
    int x0, y0; float w[4];
    bilinear_taps(f, uv, x0, y0, w);
    const int sx[4] = {x0, x0 + 1, x0, x0 + 1}, sy[4] = {y0, y0, y0 + 1, y0 + 1};
    F4 out(0.0f);
    float sum = 0.0f;
    for (int i = 0; i < 4; ++i) {
        float wt = w[i] * cw[i];
        float weight = (wt < 1e-6f) ? 1e-6f : wt;  // max1f
        sum += weight;
        out += ld4(b, f, sx[i], sy[i]) * weight;
    }
    out /= sum;
    return out;
}
float bilinear_custom1(const std::vector<float> &b, const Frame &f, F2 uv, const F4 &cw) {  // Sampler.h:396-450
    int x0, y0; float w[4];
    bilinear_taps(f, uv, x0, y0, w);
    const int sx[4] = {x0, x0 + 1, x0, x0 + 1}, sy[4] = {y0, y0, y0 + 1, y0 + 1};
    float out = 0.0f, sum = 0.0f;
    for (int i = 0; i < 4; ++i) {
        float wt = w[i] * cw[i];
        float weight = (wt < 1e-6f) ? 1e-6f : wt;
        sum += weight;
        out += ld1(b, f, sx[i], sy[i]) * weight;
    }
    out /= sum;
    return out;
}

}  // namespace

// ---------------------------------------------------------------- D1
void pass_firefly(const Scene &s, Frame &f, int parity, float phiL) {
    const int W = f.W, H = f.H;
    const size_t stride = (size_t)W * H;
    const std::vector<F4> illum0 = f.illum;
    const std::vector<Reservoir> res0(f.reservoir.begin() + parity * stride, f.reservoir.begin() + (parity + 1) * stride);
    const float weightThreshold = 80.0f, minWeight = 5.0f, normalThreshold = 0.8f, depthSigma = 0.02f;
    const int tilesX = (W + 7) / 8, tilesY = (f.by1() - f.by0() + 3) / 4;
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < tilesX * tilesY; ++t) {
        const int tx0 = (t % tilesX) * 8, ty0 = f.by0() + (t / tilesX) * 4;
        float v[32];
        unsigned cnt[32];
        for (int l = 0; l < 32; ++l) {
            int x = tx0 + (l & 7), y = ty0 + (l >> 3);
            v[l] = 0.0f; cnt[l] = 0;
            if (x >= W || y >= f.by1()) continue;
            size_t i = (size_t)y * W + x;
            if (f.depth[i] > kRange) continue;
            const Reservoir &r = res0[i];
            bool valid = r.lightData != 0 && std::isfinite(r.weightSum) && r.weightSum > 0.0f;
            v[l] = valid ? r.weightSum : 0.0f;
            cnt[l] = valid ? 1u : 0u;
        }
        for (int off = 16; off > 0; off >>= 1)
            for (int l = 0; l < off; ++l) { v[l] += v[l + off]; cnt[l] += cnt[l + off]; }
        const float tileSum = v[0];
        const unsigned tileCnt = cnt[0];
        for (int l = 0; l < 32; ++l) {
            int x = tx0 + (l & 7), y = ty0 + (l >> 3);
            if (x >= W || y >= f.by1()) continue;
            size_t i = (size_t)y * W + x;
            const float cd = f.depth[i];
            if (cd > kRange) continue;
            Reservoir r = res0[i];
            const float cw = r.weightSum;
            if (!(r.lightData != 0 && std::isfinite(cw) && cw > 0.0f)) continue;
            const float nSum = tileSum - cw;
            const int nCnt = (int)tileCnt - 1;
            bool firefly = false;
            if (cw >= minWeight) {
                if (nCnt <= 0) firefly = true;
                else {
                    const float avg = nSum / float(nCnt);
                    if (avg > 0.0f && cw > avg * weightThreshold) firefly = true;
                }
            }
            if (!firefly) continue;
            const F4 cc4 = illum0[i];
            const float cLum = luminance(cc4.xyz());
            F3 cN = f.normalRough[i].xyz();
            const float cl_ = length(cN);
            if (cl_ > 0.0f) cN /= cl_; else cN = F3(0.0f, 1.0f, 0.0f);
            const float cMat = f.material[i];
            const F3 cWP = world_pos(s.cam, x, y, cd);
            const float g[3] = {1.0f, 2.0f, 1.0f};
            F4 filt = cc4;
            float filtW = 1.0f;
            F4 fb = cc4 * (g[0] * g[0]);
            float fbW = g[0] * g[0];
            const float depthScale = std::fmax(std::fabs(cd), 1.0f);
            const float nwp = normal_weight_param(1.0f, 0.25f);
            Reservoir best = r;
            float bestScore = FLT_MAX;
            bool repl = false;
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    if (dx == 0 && dy == 0) continue;
                    const int sx = x + dx, sy = y + dy;
                    if (sx < 0 || sy < 0 || sx >= W || sy >= H) continue;
                    const float gw = g[std::abs(dx)] * g[std::abs(dy)];
                    const size_t j = (size_t)sy * W + sx;
                    const F4 sc4 = illum0[j];
                    fb += sc4 * gw;
                    fbW += gw;
                    const float sd = f.depth[j];
                    if (sd > kRange) continue;
                    F3 sN = f.normalRough[j].xyz();
                    const float sl = length(sN);
                    if (sl <= 0.0f) continue;
                    sN /= sl;
                    const float nd = dot(cN, sN);
                    if (nd < normalThreshold) continue;
                    const float sMat = f.material[j];
                    if (std::fabs(sMat - cMat) > 0.5f) continue;
                    const F3 sWP = world_pos(s.cam, sx, sy, sd);
                    const float geo = plane_weight(cWP, cN, sWP, depthSigma * depthScale);
                    if (geo <= 0.0f) continue;
                    const float nw = nonexp_weight(acos_approx(clampf(nd, -1.0f, 1.0f)), nwp, 0.0f);
                    const float dw = std::exp(-std::fabs(sd - cd) / (depthScale * depthSigma + 1e-6f));
                    const float lw = std::exp(-std::fabs(luminance(sc4.xyz()) - cLum) * phiL);
                    const float tw = gw * geo * nw * dw * lw;
                    if (tw > 1e-5f) {
                        filt += sc4 * tw;
                        filtW += tw;
                    }
                    const Reservoir &nr = res0[j];
                    const bool nValid = nr.lightData != 0 && std::isfinite(nr.weightSum) && nr.weightSum > 0.0f &&
                                        nr.weightSum < cw;
                    if (nValid) {
                        const float dt = std::fabs(sd - cd) / (depthScale + 1e-6f);
                        const float nt = 1.0f - clampf(nd, 0.0f, 1.0f);
                        const float wd = std::fabs(nr.weightSum - cw);
                        const float score = dt + nt + 0.25f * wd;
                        if (score < bestScore) { bestScore = score; best = nr; repl = true; }
                    }
                }
            F4 outc;
            if (filtW > 0.0f) outc = filt / filtW;
            else if (fbW > 0.0f) outc = fb / fbW;
            else outc = cc4;
            f.illum[i] = outc;
            Reservoir &dst = f.reservoir[parity * stride + i];
            if (repl) dst = best;
            else {
                Reservoir c2 = r;
                float avg = (nCnt > 0) ? (nSum / float(nCnt)) : minWeight;
                float tgt = (nCnt > 0) ? (avg * weightThreshold) : minWeight;
                tgt = std::fmax(tgt, minWeight);
                c2.weightSum = std::fmin(c2.weightSum, tgt);
                dst = c2;
            }
        }
    }
}

// ---------------------------------------------------------------- D2
void pass_copy_sky(Frame &f) {
    for (size_t i = (size_t)f.by0() * f.W; i < (size_t)f.by1() * f.W; ++i)
        if (f.depth[i] > kRange) f.output[i] = f.illum[i];
}

// ---------------------------------------------------------------- D3
void pass_temporal(const Scene &s, Frame &f, const DenoiseParams &p) {
    const int W = f.W, H = f.H;
    const Camera &cam = s.cam, &pc = s.prevCam;
    const F2 invScreen(1.0f / (float)W, 1.0f / (float)H);
    const Q rot = rotation_between(Q(pc.dir, 0.f), Q(cam.dir, 0.f));
#pragma omp parallel for schedule(dynamic, 4)
    for (int y = f.by0(); y < f.by1(); ++y)
        for (int x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            const float z = f.depth[i];
            if (z > p.denoisingRange) continue;
            F3 cN = f.normalRough[i].xyz();
            F3 avgN = cN;
            for (int a = -1; a <= 1; ++a)
                for (int b = -1; b <= 1; ++b) {
                    if (a == 0 && b == 0) continue;
                    avgN += ld4(f.normalRough, f, x + a, y + b).xyz();
                }
            avgN /= 9.0f;
            F2 pixelUv = (F2((float)x, (float)y) + 0.5f) * invScreen;
            F2 curUV = (F2((float)x, (float)y) + 0.5f) * cam.invRes;
            F3 view = cam.uv_to_dir(curUV);
            F3 cWP = world_pos(cam, x, y, z);
            F3 V = -normalize(view);
            float NoV = std::fabs(dot(cN, V));
            F3 mv = f.motion[i].xyz();
            F3 prevWP = cWP + mv;
            F2 prevUV = pc.dir_to_uv(normalize(prevWP - pc.pos));
            F3 illum = f.illum[i].xyz();
            float m1 = luminance(illum), m2 = m1 * m1;
            F3 camDelta = pc.pos - cam.pos;
            auto parallax = [&](const F3 &X, F2 uvZero, const Camera &c) {
                F2 uvv = c.dir_to_uv(normalize(X - c.pos));
                F2 d = (uvv - uvZero) * F2((float)W, (float)H);
                return std::sqrt(d.x * d.x + d.y * d.y);
            };
            float par1 = parallax(prevWP + camDelta, pixelUv, pc);
            float par2 = parallax(prevWP - camDelta, prevUV, cam);
            float parMax = mymax(par1, par2);
            float thrB = p.disocclusionThreshold + (1.5f / (float)H);
            float thrA = p.disocclusionThresholdAlternate + (1.5f / (float)H);
            float thr = lerpf(thrB, thrA, 0.0f);

            // loadSurfaceMotionBasedPrevData (TemporalAccumulation.h:29-215)
            F3 nIn = normalize(avgN);
            F3 dp = prevWP - pc.pos;
            float estDepth = length(dp);
            F2 ppf(prevUV.x * (float)W, prevUV.y * (float)H);
            int ox = (int)std::floor(ppf.x - 0.5f), oy = (int)std::floor(ppf.y - 0.5f);
            float pixelSize = cam.pixel_world_size_scale() * z;
            float frustum = pixelSize * (float)(W < H ? W : H);
            // TemporalAccumulation.h:82-83: `float disocclusionThresholdSlopeScale = 1.0 / lerp(...)`
            float slope = (float)(1.0 / (double)lerpf(lerpf(0.05f, 1.0f, NoV), 1.0f, saturate(parMax / 30.0f)));
            float t0 = saturate(thr * slope) * frustum;
            F4 thr4(t0);
            {  // IsInScreenBilinear with the Float4 quirk (DenoiserCommon.h:82-104)
                float r[4] = {ox >= 0 ? 1.f : 0.f, oy >= 0 ? 1.f : 0.f, ox + 1 >= 0 ? 1.f : 0.f, oy + 1 >= 0 ? 1.f : 0.f};
                float cmp[4] = {ox < W ? 1.f : 0.f, oy < H ? 1.f : 0.f, ox + 1 < W ? 1.f : 0.f, oy + 1 < H ? 1.f : 0.f};
                for (int k = 0; k < 4; ++k) r[k] *= cmp[k];
                F4 a(r[0], r[2], r[0], r[2]), b(r[1], r[1], r[3], r[3]);
                thr4 *= (a * b);
            }
            thr4 -= 1e-6f;
            static const int bc[4][2][2] = {{{0, -1}, {-1, 0}}, {{1, -1}, {2, 0}}, {{-1, 1}, {0, 2}}, {{2, 1}, {1, 2}}};
            static const int bl[4][2] = {{0, 0}, {1, 0}, {0, 1}, {1, 1}};
            float bicValid = 1.0f;
            F4 tapsValid(0.0f);
            for (int a = 0; a < 4; ++a)
                for (int b = 0; b < 2; ++b) {
                    float pz = ld1(f.prevDepth, f, ox + bc[a][b][0], oy + bc[a][b][1]);
                    bicValid *= std::fabs(pz - estDepth) > thr4[a] ? 0.0f : 1.0f;
                }
            for (int a = 0; a < 4; ++a) {
                float pz = ld1(f.prevDepth, f, ox + bl[a][0], oy + bl[a][1]);
                float v = std::fabs(pz - estDepth) > thr4[a] ? 0.0f : 1.0f;
                bicValid *= v;
                tapsValid[a] = v;
            }
            F3 pnf = normalize(bicubic_smoothstep3(f.prevNormalRough, f, prevUV));
            F3 pnr = normalize(rotate(rot, Q(pnf, 0.f)).v);
            if (dot(nIn, pnr) < 0.0f) { tapsValid = F4(0.0f); bicValid = 0.0f; }
            bool useBic = bicValid > 0;
            F4 prevI = useBic ? bicubic12<true>(f.prevIllum, f, prevUV) : bilinear_custom4(f.prevIllum, f, prevUV, tapsValid);
            F3 prevF = useBic ? bicubic12<false>(f.prevFast, f, prevUV).xyz()
                              : bilinear_custom4(f.prevFast, f, prevUV, tapsValid).xyz();
            prevI = max4f(prevI, F4(0.0f));
            prevF = max3f(prevF, F3(0.0f));
            float found = (bicValid > 0.0f) ? 2.0f : 1.0f;
            int bx0, by0; float bw[4];
            bilinear_taps(f, prevUV, bx0, by0, bw);
            float quality = (bicValid > 0) ? 1.0f : dot(F4(bw[0], bw[1], bw[2], bw[3]), F4(1.0f));
            float hist;
            if (dot(tapsValid, F4(1.0f)) == 0.0f) { found = 0.0f; quality = 0.0f; hist = 0.0f; }
            else hist = bilinear_custom1(f.prevHistLen, f, prevUV, tapsValid);

            hist = hist + 1.0f;
            F3 Vp = normalize(prevWP - pc.pos);
            float NoVp = std::fabs(dot(cN, Vp));
            float sq = (NoVp + 1e-3f) / (NoV + 1e-3f);
            sq *= sq;
            sq *= sq;
            quality *= lerpf(0.1f, 1.0f, saturate(sq));
            if (quality < 1.0f) {
                hist *= std::sqrt(quality);
                hist = mymax(hist, 1.0f);
            }
            hist = mymin(hist, p.maxAccumulatedFrameNum);
            float alpha = (found > 0) ? mymax(1.0f / (p.maxAccumulatedFrameNum + 1.0f), 1.0f / hist) : 1.0f;
            float alphaR = (found > 0) ? mymax(1.0f / (p.maxFastAccumulatedFrameNum + 1.0f), 1.0f / hist) : 1.0f;
            F4 acc = lerp4(prevI, F4(illum, m2), alpha);
            F3 accR = lerp3(prevF, illum, alphaR);
            f.ping[i] = acc;
            f.pong[i] = F4(accR, 0.0f);
            f.histLen[i] = hist;
        }
}

// ---------------------------------------------------------------- D4
void pass_history_fix(const Scene &s, Frame &f) {
    const int W = f.W, H = f.H;
    const std::vector<F4> ping = f.ping;
#pragma omp parallel for schedule(dynamic, 4)
    for (int y = f.by0(); y < f.by1(); ++y)
        for (int x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            const float z = f.depth[i], hist = f.histLen[i];
            if (z > kRange || hist > 4.0f) continue;
            const float cMat = ld_ushort(f.material, f, x, y);
            const F3 cN = f.normalRough[i].xyz();
            const F3 cWP = world_pos(s.cam, x, y, z);
            const float dthr = 0.003f * z;
            F4 sum = ping[i];
            float wsum = 1.0f;
            const float r = std::exp2(4.0f - hist) + 1.0f;
            for (int j = -2; j <= 2; ++j)
                for (int k = -2; k <= 2; ++k) {
                    const int sx = x + (int)(k * r), sy = y + (int)(j * r);
                    const bool inside = sx >= 0 && sy >= 0 && sx < W && sy < H;
                    if (k == 0 && j == 0) continue;
                    const float sMat = ld_ushort(f.material, f, sx, sy);
                    const F3 sN = ld4(f.normalRough, f, sx, sy).xyz();
                    const float sz = ld1(f.depth, f, sx, sy);
                    const F3 sWP = world_pos(s.cam, sx, sy, sz);
                    float w = plane_weight(cWP, cN, sWP, dthr);
                    w *= std::pow(std::fmax(0.01f, dot(cN, sN)), 8.0f);
                    w = inside ? w : 0;
                    w *= (float)(sMat == cMat);
                    if (w > 1e-4f) {
                        sum += ld4(ping, f, sx, sy) * w;
                        wsum += w;
                    }
                }
            f.pong[i] = sum / wsum;
        }
}

// ---------------------------------------------------------------- D5
void pass_history_clamp(Frame &f) {
    const int W = f.W;
#pragma omp parallel for schedule(dynamic, 4)
    for (int y = f.by0(); y < f.by1(); ++y)
        for (int x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            f.clampBits[i] = 0.0f;
            if (f.depth[i] > kRange) continue;
            const float hist = f.histLen[i];
            F3 m1(0.0f), m2(0.0f), nm1(0.0f);
            float nm2 = 0.0f;
            for (int dx = -2; dx <= 2; ++dx)
                for (int dy = -2; dy <= 2; ++dy) {
                    F3 sy = rgb_to_ycocg(ld4(f.pong, f, x + dx, y + dy).xyz());
                    m1 += sy;
                    m2 += sy * sy;
                    F3 nz = ld4(f.illum, f, x + dx, y + dy).xyz();
                    float nl = luminance(nz);
                    nm1 += nz;
                    nm2 += nl * nl;
                }
            m1 /= 25.0f; m2 /= 25.0f; nm1 /= 25.0f; nm2 /= 25.0f;
            F3 sigma = sqrt3f(max3f(F3(0.0f), m2 - m1 * m1));
            F3 cmin = m1 - 2.0f * sigma, cmax = m1 + 2.0f * sigma;
            F3 center = rgb_to_ycocg(f.pong[i].xyz());
            // LinearMath.h:69-72 templates: Float3 operator< / > compare .x only
            f.clampBits[i] = (float)((cmin.x < center.x ? 1 : 0) | (cmax.x > center.x ? 2 : 0) | (hist > 4.0f ? 4 : 0));
            cmin = (cmin.x < center.x) ? cmin : center;
            cmax = (cmax.x > center.x) ? cmax : center;
            F4 pi = f.ping[i];
            F3 dY = rgb_to_ycocg(pi.xyz());
            F3 cY = clamp3f(dY, cmin, cmax);
            F3 cRgb = ycocg_to_rgb(cY);
            F4 outD(cRgb, pi.w);
            F3 respC = ycocg_to_rgb(center);
            F4 outR(respC, 0.0f);
            if (hist <= 4.0f) outD.set_xyz(outR.xyz());
            float factor = (cY.x - dY.x) == 0.0f ? 0.0f : saturate((cY.x - dY.x) / (center.x - dY.x));
            // test diagnostic bit 8: the factor's quotient ill-conditioned (see denoise.hip)
            if (hist > 4.0f && factor > 0.0f && factor < 1.0f &&
                std::fabs(center.x - dY.x) <= 1e-3f * std::fmax(std::fabs(center.x), std::fabs(dY.x)))
                f.clampBits[i] += 8.0f;
            if (hist <= 4.0f) factor = 1.0f;
            float hdl = 10.0f * 0.3f * luminance(abs3(respC - pi.xyz()));
            hdl *= factor;
            if (hist <= 4.0f) hdl = 0.0f;
            F3 dist = nm1 - respC;
            float distL = luminance(abs3(dist));
            F3 acc = (distL == 0.0f) ? F3(0.0f) : dist * hdl / distL;
            float accL = luminance(abs3(acc));
            float ratio = (accL == 0.0f) ? 0.0f : distL / accL;
            if (ratio < 1.0) acc *= ratio;
            if (ratio <= 0.0f) acc = F3(0.0f);
            outD.set_xyz(outD.xyz() + acc);
            outR.set_xyz(outR.xyz() + acc);
            float dL = luminance(pi.xyz()), nL = luminance(nm1);
            float tSig = 0.5f * std::sqrt(std::fmax(0.0f, nm2 - nL * nL));
            float sSig = 4.5f * sigma.x;
            float reset = 0.5f * std::fmax(0.0f, std::fabs(dL - nL) - sSig - tSig) /
                          (1.0e-6f + std::fmax(dL, nL) + sSig + tSig);
            reset = saturate(reset);
            F3 noisyC = f.illum[i].xyz();
            outD.set_xyz(lerp3(outD.xyz(), noisyC, reset));
            outR.set_xyz(lerp3(outR.xyz(), noisyC, reset));
            float oL = luminance(outD.xyz());
            outD.w += (oL * oL - dL * dL);
            outD.w = std::fmax(0.0f, outD.w);
            f.prevIllum[i] = outD;
            f.prevFast[i] = outR;
            f.prevHistLen[i] = hist;
        }
}

// ---------------------------------------------------------------- D6
void pass_atrous_smem(const Scene &s, Frame &f, const DenoiseParams &p) {
    const int W = f.W, H = f.H;
    // world position + material per clamped pixel, as the LDS preload computes it
    std::vector<F4> wpm((size_t)W * H);
#pragma omp parallel for
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            size_t i = (size_t)y * W + x;
            wpm[i] = F4(world_pos(s.cam, x, y, f.depth[i]), f.material[i]);
        }
    const float k3[2] = {0.44198f, 0.27901f};
#pragma omp parallel for schedule(dynamic, 4)
    for (int y = f.by0(); y < f.by1(); ++y)
        for (int x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            const float z = f.depth[i];
            if (z > 500000.0f) continue;
            const F3 cN = f.normalRough[i].xyz();
            const F3 cWP = wpm[i].xyz();
            const float cMat = wpm[i].w;
            const float hist = f.histLen[i];
            if (hist >= (float)3u) {
                F4 vs(0.0f);
                const float kern[4] = {1.0f / 4.0f, 1.0f / 8.0f, 1.0f / 8.0f, 1.0f / 16.0f};
                for (int dx = -1; dx <= 1; ++dx)
                    for (int dy = -1; dy <= 1; ++dy)
                        vs += ld4(f.prevIllum, f, x + dx, y + dy) * kern[std::abs(dx) * 2 + std::abs(dy)];
                float vm1 = luminance(vs.xyz());
                float var = std::fmax(0.0f, vs.w - vm1 * vm1);
                float cLum = luminance(f.prevIllum[i].xyz());
                float phiInv = 1.0f / std::fmax(1.0e-4f, p.phiLuminance * std::sqrt(var));
                float nwp = normal_weight_param(1.0f, p.lobeAngleFraction);
                float sumW = 0.0f;
                F4 sum(0.0f);
                float dthr = p.depthThreshold * z;
                for (int cx = -1; cx <= 1; ++cx)
                    for (int cy = -1; cy <= 1; ++cy) {
                        const int px = x + cx, py = y + cy;
                        const bool isC = cx == 0 && cy == 0;
                        const bool inside = px >= 0 && py >= 0 && px < W && py < H;
                        const float kernel = inside ? k3[std::abs(cx)] * k3[std::abs(cy)] : 0.0f;
                        const size_t j = (size_t)cl(py, H) * W + cl(px, W);
                        const F3 sN = f.normalRough[j].xyz();
                        const F3 sWP = wpm[j].xyz();
                        const float sMat = wpm[j].w;
                        float geo = plane_weight(cWP, cN, sWP, dthr);
                        geo *= kernel;
                        float nw = nonexp_weight(acos_approx(dot(cN, sN)), nwp, 0.0f);
                        F4 si = f.prevIllum[j];
                        float sLum = luminance(si.xyz());
                        float lw = std::fabs(cLum - sLum) * phiInv;
                        float w = geo * nw * std::exp(-lw);
                        w = isC ? kernel : w;
                        w *= (float)(sMat == cMat);
                        sumW += w;
                        sum += w * si;
                    }
                sumW = mymax(sumW, 1e-6f);
                sum /= sumW;
                float o1 = luminance(sum.xyz());
                float v2 = std::fmax(0.0f, sum.w - o1 * o1);
                f.ping[i] = F4(sum.xyz(), v2);
            } else {
                float sw = 0.0f, s1 = 0.0f, s2 = 0.0f;
                F3 si(0.0f);
                float nwp = normal_weight_param(1.0f, p.lobeAngleFraction);
                for (int cx = -2; cx <= 2; ++cx)
                    for (int cy = -2; cy <= 2; ++cy) {
                        const size_t j = (size_t)cl(y + cy, H) * W + cl(x + cx, W);
                        const F3 sN = f.normalRough[j].xyz();
                        const float sMat = wpm[j].w;
                        float nw = nonexp_weight(acos_approx(dot(cN, sN)), nwp, 0.0f);
                        F4 smp = f.prevIllum[j];
                        F3 sill = smp.xyz();
                        float sm1 = luminance(sill), sm2 = smp.w;
                        float w = nw * 1.0f;
                        w *= (float)(sMat == cMat);
                        sw += w;
                        si += sill * w;
                        s1 += sm1 * w;
                        s2 += sm2 * w;
                    }
                float boost = mymax(1.0f, 4.0f / (hist + 1.0f));
                sw = mymax(sw, 1e-6f);
                si /= sw;
                s1 /= sw;
                s2 /= sw;
                float var = std::fmax(0.0f, s2 - s1 * s1);
                var *= boost;
                f.ping[i] = F4(si, var);
            }
        }
}

// ---------------------------------------------------------------- D7
void pass_atrous(const Scene &s, Frame &f, const std::vector<F4> &in, std::vector<F4> &out, const DenoiseParams &p,
                 unsigned frameIndex, unsigned step) {
    const int W = f.W, H = f.H;
    const float k3[2] = {0.44198f, 0.27901f};
#pragma omp parallel for schedule(dynamic, 4)
    for (int y = f.by0(); y < f.by1(); ++y)
        for (int x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            const float z = f.depth[i];
            if (z > 500000.0f) continue;
            const float cMat = ld_ushort(f.material, f, x, y);
            const F3 cN = f.normalRough[i].xyz();
            const F3 cWP = world_pos(s.cam, x, y, z);
            const float hist = f.histLen[i];
            float lobe = p.lobeAngleFraction / std::sqrt((float)step);
            lobe = lerpf(0.99f, lobe, saturate(hist / 5.0f));
            const F4 c = in[i];
            const float cLum = luminance(c.xyz());
            const float phiInv = 1.0f / std::fmax(1.0e-4f, p.phiLuminance * std::sqrt(c.w));
            const float nwp = normal_weight_param(1.0f, lobe);
            float sumW = 0.44198f * 0.44198f;
            F4 sum = c * F4(F3(sumW), sumW * sumW);
            const float dthr = p.depthThreshold * z;
            int ofx = 0, ofy = 0;
            if (step > 4) {
                uint32_t st = rng_init((uint32_t)x, (uint32_t)y, frameIndex);
                st = seq_hash(st);
                uint32_t u0 = st;
                st = seq_hash(st);
                uint32_t u1 = st;
                F2 r(u0 / 4294967295.0f, u1 / 4294967295.0f);
                F2 o = F2((float)step) * 0.5f * (r - 0.5f);
                ofx = (int)o.x;
                ofy = (int)o.y;
            }
            const float maxRel = -std::log(saturate(0.0f));
            for (int yy = -1; yy <= 1; ++yy)
                for (int xx = -1; xx <= 1; ++xx) {
                    if (xx == 0 && yy == 0) continue;
                    const int px = x + ofx + xx * (int)step, py = y + ofy + yy * (int)step;
                    const bool inside = px >= 0 && py >= 0 && px < W && py < H;
                    const float kernel = k3[std::abs(xx)] * k3[std::abs(yy)];
                    const float sMat = ld_ushort(f.material, f, px, py);
                    const F3 sN = ld4(f.normalRough, f, px, py).xyz();
                    const float sz = ld1(f.depth, f, px, py);
                    const F3 sWP = world_pos(s.cam, px, py, sz);
                    float geo = plane_weight(cWP, cN, sWP, dthr);
                    geo *= kernel;
                    geo *= float(inside && sz < 500000.0f);
                    float nw = nonexp_weight(acos_approx(dot(cN, sN)), nwp, 0.0f);
                    float w = geo * nw;
                    w *= (float)(sMat == cMat);
                    if (w > 1e-4f) {
                        F4 sv = ld4(in, f, px, py);
                        float sLum = luminance(sv.xyz());
                        float lw = std::fabs(cLum - sLum) * phiInv;
                        lw = std::fmin(maxRel, lw);
                        w *= std::exp(-lw);
                        sumW += w;
                        sum += F4(F3(w), w * w) * sv;
                    }
                }
            out[i] = sum / F4(F3(sumW), sumW * sumW);
        }
}

// ---------------------------------------------------------------- D8
void pass_copy_nonsky(Frame &f, const std::vector<F4> &in) {
    for (size_t i = (size_t)f.by0() * f.W; i < (size_t)f.by1() * f.W; ++i)
        if (!(f.depth[i] > kRange)) f.output[i] = F4(in[i].xyz() * f.albedo[i].xyz(), 0.0f);
}
// frame 0 (Denoiser.cu:121-142): history := noisy input, zero history length (band rows)
void pass_frame0(Frame &f) {
    for (size_t i = (size_t)f.by0() * f.W; i < (size_t)f.by1() * f.W; ++i) {
        f.prevIllum[i] = f.illum[i];
        f.prevFast[i] = f.illum[i];
        f.histLen[i] = 0.0f;
        f.prevHistLen[i] = 0.0f;
    }
}
void pass_history_copies(Frame &f) {
    f.prevNormalRough = f.normalRough;
    f.prevDepth = f.depth;
    f.prevMaterial = f.material;
}

// ---------------------------------------------------------------- D0
void denoise_frame(const Scene &s, Frame &f, const DenoiseParams &p, int frameNum, int it) {
    const int used = it > 0 ? it - 1 : 0;
    if (p.enableFireflyFilter) pass_firefly(s, f, used & 1, p.phiLuminance);
    pass_copy_sky(f);
    if (frameNum == 0) pass_frame0(f);
    int fin = 0;
    if (p.enableTemporalAccumulation && frameNum > 0) {
        pass_temporal(s, f, p);
        fin = 1;
        if (p.enableHistoryFix) { pass_history_fix(s, f); fin = 2; }
        if (p.enableHistoryClamping) { pass_history_clamp(f); fin = 3; }
    }
    if (p.enableSpatialFiltering) {
        pass_atrous_smem(s, f, p);
        fin = 1;
        if (p.atrousIterationNum > 0) {
            int idx = 1;
            unsigned step = 1u << idx;
            const int maxIt = p.atrousIterationNum * 2;
            while (idx < maxIt) {
                pass_atrous(s, f, f.ping, f.pong, p, (unsigned)it, step);
                ++idx; step = 1u << idx;
                pass_atrous(s, f, f.pong, f.ping, p, (unsigned)it, step);
                ++idx; step = 1u << idx;
            }
            pass_atrous(s, f, f.ping, f.pong, p, (unsigned)it, step);
            fin = 2;
        }
    }
    const std::vector<F4> &fo = fin == 1 ? f.ping : (fin == 2 ? f.pong : (fin == 3 ? f.prevIllum : f.illum));
    pass_copy_nonsky(f, fo);
    pass_history_copies(f);
}

}  // namespace orc
