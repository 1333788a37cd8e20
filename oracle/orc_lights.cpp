// ORACLE (test infrastructure only -- never linked into the product path).
// CPU restatement of the reference's emissive-triangle light table for the instanced
// meshes:
//   VoxelEngine.cu:33-39    applyTransform (3x4 row-major, evaluated as written)
//   VoxelEngine.cu:53-116   generateLightInfosKernel: one record per (instance, triangle)
//   Light.h:85-137          TriangleLight::Create / Store (f16 scalars and radiance,
//                           octahedral unorm16x2 edge directions)
//   LinearMath.h:2069-2122  octahedral encode / decode
//   VoxelEngine.cu:139-147  extractRadianceKernel: weight = luminance(radiance) * area of the
//                           decoded record
// The f32 -> f16 conversion (__float2half_rn) is restated in software: round to nearest
// even, subnormal halves, overflow to infinity.
#include <cmath>
#include <cstdint>
#include <cstring>

#include "orc_math.h"

using namespace orc;

namespace {

uint32_t f32_to_f16(float f) {
    uint32_t x;
    std::memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t ax = x & 0x7FFFFFFFu;
    if (ax >= 0x7F800000u) return sign | (ax > 0x7F800000u ? 0x7E00u : 0x7C00u);  // NaN / inf
    if (ax >= 0x477FF000u) return sign | 0x7C00u;                                 // rounds past 65504
    if (ax < 0x33000000u) return sign;                                             // < 2^-25: to zero
    int e = (int)(ax >> 23) - 127;
    uint32_t m = (ax & 0x7FFFFFu) | 0x800000u;  // 24-bit significand
    uint32_t shift, base;
    if (e < -14) {  // subnormal half: value = m * 2^(e-23), unit 2^-24
        shift = (uint32_t)(-14 - e) + 13;
        base = 0;
    } else {
        shift = 13;
        base = (uint32_t)(e + 15) << 10;
        m &= 0x7FFFFFu;
    }
    uint32_t q = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1u), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (q & 1u))) ++q;
    return sign | (base + q);  // a carry out of the mantissa bumps the exponent, as it should
}

float f16_to_f32(uint32_t h) {
    const uint32_t sign = (h & 0x8000u) << 16, e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
    float v;
    if (e == 0) v = std::ldexp((float)m, -24);
    else if (e == 31) v = m ? NAN : INFINITY;
    else v = std::ldexp((float)(m | 0x400u), (int)e - 25);
    uint32_t b;
    std::memcpy(&b, &v, 4);
    b |= sign;
    std::memcpy(&v, &b, 4);
    return v;
}

float sgn_nz(float v) { return v >= 0.0f ? 1.0f : -1.0f; }

uint32_t oct_encode(const F3 &n) {
    const float inv = 1.0f / (std::fabs(n.x) + std::fabs(n.y) + std::fabs(n.z));
    float px = n.x * inv, py = n.y * inv;
    if (n.z < 0.0f) {
        const float wx = (1.0f - std::fabs(py)) * sgn_nz(px), wy = (1.0f - std::fabs(px)) * sgn_nz(py);
        px = wx;
        py = wy;
    }
    px = saturate(px * 0.5f + 0.5f);
    py = saturate(py * 0.5f + 0.5f);
    return (uint32_t)(px * 65534.0f) | ((uint32_t)(py * 65534.0f) << 16);
}

F3 oct_decode(uint32_t u) {
    float px = saturate((float)(u & 0xFFFFu) / 65534.0f), py = saturate((float)(u >> 16) / 65534.0f);
    px = px * 2.0f - 1.0f;
    py = py * 2.0f - 1.0f;
    F3 n(px, py, 1.0f - std::fabs(px) - std::fabs(py));
    const float t = std::fmax(0.0f, -n.z);
    n.x += n.x >= 0.0f ? -t : t;
    n.y += n.y >= 0.0f ? -t : t;
    return normalize(n);
}

}  // namespace

extern "C" {

uint32_t orc_f32_to_f16(float f) { return f32_to_f16(f); }
float orc_f16_to_f32(uint32_t h) { return f16_to_f32(h); }
uint32_t orc_oct_encode(const float n[3]) { return oct_encode(F3(n[0], n[1], n[2])); }
void orc_oct_decode(uint32_t u, float out[3]) {
    const F3 n = oct_decode(u);
    out[0] = n.x; out[1] = n.y; out[2] = n.z;
}

// records: 8 x u32 per light (center xyz as f32 bits, scalars, radiance lo/hi, direction1, direction2)
void orc_tri_lights(const float *tri, int nTri, const int *inst, int nInst, const float rad[3], uint32_t *out,
                    float *weight) {
    for (int ii = 0; ii < nInst; ++ii)
        for (int ti = 0; ti < nTri; ++ti) {
            const float t[12] = {1.0f, 0.0f, 0.0f, (float)inst[ii * 3],
                                 0.0f, 1.0f, 0.0f, (float)inst[ii * 3 + 1],
                                 0.0f, 0.0f, 1.0f, (float)inst[ii * 3 + 2]};
            F3 v[3];
            for (int k = 0; k < 3; ++k) {
                const float *p = tri + (size_t)ti * 9 + k * 3;
                v[k] = F3(t[0] * p[0] + t[1] * p[1] + t[2] * p[2] + t[3], t[4] * p[0] + t[5] * p[1] + t[6] * p[2] + t[7],
                          t[8] * p[0] + t[9] * p[1] + t[10] * p[2] + t[11]);
            }
            const F3 e1 = v[1] - v[0], e2 = v[2] - v[0];
            const F3 c = v[0] + (e1 + e2) / 3.0f;
            uint32_t *o = out + ((size_t)ii * nTri + ti) * 8;
            std::memcpy(o, &c.x, 4);
            std::memcpy(o + 1, &c.y, 4);
            std::memcpy(o + 2, &c.z, 4);
            o[3] = f32_to_f16(length(e1)) | (f32_to_f16(length(e2)) << 16);
            o[4] = f32_to_f16(rad[0]) | (f32_to_f16(rad[1]) << 16);
            o[5] = f32_to_f16(rad[2]) | (f32_to_f16(0.0f) << 16);
            o[6] = oct_encode(normalize(e1));
            o[7] = oct_encode(normalize(e2));
            const F3 d1 = oct_decode(o[6]) * f16_to_f32(o[3] & 0xFFFFu), d2 = oct_decode(o[7]) * f16_to_f32(o[3] >> 16);
            const F3 r(f16_to_f32(o[4] & 0xFFFFu), f16_to_f32(o[4] >> 16), f16_to_f32(o[5] & 0xFFFFu));
            const float nl = length(cross(d1, d2));
            const float area = nl > 0.0f ? 0.5f * nl : 0.0f;
            weight[(size_t)ii * nTri + ti] = luminance(r) * area;
        }
}

// Instanced-mesh closest hit by brute force (the reference's IAS query; meshes.hip walks a BVH
// and must agree exactly): every instance row in order, the ray origin translated by -cell
// (the instance transform), Moller-Trumbore with plain IEEE arithmetic in the kernel's order,
// the first strictly closer hit wins (= ties to the smaller row, then triangle).
void orc_mesh_probe(const float *tris, const int *triOff, const int *triCnt, const float *cells, int nInst,
                    const float *rays, int n, int cull, float *out, int *ids) {
    auto dt3 = [](const F3 &a, const F3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; };
    auto cr3 = [](const F3 &a, const F3 &b) {
        return F3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
    };
    for (int r = 0; r < n; ++r) {
        const float *ry = rays + (size_t)r * 8;
        const F3 o(ry[0], ry[1], ry[2]), d(ry[4], ry[5], ry[6]);
        const float tmin = ry[3];
        float bt = ry[7], bu = 0.0f, bv = 0.0f;
        int bi = -1, bk = -1;
        for (int i = 0; i < nInst; ++i) {
            const F3 oo(o.x - cells[i * 3], o.y - cells[i * 3 + 1], o.z - cells[i * 3 + 2]);
            for (int k = 0; k < triCnt[i]; ++k) {
                const float *t9 = tris + ((size_t)triOff[i] + k) * 9;
                const F3 v0(t9[0], t9[1], t9[2]), v1(t9[3], t9[4], t9[5]), v2(t9[6], t9[7], t9[8]);
                const F3 e1 = v1 - v0, e2 = v2 - v0;
                const F3 p = cr3(d, e2);
                const float det = dt3(e1, p);
                if (cull ? !(det > 0.0f) : !(det != 0.0f)) continue;
                const float inv = 1.0f / det;
                const F3 s = oo - v0;
                const float u = dt3(s, p) * inv;
                if (!(u >= 0.0f && u <= 1.0f)) continue;
                const F3 q = cr3(s, e1);
                const float v = dt3(d, q) * inv;
                if (!(v >= 0.0f && u + v <= 1.0f)) continue;
                const float t = dt3(e2, q) * inv;
                if (!(t >= tmin && t <= bt)) continue;
                if (bi >= 0 && !(t < bt)) continue;
                bt = t; bu = u; bv = v; bi = i; bk = k;
            }
        }
        out[r * 4] = bt; out[r * 4 + 1] = bu; out[r * 4 + 2] = bv; out[r * 4 + 3] = bi >= 0 ? 1.0f : 0.0f;
        ids[r * 2] = bi; ids[r * 2 + 1] = bk;
    }
}

}  // extern "C"
