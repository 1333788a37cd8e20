// ORACLE (test infrastructure only -- never linked into the product path).
// Instanced block meshes in the path tracer (the rendering half):
//   brute-force ray queries over every instance row and triangle (the reference's IAS query,
//   closesthit.cu / RayGen.cu:49-52 with CULL_BACK for radiance rays, closesthit.cu:616-625
//   without culling for visibility rays), Moller-Trumbore in plain IEEE arithmetic in the
//   order meshes.hip evaluates it;
//   the general self-intersection-safe spawn of a triangle hit under its instance's
//   translation (SelfHit.h:150-193, 539-656; closesthit.cu:38-73);
//   TriangleLight::Create of a light record (Light.h:85-122).
// Defined semantics: the barycentrics are this test's (OptiX's are not reproducible); rsqrtf in
// SelfHit's normalisations is the correctly rounded 1 / sqrt; the directed roundings are
// emulated through binary64 exactly as the HIP side does (orc_math.h round_up_f).
#include <cmath>
#include <cstdint>
#include <cstring>

#include "orc_trace.h"

extern "C" float orc_f16_to_f32(uint32_t h);
extern "C" void orc_oct_decode(uint32_t u, float out[3]);

namespace orc {
namespace {

float dt3(const F3 &a, const F3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
F3 cr3(const F3 &a, const F3 &b) { return F3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }

bool tri_hit(const F3 &o, const F3 &d, const float *t9, float tmin, float tmax, bool cull, float &t, float &u,
             float &v) {
    const F3 v0(t9[0], t9[1], t9[2]), v1(t9[3], t9[4], t9[5]), v2(t9[6], t9[7], t9[8]);
    const F3 e1 = v1 - v0, e2 = v2 - v0;
    const F3 p = cr3(d, e2);
    const float det = dt3(e1, p);
    if (cull ? !(det > 0.0f) : !(det != 0.0f)) return false;
    const float inv = 1.0f / det;
    const F3 s = o - v0;
    const float uu = dt3(s, p) * inv;
    if (!(uu >= 0.0f && uu <= 1.0f)) return false;
    const F3 q = cr3(s, e1);
    const float vv = dt3(d, q) * inv;
    if (!(vv >= 0.0f && uu + vv <= 1.0f)) return false;
    const float tt = dt3(e2, q) * inv;
    if (!(tt >= tmin && tt <= tmax)) return false;
    t = tt; u = uu; v = vv;
    return true;
}

// SelfIntersectionAvoidance helpers (SelfHit.h:69-127)
float dot_rn(const F3 &u, const F3 &v) { return std::fma(u.x, v.x, std::fma(u.y, v.y, u.z * v.z)); }
float dot_abs_rn(const F3 &u, const F3 &v) {
    return std::fma(std::fabs(u.x), std::fabs(v.x), std::fma(std::fabs(u.y), std::fabs(v.y), std::fabs(u.z) * std::fabs(v.z)));
}
float fmmsf(float a, float b, float c, float d) {
    const float cd = c * d;
    const float e = std::fma(-c, d, cd);
    const float f = std::fma(a, b, -cd);
    return f + e;
}
F3 sia_cross(const F3 &a, const F3 &b) {
    return F3(fmmsf(a.y, b.z, a.z, b.y), fmmsf(a.z, b.x, a.x, b.z), fmmsf(a.x, b.y, a.y, b.x));
}
float rsqrt_rn(float x) { return 1.0f / std::sqrt(x); }
F3 sia_normalize(const F3 &u) {
    const float s = rsqrt_rn(dot_rn(u, u));
    return F3(u.x * s, u.y * s, u.z * s);
}
// a*b + c*d + e*f with the inner terms of the instance matrices written out (rows of the identity)
float row_apply(float r0, float r1, float r2, const F3 &p) { return std::fma(r0, p.x, std::fma(r1, p.y, r2 * p.z)); }
float row_abs_ru(float r0, float r1, float r2, const F3 &p) {
    return fma_ru(std::fabs(p.x), std::fabs(r0), fma_ru(std::fabs(p.y), std::fabs(r1), mul_ru(std::fabs(p.z), std::fabs(r2))));
}
float sub_ru(float a, float b) { return add_ru(a, -b); }

}  // namespace

MeshHit mesh_closest_hit(const MeshSet &m, const F3 &o, const F3 &d, float tmax) {
    MeshHit b;
    b.t = tmax;
    for (int i = 0; i < (int)m.inst.size(); ++i) {
        const MeshInstance &mi = m.inst[i];
        const int n = m.triCnt[mi.block];
        if (n == 0) continue;
        const F3 oo(o.x - mi.cell.x, o.y - mi.cell.y, o.z - mi.cell.z);
        for (int k = 0; k < n; ++k) {
            float t, u, v;
            if (!tri_hit(oo, d, &m.pos[((size_t)m.triOff[mi.block] + k) * 9], 0.0f, b.t, true, t, u, v)) continue;
            if (b.hit && !(t < b.t)) continue;
            b.hit = true; b.t = t; b.u = u; b.v = v; b.row = i; b.tri = k;
        }
    }
    return b;
}

bool mesh_any_hit(const MeshSet &m, const F3 &o, const F3 &d, float tmin, float tmax) {
    for (const MeshInstance &mi : m.inst) {
        const int n = m.triCnt[mi.block];
        const F3 oo(o.x - mi.cell.x, o.y - mi.cell.y, o.z - mi.cell.z);
        for (int k = 0; k < n; ++k) {
            float t, u, v;
            if (tri_hit(oo, d, &m.pos[((size_t)m.triOff[mi.block] + k) * 9], tmin, tmax, false, t, u, v)) return true;
        }
    }
    return false;
}

void mesh_spawn(const MeshSet &m, const MeshHit &h, F3 &front, F3 &back, F3 &normal) {
    const MeshInstance &mi = m.inst[h.row];
    const float *t9 = &m.pos[((size_t)m.triOff[mi.block] + h.tri) * 9];
    const F3 v0(t9[0], t9[1], t9[2]), v1(t9[3], t9[4], t9[5]), v2(t9[6], t9[7], t9[8]);
    // getSafeTriangleSpawnOffset (object space)
    const F3 e1(v1.x - v0.x, v1.y - v0.y, v1.z - v0.z), e2(v2.x - v0.x, v2.y - v0.y, v2.z - v0.z);
    const F3 objP(v0.x + std::fma(h.u, e1.x, h.v * e2.x), v0.y + std::fma(h.u, e1.y, h.v * e2.y),
                  v0.z + std::fma(h.u, e1.z, h.v * e2.z));
    const float c0 = 5.9604648328104529e-08f, c1 = 1.1920930376163769e-07f;
    const float epsX = mul_ru(c1, add_ru(add_ru(std::fabs(e1.x), std::fabs(e2.x)), std::fabs(sub_ru(e1.x, e2.x))));
    const float epsY = mul_ru(c1, add_ru(add_ru(std::fabs(e1.y), std::fabs(e2.y)), std::fabs(sub_ru(e1.y, e2.y))));
    const float epsZ = mul_ru(c1, add_ru(add_ru(std::fabs(e1.z), std::fabs(e2.z)), std::fabs(sub_ru(e1.z, e2.z))));
    const float eps = std::fmax(std::fmax(epsX, epsY), epsZ);
    const F3 triErr(fma_ru(c0, std::fabs(v0.x), eps), fma_ru(c0, std::fabs(v0.y), eps), fma_ru(c0, std::fabs(v0.z), eps));
    F3 n = sia_normalize(sia_cross(e1, e2));
    float off = dot_abs_rn(triErr, n);
    // one instance transform: object to world = translation by the cell, world to object = -cell
    const F3 T = mi.cell;
    const float cI = 1.19209317972490680404007434844970703125E-7f;
    const F3 wldP(row_apply(1.0f, 0.0f, 0.0f, objP) + T.x, row_apply(0.0f, 1.0f, 0.0f, objP) + T.y,
                  row_apply(0.0f, 0.0f, 1.0f, objP) + T.z);
    const F3 wldErr(fma_ru(cI, row_abs_ru(1.0f, 0.0f, 0.0f, objP), mul_ru(cI, std::fabs(T.x))),
                    fma_ru(cI, row_abs_ru(0.0f, 1.0f, 0.0f, objP), mul_ru(cI, std::fabs(T.y))),
                    fma_ru(cI, row_abs_ru(0.0f, 0.0f, 1.0f, objP), mul_ru(cI, std::fabs(T.z))));
    const F3 wldN(row_apply(1.0f, 0.0f, 0.0f, n), row_apply(0.0f, 1.0f, 0.0f, n), row_apply(0.0f, 0.0f, 1.0f, n));
    const F3 objErr(fma_ru(cI, row_abs_ru(1.0f, 0.0f, 0.0f, wldP), fma_ru(cI, std::fabs(-T.x), 0.0f)),
                    fma_ru(cI, row_abs_ru(0.0f, 1.0f, 0.0f, wldP), fma_ru(cI, std::fabs(-T.y), 0.0f)),
                    fma_ru(cI, row_abs_ru(0.0f, 0.0f, 1.0f, wldP), fma_ru(cI, std::fabs(-T.z), 0.0f)));
    off = add_ru(dot_abs_rn(objErr, n), off);
    n = wldN;
    const float rcp = rsqrt_rn(dot_rn(n, n));
    n = F3(n.x * rcp, n.y * rcp, n.z * rcp);
    off = std::fma(off, rcp, dot_abs_rn(wldErr, n));
    // offsetSpawnPoint: round away from the surface
    const float p[3] = {wldP.x, wldP.y, wldP.z}, dn[3] = {n.x, n.y, n.z};
    float fr[3], bk[3];
    for (int a = 0; a < 3; ++a) {
        fr[a] = dn[a] > 0.f ? fma_ru(off, dn[a], p[a]) : fma_rd(off, dn[a], p[a]);
        bk[a] = dn[a] > 0.f ? fma_rd(-off, dn[a], p[a]) : fma_ru(-off, dn[a], p[a]);
    }
    front = F3(fr[0], fr[1], fr[2]);
    back = F3(bk[0], bk[1], bk[2]);
    normal = n;
}

F2 mesh_texcoord(const MeshSet &m, const MeshHit &h) {
    const MeshInstance &mi = m.inst[h.row];
    const float *t6 = &m.uv[((size_t)m.triOff[mi.block] + h.tri) * 6];
    const float alpha = 1.0f - h.u - h.v;
    const F2 a(t6[0], t6[1]), b(t6[2], t6[3]), c(t6[4], t6[5]);
    return a * alpha + b * h.u + c * h.v;
}

TriLight tri_light(const MeshSet &m, int k) {
    const uint32_t *r = &m.lights[(size_t)k * 8];
    TriLight L;
    const float f0 = orc_f16_to_f32(r[3] & 0xFFFFu), f1 = orc_f16_to_f32(r[3] >> 16);
    float d1[3], d2[3];
    orc_oct_decode(r[6], d1);
    orc_oct_decode(r[7], d2);
    L.edge1 = F3(d1[0], d1[1], d1[2]) * f0;
    L.edge2 = F3(d2[0], d2[1], d2[2]) * f1;
    float c[3];
    std::memcpy(c, r, 12);
    L.base = F3(c[0], c[1], c[2]) - (L.edge1 + L.edge2) / 3.0f;
    L.radiance = F3(orc_f16_to_f32(r[4] & 0xFFFFu), orc_f16_to_f32(r[4] >> 16), orc_f16_to_f32(r[5] & 0xFFFFu));
    const F3 ln = cross(L.edge1, L.edge2);
    const float len = length(ln);
    if (len > 0.0f) {
        L.area = 0.5f * len;
        L.normal = ln / len;
    } else {
        L.area = 0.0f;
        L.normal = F3(0.0f);
    }
    return L;
}

}  // namespace orc
