// vxpt -- device-side instanced-mesh queries and hit geometry, shared by
// meshes.hip (the probe kernels) and trace.hip (the path kernels).  See meshes.hip for the BVH
// walk's design notes.  The walk is host + device code: the CPU tests run it on the host
// (tests/native/mesh_walk_driver.hip).
#pragma once
#include "vx_internal.hpp"

namespace vx {
namespace {

VX_HD float dt3(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
VX_HD V3 cr3(V3 a, V3 b) { return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }

VX_HD bool tri_hit(V3 o, V3 d, const float *t9, float tmin, float tmax, int cull, float &t, float &u, float &v) {
    const V3 v0(t9[0], t9[1], t9[2]), v1(t9[3], t9[4], t9[5]), v2(t9[6], t9[7], t9[8]);
    const V3 e1 = v1 - v0, e2 = v2 - v0;
    const V3 p = cr3(d, e2);
    const float det = dt3(e1, p);
    if (cull ? !(det > 0.0f) : !(det != 0.0f)) return false;
    const float inv = 1.0f / det;
    const V3 s = o - v0;
    const float uu = dt3(s, p) * inv;
    if (!(uu >= 0.0f && uu <= 1.0f)) return false;
    const V3 q = cr3(s, e1);
    const float vv = dt3(d, q) * inv;
    if (!(vv >= 0.0f && uu + vv <= 1.0f)) return false;
    const float tt = dt3(e2, q) * inv;
    if (!(tt >= tmin && tt <= tmax)) return false;
    t = tt; u = uu; v = vv;
    return true;
}

// slab test against a widened box; an axis the ray does not move along only checks the origin
VX_HD bool box_hit(const BvhNode &n, V3 o, V3 inv, V3 d, float tmin, float tmax, float &tEnter) {
    float t0 = tmin, t1 = tmax;
    const float oo[3] = {o.x, o.y, o.z}, ii[3] = {inv.x, inv.y, inv.z}, dd[3] = {d.x, d.y, d.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (dd[k] == 0.0f) {
            if (oo[k] < n.lo[k] || oo[k] > n.hi[k]) return false;
            continue;
        }
        const float a = (n.lo[k] - oo[k]) * ii[k], b = (n.hi[k] - oo[k]) * ii[k];
        t0 = fmaxf(t0, fminf(a, b));
        t1 = fminf(t1, fmaxf(a, b));
    }
    tEnter = t0;
    return t0 <= t1;
}

// The walk keeps ONE per-thread stack for both levels: a BLAS walk runs on the entries above the
// TLAS's pending ones and is done before the TLAS walk pops again (live entries <= tlasDepth +
// blasDepth + 1).  An entry is (node, entry distance of its box): a popped node whose box starts
// past the current closest hit is dropped without loading it, and a node that is loaded is not
// box-tested again (its test at push time with the then-current interval stays valid: a later,
// shorter interval that still reaches the entry distance contains the box's entry point).  It lives
// in scratch: a 24-entry LDS stack (entry k of lane t at lds[k * 256 + t], conflict-free) was
// measured 4 % slower on tools/mesh_probe_bench.py (16.0 vs 15.4 ms) -- 24 KiB per block cut
// occupancy from 8 to 6 waves/SIMD, and the walk is bound by the node and triangle loads, not by
// the stack.
struct ScratchStack {
    int s[84];    // node index; 2 x (the builder's depth limit 40 + 2)
    float t[84];  // its box's entry distance
};

template <class S>
VX_HD void stack_push(S &st, int &sp, int node, float te) {
    st.s[sp] = node;
    st.t[sp] = te;
    ++sp;
}

// push the children of an inner node, the nearer one on top (visited first, so the closest hit
// shrinks the interval early); a child whose box the ray misses is not pushed
template <class S>
VX_HD void push_children(const BvhNode *nodes, int base, int left, V3 o, V3 inv, V3 d, float tmin, float tmax,
                        S &stack, int &sp) {
    float ta, tb;
    const bool ha = box_hit(nodes[base + left], o, inv, d, tmin, tmax, ta);
    const bool hb = box_hit(nodes[base + left + 1], o, inv, d, tmin, tmax, tb);
    if (ha && hb) {
        const bool aFirst = ta <= tb;
        stack_push(stack, sp, base + (aFirst ? left + 1 : left), aFirst ? tb : ta);
        stack_push(stack, sp, base + (aFirst ? left : left + 1), aFirst ? ta : tb);
    } else if (ha) {
        stack_push(stack, sp, base + left, ta);
    } else if (hb) {
        stack_push(stack, sp, base + left + 1, tb);
    }
}

struct Best {
    float t, u, v;
    int inst, tri;
    int leaf;  // the triangle's index in BLAS leaf order (its vertices at MeshDev::tri + 9 * leaf)
    VX_HD bool better(float tt, int i, int k) const {
        return inst < 0 || tt < t || (tt == t && (i < inst || (i == inst && k < tri)));
    }
};

template <bool kAny, class S>
VX_HD bool blas_walk(const MeshDev &m, int row, int block, V3 o, V3 d, V3 inv, float tmin, int cull, Best &b,
                    S &stack, const int sp0) {
    const int2 r = m.root[block];
    if (r.x < 0) return false;
    float te0;
    if (!box_hit(m.blas[r.x], o, inv, d, tmin, b.t, te0)) return false;
    int sp = sp0;
    stack_push(stack, sp, r.x, te0);
    while (sp > sp0) {
        --sp;
        if (stack.t[sp] > b.t) continue;
        const BvhNode n = m.blas[stack.s[sp]];
        if (n.count == 0) {
            push_children(m.blas, r.x, n.left, o, inv, d, tmin, b.t, stack, sp);
            continue;
        }
        for (int k = 0; k < n.count; ++k) {
            const int ti = r.y + n.left + k;
            float t, u, v;
            if (tri_hit(o, d, m.tri + (size_t)ti * 9, tmin, b.t, cull, t, u, v)) {
                const int id = m.triId[ti];
                if (kAny) { b.t = t; b.u = u; b.v = v; b.inst = row; b.tri = id; b.leaf = ti; return true; }
                if (b.better(t, row, id)) { b.t = t; b.u = u; b.v = v; b.inst = row; b.tri = id; b.leaf = ti; }
            }
        }
    }
    return false;
}

template <bool kAny, class S>
VX_HD void mesh_walk(const MeshDev &m, V3 o, V3 d, V3 inv, float tmin, int cull, Best &b, S &stack) {
    if (m.nInst <= 0) return;
    float te0;
    if (!box_hit(m.tlas[0], o, inv, d, tmin, b.t, te0)) return;
    int sp = 0;
    stack_push(stack, sp, 0, te0);
    while (sp > 0) {
        --sp;
        if (stack.t[sp] > b.t) continue;
        const BvhNode nd = m.tlas[stack.s[sp]];
        if (nd.count == 0) {
            push_children(m.tlas, 0, nd.left, o, inv, d, tmin, b.t, stack, sp);
            continue;
        }
        for (int k = 0; k < nd.count; ++k) {
            const MeshInst mi = m.inst[nd.left + k];
            const V3 oo(o.x - mi.cell[0], o.y - mi.cell[1], o.z - mi.cell[2]);
            if (blas_walk<kAny>(m, mi.row, mi.block, oo, d, inv, tmin, cull, b, stack, sp)) return;
        }
    }
}


// ---------------------------------------------------------------- mesh hit geometry
// SelfIntersectionAvoidance (SelfHit.h:69-193, 539-656) for a triangle of an instance whose
// transform is a translation by its cell: object-space point and error bound, normal, the
// instance transform's error terms, then offsetSpawnPoint.  The oracle (orc_mesh.cpp) states the
// same operations; rsqrtf is the correctly rounded 1 / sqrt there and here.
VX_D float sia_dot_rn(V3 u, V3 v) { return fmaf(u.x, v.x, fmaf(u.y, v.y, u.z * v.z)); }
VX_D float sia_dot_abs_rn(V3 u, V3 v) {
    return fmaf(fabsf(u.x), fabsf(v.x), fmaf(fabsf(u.y), fabsf(v.y), fabsf(u.z) * fabsf(v.z)));
}
VX_D V3 sia_normalize(V3 u) {
    const float s = 1.0f / sqrtf(sia_dot_rn(u, u));
    return V3(u.x * s, u.y * s, u.z * s);
}
VX_D float row_apply(float r0, float r1, float r2, V3 p) { return fmaf(r0, p.x, fmaf(r1, p.y, r2 * p.z)); }
VX_D float row_abs_ru(float r0, float r1, float r2, V3 p) {
    return fma_ru(fabsf(p.x), fabsf(r0), fma_ru(fabsf(p.y), fabsf(r1), mul_ru(fabsf(p.z), fabsf(r2))));
}
VX_D float sub_ru(float a, float b) { return add_ru(a, -b); }

VX_D void mesh_spawn(V3 v0, V3 v1, V3 v2, float bu, float bv, V3 T, V3 &front, V3 &back, V3 &normal) {
    const V3 e1(v1.x - v0.x, v1.y - v0.y, v1.z - v0.z), e2(v2.x - v0.x, v2.y - v0.y, v2.z - v0.z);
    const V3 objP(v0.x + fmaf(bu, e1.x, bv * e2.x), v0.y + fmaf(bu, e1.y, bv * e2.y), v0.z + fmaf(bu, e1.z, bv * e2.z));
    const float c0 = 5.9604648328104529e-08f, c1 = 1.1920930376163769e-07f;
    const float epsX = mul_ru(c1, add_ru(add_ru(fabsf(e1.x), fabsf(e2.x)), fabsf(sub_ru(e1.x, e2.x))));
    const float epsY = mul_ru(c1, add_ru(add_ru(fabsf(e1.y), fabsf(e2.y)), fabsf(sub_ru(e1.y, e2.y))));
    const float epsZ = mul_ru(c1, add_ru(add_ru(fabsf(e1.z), fabsf(e2.z)), fabsf(sub_ru(e1.z, e2.z))));
    const float eps = fmaxf(fmaxf(epsX, epsY), epsZ);
    const V3 triErr(fma_ru(c0, fabsf(v0.x), eps), fma_ru(c0, fabsf(v0.y), eps), fma_ru(c0, fabsf(v0.z), eps));
    V3 n = sia_normalize(V3(dop(e1.y, e2.z, e1.z, e2.y), dop(e1.z, e2.x, e1.x, e2.z), dop(e1.x, e2.y, e1.y, e2.x)));
    float off = sia_dot_abs_rn(triErr, n);
    const float cI = 1.19209317972490680404007434844970703125E-7f;
    const V3 wldP(row_apply(1.0f, 0.0f, 0.0f, objP) + T.x, row_apply(0.0f, 1.0f, 0.0f, objP) + T.y,
                  row_apply(0.0f, 0.0f, 1.0f, objP) + T.z);
    const V3 wldErr(fma_ru(cI, row_abs_ru(1.0f, 0.0f, 0.0f, objP), mul_ru(cI, fabsf(T.x))),
                    fma_ru(cI, row_abs_ru(0.0f, 1.0f, 0.0f, objP), mul_ru(cI, fabsf(T.y))),
                    fma_ru(cI, row_abs_ru(0.0f, 0.0f, 1.0f, objP), mul_ru(cI, fabsf(T.z))));
    const V3 wldN(row_apply(1.0f, 0.0f, 0.0f, n), row_apply(0.0f, 1.0f, 0.0f, n), row_apply(0.0f, 0.0f, 1.0f, n));
    const V3 objErr(fma_ru(cI, row_abs_ru(1.0f, 0.0f, 0.0f, wldP), fma_ru(cI, fabsf(-T.x), 0.0f)),
                    fma_ru(cI, row_abs_ru(0.0f, 1.0f, 0.0f, wldP), fma_ru(cI, fabsf(-T.y), 0.0f)),
                    fma_ru(cI, row_abs_ru(0.0f, 0.0f, 1.0f, wldP), fma_ru(cI, fabsf(-T.z), 0.0f)));
    off = add_ru(sia_dot_abs_rn(objErr, n), off);
    n = wldN;
    const float rcp = 1.0f / sqrtf(sia_dot_rn(n, n));
    n = V3(n.x * rcp, n.y * rcp, n.z * rcp);
    off = fmaf(off, rcp, sia_dot_abs_rn(wldErr, n));
    front = V3(n.x > 0.f ? fma_ru(off, n.x, wldP.x) : fma_rd(off, n.x, wldP.x),
               n.y > 0.f ? fma_ru(off, n.y, wldP.y) : fma_rd(off, n.y, wldP.y),
               n.z > 0.f ? fma_ru(off, n.z, wldP.z) : fma_rd(off, n.z, wldP.z));
    back = V3(n.x > 0.f ? fma_rd(-off, n.x, wldP.x) : fma_ru(-off, n.x, wldP.x),
              n.y > 0.f ? fma_rd(-off, n.y, wldP.y) : fma_ru(-off, n.y, wldP.y),
              n.z > 0.f ? fma_rd(-off, n.z, wldP.z) : fma_ru(-off, n.z, wldP.z));
    normal = n;
}

// ---------------------------------------------------------------- triangle lights
// __half2float and octToNdirUnorm32 (LinearMath.h:2069-2089) of a LightInfo record
VX_D float f16_float(uint32_t b) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(b & 0xFFFFu)); }
VX_D V3 oct_decode(uint32_t u) {
    float px = saturate((float)(u & 0xFFFFu) / 65534.0f), py = saturate((float)(u >> 16) / 65534.0f);
    px = px * 2.0f - 1.0f;
    py = py * 2.0f - 1.0f;
    V3 n(px, py, 1.0f - fabsf(px) - fabsf(py));
    const float t = fmaxf(0.0f, -n.z);
    n.x += n.x >= 0.0f ? -t : t;
    n.y += n.y >= 0.0f ? -t : t;
    return normalize(n);
}
// TriangleLight::Create (Light.h:85-122)
struct TriL { V3 base, e1, e2, rad, n; float area; };
VX_D TriL tri_light(const LightInfo &li) {
    TriL t;
    t.e1 = oct_decode(li.direction1) * f16_float(li.scalars);
    t.e2 = oct_decode(li.direction2) * f16_float(li.scalars >> 16);
    t.base = V3(li.center[0], li.center[1], li.center[2]) - (t.e1 + t.e2) / 3.0f;
    t.rad = V3(f16_float(li.radiance[0]), f16_float(li.radiance[0] >> 16), f16_float(li.radiance[1]));
    const V3 ln = cross(t.e1, t.e2);
    const float len = length(ln);
    if (len > 0.0f) { t.area = 0.5f * len; t.n = ln / len; }
    else { t.area = 0.0f; t.n = V3(0.0f); }
    return t;
}

}  // namespace
}  // namespace vx
