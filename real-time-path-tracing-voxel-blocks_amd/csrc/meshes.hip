// vxpt -- ray queries against the instanced block meshes (geometry half).
//
// The reference puts every instanced block's mesh into an OptiX IAS (one instance per cell,
// transform = translation by the cell, VoxelEngine.cu:323-384; OptixRenderer.cpp:723-770) and
// lets the RT cores find the closest triangle.  Here: a two-level BVH built on the host
// (vxpt_host.cpp build_mesh_bvh) and walked by one thread per ray -- TLAS over the instances'
// world boxes, then the instance's BLAS in object space with the ray origin translated by
// -cell (as the IAS transform does) -- with an explicit triangle test:
//   Moller-Trumbore, plain IEEE products and sums in a fixed order (the oracle repeats it
//   operation for operation), hit when det != 0 (det > 0 with back-face culling: the
//   reference's radiance rays cull back faces, its visibility rays do not), u, v >= 0,
//   u + v <= 1, tmin <= t <= tmax;
//   closest hit with a total order on ties (t, then instance row, then triangle), so the
//   traversal order cannot change the answer.
// Node boxes are widened on the host; box culling therefore never drops a triangle the test
// would accept, and the BVH walk equals the brute-force loop of the oracle exactly.
#include "vx_internal.hpp"

namespace vx {
namespace {

VX_D float dt3(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
VX_D V3 cr3(V3 a, V3 b) { return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }

VX_D bool tri_hit(V3 o, V3 d, const float *t9, float tmin, float tmax, int cull, float &t, float &u, float &v) {
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
VX_D bool box_hit(const BvhNode &n, V3 o, V3 inv, V3 d, float tmin, float tmax, float &tEnter) {
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

// push the children of an inner node, the nearer one on top (visited first, so the closest hit
// shrinks the interval early); a child whose box the ray misses is not pushed
template <class S>
VX_D void push_children(const BvhNode *nodes, int base, int left, V3 o, V3 inv, V3 d, float tmin, float tmax,
                        S &stack, int &sp) {
    float ta, tb;
    const bool ha = box_hit(nodes[base + left], o, inv, d, tmin, tmax, ta);
    const bool hb = box_hit(nodes[base + left + 1], o, inv, d, tmin, tmax, tb);
    if (ha && hb) {
        const bool aFirst = ta <= tb;
        stack[sp++] = base + (aFirst ? left + 1 : left);
        stack[sp++] = base + (aFirst ? left : left + 1);
    } else if (ha) {
        stack[sp++] = base + left;
    } else if (hb) {
        stack[sp++] = base + left + 1;
    }
}

// The walk keeps ONE per-thread stack for both levels: a BLAS walk runs on the entries above the
// TLAS's pending ones and is done before the TLAS walk pops again (live entries <= tlasDepth +
// blasDepth + 1).  It lives in scratch: a 24-entry LDS stack (entry k of lane t at
// lds[k * 256 + t], conflict-free) was measured 4 % slower on tools/mesh_probe_bench.py (16.0 vs
// 15.4 ms) -- 24 KiB per block cut occupancy from 8 to 6 waves/SIMD, and the walk is bound by
// the node and triangle loads, not by the stack.
struct ScratchStack {
    int s[84];  // 2 x (the builder's depth limit 40 + 2)
    VX_D int &operator[](int k) { return s[k]; }
};

struct Best {
    float t, u, v;
    int inst, tri;
    VX_D bool better(float tt, int i, int k) const {
        return inst < 0 || tt < t || (tt == t && (i < inst || (i == inst && k < tri)));
    }
};

template <bool kAny, class S>
VX_D bool blas_walk(const MeshDev &m, int row, int block, V3 o, V3 d, V3 inv, float tmin, int cull, Best &b,
                    S &stack, const int sp0) {
    const int2 r = m.root[block];
    if (r.x < 0) return false;
    int sp = sp0;
    stack[sp++] = r.x;
    while (sp > sp0) {
        const BvhNode n = m.blas[stack[--sp]];
        float te;
        if (!box_hit(n, o, inv, d, tmin, b.t, te)) continue;
        if (n.count == 0) {
            push_children(m.blas, r.x, n.left, o, inv, d, tmin, b.t, stack, sp);
            continue;
        }
        for (int k = 0; k < n.count; ++k) {
            const int ti = r.y + n.left + k;
            float t, u, v;
            if (tri_hit(o, d, m.tri + (size_t)ti * 9, tmin, b.t, cull, t, u, v)) {
                const int id = m.triId[ti];
                if (kAny) { b.t = t; b.u = u; b.v = v; b.inst = row; b.tri = id; return true; }
                if (b.better(t, row, id)) { b.t = t; b.u = u; b.v = v; b.inst = row; b.tri = id; }
            }
        }
    }
    return false;
}

template <bool kAny, class S>
VX_D void mesh_walk(const MeshDev &m, V3 o, V3 d, V3 inv, float tmin, int cull, Best &b, S &stack) {
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const BvhNode nd = m.tlas[stack[--sp]];
        float te;
        if (!box_hit(nd, o, inv, d, tmin, b.t, te)) continue;
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

__global__ __launch_bounds__(256) void k_mesh_probe(MeshDev m, const float *rays, int n, int cull, float *out, int *ids) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float *r = rays + (size_t)i * 8;
    const V3 o(r[0], r[1], r[2]), d(r[4], r[5], r[6]);
    const float tmin = r[3];
    const V3 inv(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    Best b{r[7], 0.0f, 0.0f, -1, -1};
    if (m.nInst > 0) {
        ScratchStack st;
        mesh_walk<false>(m, o, d, inv, tmin, cull, b, st);
    }
    out[(size_t)i * 4] = b.t;
    out[(size_t)i * 4 + 1] = b.u;
    out[(size_t)i * 4 + 2] = b.v;
    out[(size_t)i * 4 + 3] = b.inst >= 0 ? 1.0f : 0.0f;
    ids[(size_t)i * 2] = b.inst;
    ids[(size_t)i * 2 + 1] = b.tri;
}

// visibility: occluded[i] = 1 iff some instanced-mesh triangle (both faces) lies in [tmin, tmax]
__global__ __launch_bounds__(256) void k_mesh_occluded(MeshDev m, const float *rays, int n, unsigned char *occluded) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float *r = rays + (size_t)i * 8;
    const V3 o(r[0], r[1], r[2]), d(r[4], r[5], r[6]);
    const float tmin = r[3];
    const V3 inv(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    Best b{r[7], 0.0f, 0.0f, -1, -1};
    if (m.nInst > 0) {
        ScratchStack st;
        mesh_walk<true>(m, o, d, inv, tmin, 0, b, st);
    }
    occluded[i] = b.inst >= 0 ? 1 : 0;
}

}  // namespace

hipError_t launch_mesh_occluded(const MeshDev &m, const float *rays, int n, unsigned char *occluded, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_mesh_occluded, dim3((n + 255) / 256), dim3(256), 0, st, m, rays, n, occluded);
    return hipGetLastError();
}

hipError_t launch_mesh_probe(const MeshDev &m, const float *rays, int n, int cull, float *out, int *ids,
                             hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_mesh_probe, dim3((n + 255) / 256), dim3(256), 0, st, m, rays, n, cull, out, ids);
    return hipGetLastError();
}

}  // namespace vx
