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
#include "vx_mesh.hpp"

namespace vx {
namespace {

__global__ __launch_bounds__(256) void k_mesh_probe(MeshDev m, const float *rays, int n, int cull, float *out, int *ids) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float *r = rays + (size_t)i * 8;
    const V3 o(r[0], r[1], r[2]), d(r[4], r[5], r[6]);
    const float tmin = r[3];
    const V3 inv(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    Best b{r[7], 0.0f, 0.0f, -1, -1, -1};
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
    Best b{r[7], 0.0f, 0.0f, -1, -1, -1};
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
