// CPU test driver (host code only, no kernel launch): the library's instanced-mesh BVH (bvh_build.hpp,
// laid out as vxpt_host.cpp build_blas / build_tlas do) walked by the library's own walk (vx_mesh.hpp,
// host + device) for the probe kernels' queries (meshes.hip k_mesh_probe / k_mesh_occluded).
// Usage: mesh_walk_driver meshes.bin rays.bin out.bin
//   meshes.bin: 32 x (int32 n, n x 9 f32 triangles) per block id, int32 rows, rows x 5 int32
//               (object = block - 1, instance id, x, y, z)
//   rays.bin:   8 f32 per ray (origin, tmin, direction, tmax)
//   out.bin:    13 int32 per ray: closest without culling (t, u, v bits, hit, row, triangle), the same
//               with back faces culled, occluded
#include <cstdio>
#include <vector>

#include "bvh_build.hpp"
#include "vx_mesh.hpp"

using namespace vx;

int main(int argc, char **argv) {
    if (argc < 4) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    auto rd = [&](void *p, size_t n) { return fread(p, 1, n, f) == n; };
    std::vector<std::vector<float>> tris(32);
    for (int b = 0; b < 32; ++b) {
        int32_t n = 0;
        if (!rd(&n, 4)) return 1;
        tris[b].resize((size_t)n * 9);
        if (n && !rd(tris[b].data(), (size_t)n * 36)) return 1;
    }
    int32_t nRows = 0;
    if (!rd(&nRows, 4)) return 1;
    std::vector<int32_t> rows((size_t)nRows * 5);
    if (nRows && !rd(rows.data(), rows.size() * 4)) return 1;
    fclose(f);
    // BLAS per block type (build_blas), concatenated
    std::vector<BvhNode> blas;
    std::vector<float> blasTri;
    std::vector<int> blasTriId;
    std::vector<int2> root(32, make_int2(-1, -1));
    int maxBlasDepth = 0;
    for (int b = 0; b < 32; ++b) {
        const int nt = (int)(tris[b].size() / 9);
        if (nt == 0) continue;
        std::vector<float> box((size_t)nt * 6);
        for (int t = 0; t < nt; ++t)
            for (int k = 0; k < 3; ++k) {
                const float *v = &tris[b][(size_t)t * 9];
                box[(size_t)t * 6 + k] = std::min(v[k], std::min(v[3 + k], v[6 + k]));
                box[(size_t)t * 6 + 3 + k] = std::max(v[k], std::max(v[3 + k], v[6 + k]));
            }
        std::vector<BvhNode> nodes;
        std::vector<int> order;
        int depth = 0;
        if (!build_bvh(box, 4, nodes, order, &depth)) return 3;
        maxBlasDepth = std::max(maxBlasDepth, depth);
        root[b] = make_int2((int)blas.size(), (int)blasTriId.size());
        blas.insert(blas.end(), nodes.begin(), nodes.end());
        for (int t : order) {
            blasTri.insert(blasTri.end(), tris[b].begin() + (size_t)t * 9, tris[b].begin() + (size_t)t * 9 + 9);
            blasTriId.push_back(t);
        }
    }
    // TLAS over the instances whose block has a mesh (build_tlas)
    std::vector<MeshInst> mi;
    std::vector<float> ibox;
    for (int k = 0; k < nRows; ++k) {
        const int block = rows[k * 5] + 1;
        const int2 r = root[block];
        if (r.x < 0) continue;
        const BvhNode &rt = blas[r.x];
        const float cell[3] = {(float)rows[k * 5 + 2], (float)rows[k * 5 + 3], (float)rows[k * 5 + 4]};
        mi.push_back(MeshInst{{cell[0], cell[1], cell[2]}, block, k});
        for (int a = 0; a < 3; ++a) ibox.push_back(rt.lo[a] + cell[a]);
        for (int a = 0; a < 3; ++a) ibox.push_back(rt.hi[a] + cell[a]);
    }
    std::vector<BvhNode> tlas;
    std::vector<int> order;
    int tlasDepth = 0;
    if (!build_bvh(ibox, 2, tlas, order, &tlasDepth)) return 3;
    std::vector<MeshInst> sorted;
    for (int i : order) sorted.push_back(mi[i]);
    MeshDev m{tlas.data(), sorted.data(), blas.data(), blasTri.data(), blasTriId.data(), root.data(), (int)sorted.size()};
    fprintf(stderr, "instances %d  tlas depth %d  deepest blas %d\n", (int)sorted.size(), tlasDepth, maxBlasDepth);
    // the probe kernels' per-ray work
    FILE *fr = fopen(argv[2], "rb");
    if (!fr) return 1;
    std::vector<float> rays;
    float buf[8];
    while (fread(buf, 4, 8, fr) == 8) rays.insert(rays.end(), buf, buf + 8);
    fclose(fr);
    const size_t n = rays.size() / 8;
    std::vector<int32_t> out(n * 13, 0);
    for (size_t i = 0; i < n; ++i) {
        const float *r = &rays[i * 8];
        const V3 o(r[0], r[1], r[2]), d(r[4], r[5], r[6]);
        const float tmin = r[3];
        const V3 inv(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        for (int cull = 0; cull < 2; ++cull) {
            Best b{r[7], 0.0f, 0.0f, -1, -1, -1};
            ScratchStack st;
            mesh_walk<false>(m, o, d, inv, tmin, cull, b, st);
            int32_t *q = &out[i * 13 + 6 * cull];
            q[0] = __builtin_bit_cast(int32_t, b.t); q[1] = __builtin_bit_cast(int32_t, b.u); q[2] = __builtin_bit_cast(int32_t, b.v);
            q[3] = b.inst >= 0 ? 1 : 0; q[4] = b.inst; q[5] = b.tri;
        }
        Best b{r[7], 0.0f, 0.0f, -1, -1, -1};
        ScratchStack st;
        mesh_walk<true>(m, o, d, inv, tmin, 0, b, st);
        out[i * 13 + 12] = b.inst >= 0 ? 1 : 0;
    }
    FILE *fo = fopen(argv[3], "wb");
    if (!fo || fwrite(out.data(), 4, out.size(), fo) != out.size()) return 1;
    fclose(fo);
    return 0;
}
