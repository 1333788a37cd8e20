// vxpt -- the instanced meshes' BVH builder (host only, no HIP kernels).  Shared by vxpt_host.cpp and
// the CPU test driver (tests/native/mesh_walk_driver.hip).
#pragma once
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <vector>

#include "vx_internal.hpp"

namespace vx {

// Binned-SAH BVH over boxes (lo xyz, hi xyz per primitive): nodes[0] = root, children of an
// inner node adjacent, leaves of at most leafMax primitives (order = primitive order in the
// leaves).  Node boxes are widened by 1e-4 (1 + |coordinate|), far above the slab test's
// rounding, so box culling is conservative.  Fails past a depth of 40 (the walk's one stack holds
// 84 entries, TLAS and BLAS together) -- only for more than leafMax * 2^40 primitives, see the
// split rule below; *maxDepth = the deepest leaf.
constexpr int kBvhMaxDepth = 40;
inline bool build_bvh(const std::vector<float> &box, int leafMax, std::vector<BvhNode> &nodes, std::vector<int> &order,
               int *maxDepth) {
    const int n = (int)(box.size() / 6);
    order.resize(n);
    for (int i = 0; i < n; ++i) order[i] = i;
    nodes.assign(1, BvhNode{});
    *maxDepth = 0;
    if (n == 0) return true;
    struct Job { int node, b, e, depth; };
    std::vector<Job> jobs{{0, 0, n, 0}};
    while (!jobs.empty()) {
        const Job j = jobs.back();
        jobs.pop_back();
        if (j.depth > kBvhMaxDepth) return false;
        *maxDepth = std::max(*maxDepth, j.depth);
        float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        float clo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, chi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (int i = j.b; i < j.e; ++i) {
            const float *bx = &box[(size_t)order[i] * 6];
            for (int k = 0; k < 3; ++k) {
                lo[k] = std::min(lo[k], bx[k]);
                hi[k] = std::max(hi[k], bx[k + 3]);
                const float cc = 0.5f * (bx[k] + bx[k + 3]);
                clo[k] = std::min(clo[k], cc);
                chi[k] = std::max(chi[k], cc);
            }
        }
        BvhNode &nd = nodes[j.node];
        for (int k = 0; k < 3; ++k) {
            nd.lo[k] = lo[k] - 1e-4f * (1.0f + std::fabs(lo[k]));
            nd.hi[k] = hi[k] + 1e-4f * (1.0f + std::fabs(hi[k]));
        }
        if (j.e - j.b <= leafMax) {
            nd.left = j.b;
            nd.count = j.e - j.b;
            continue;
        }
        // binned SAH split (16 centroid bins per axis, cost = area x count on either side) while the
        // depth budget allows it: an SAH split may leave all but one primitive on one side, so it
        // is taken only if a child of n - 1 primitives still reaches its leaves within the limit
        // by median splits (levels(c) = ceil(log2(ceil(c / leafMax)))); otherwise -- and when no
        // bin boundary separates the primitives -- the median of the widest axis.  Any input of
        // at most leafMax * 2^40 primitives then stays within the depth limit.
        int axis = 0;
        for (int k = 1; k < 3; ++k)
            if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
        int mid = -1;
        const auto levels = [&](long long c) {
            int l = 0;
            for (long long cap = leafMax; cap < c; cap *= 2) ++l;
            return l;
        };
        if (j.depth + 1 + levels((long long)(j.e - j.b) - 1) <= kBvhMaxDepth) {
            constexpr int kBins = 16;
            // centroid bin, clamped (also for non-finite coordinates)
            const auto bin_of = [&](float cc, float c0, float ext) {
                const float f = (cc - c0) / ext * (float)kBins;
                return f >= 0.0f ? (f < (float)(kBins - 1) ? (int)f : kBins - 1) : 0;
            };
            float bestCost = FLT_MAX;
            int bestAxis = -1, bestBin = 0;
            for (int k = 0; k < 3; ++k) {
                const float ext = chi[k] - clo[k];
                if (!(ext > 0.0f) || !std::isfinite(ext)) continue;
                float blo[kBins][3], bhi[kBins][3];
                int cnt[kBins] = {};
                for (int q = 0; q < kBins; ++q)
                    for (int a = 0; a < 3; ++a) { blo[q][a] = FLT_MAX; bhi[q][a] = -FLT_MAX; }
                for (int i = j.b; i < j.e; ++i) {
                    const float *bx = &box[(size_t)order[i] * 6];
                    const int q = bin_of(0.5f * (bx[k] + bx[k + 3]), clo[k], ext);
                    cnt[q]++;
                    for (int a = 0; a < 3; ++a) {
                        blo[q][a] = std::min(blo[q][a], bx[a]);
                        bhi[q][a] = std::max(bhi[q][a], bx[a + 3]);
                    }
                }
                auto area = [](const float *lo3, const float *hi3) {
                    const float dx = hi3[0] - lo3[0], dy = hi3[1] - lo3[1], dz = hi3[2] - lo3[2];
                    return dx * dy + dy * dz + dz * dx;
                };
                float rArea[kBins];
                int rCnt[kBins];
                float rl[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, rh[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
                for (int q = kBins - 1, c = 0; q > 0; --q) {
                    c += cnt[q];
                    for (int a = 0; a < 3; ++a) { rl[a] = std::min(rl[a], blo[q][a]); rh[a] = std::max(rh[a], bhi[q][a]); }
                    rCnt[q] = c;
                    rArea[q] = c ? area(rl, rh) : 0.0f;
                }
                float ll[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, lh[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
                for (int q = 0, c = 0; q < kBins - 1; ++q) {  // split between bins q and q + 1
                    c += cnt[q];
                    for (int a = 0; a < 3; ++a) { ll[a] = std::min(ll[a], blo[q][a]); lh[a] = std::max(lh[a], bhi[q][a]); }
                    if (c == 0 || rCnt[q + 1] == 0) continue;
                    const float cost = area(ll, lh) * c + rArea[q + 1] * rCnt[q + 1];
                    if (cost < bestCost) { bestCost = cost; bestAxis = k; bestBin = q; }
                }
            }
            if (bestAxis >= 0) {
                const float ext = chi[bestAxis] - clo[bestAxis], c0 = clo[bestAxis];
                auto it = std::stable_partition(order.begin() + j.b, order.begin() + j.e, [&](int x) {
                    const float *bx = &box[(size_t)x * 6];
                    return bin_of(0.5f * (bx[bestAxis] + bx[bestAxis + 3]), c0, ext) <= bestBin;
                });
                mid = (int)(it - order.begin());
            }
        }
        if (mid <= j.b || mid >= j.e) {
            mid = (j.b + j.e) / 2;
            std::nth_element(order.begin() + j.b, order.begin() + mid, order.begin() + j.e, [&](int x, int y) {
                const float cx = box[(size_t)x * 6 + axis] + box[(size_t)x * 6 + axis + 3];
                const float cy = box[(size_t)y * 6 + axis] + box[(size_t)y * 6 + axis + 3];
                return cx < cy || (cx == cy && x < y);
            });
        }
        const int left = (int)nodes.size();
        nodes[j.node].left = left;
        nodes[j.node].count = 0;
        nodes.push_back(BvhNode{});
        nodes.push_back(BvhNode{});
        jobs.push_back({left, j.b, mid, j.depth + 1});
        jobs.push_back({left + 1, mid, j.e, j.depth + 1});
    }
    return true;
}


}  // namespace vx
