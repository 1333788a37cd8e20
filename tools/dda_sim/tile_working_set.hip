// Working-set study on the CPU (not product code): the 128-byte lines the library's voxel walk
// (vx_device.hpp, run on the host: no kernel launch) reads for the rays of one 256-thread workgroup,
// to size the north_star's "LDS-staged bricks" idea against the L1 that already caches them.
// Camera rays of one k_closest workgroup (slot_pixel, trace.hip: four 8x8 pixel tiles, one per
// wave), then one diffuse bounce from each hit (cosine-distributed about the hit face, the
// secondary rays k_queue walks).  Per brick the walk visits it reads the octant table byte and,
// for an occupied brick, its u64 cube-cell mask; the hit reads its block-id byte.  Prints, per
// workgroup: walk iterations, line reads, distinct lines (mean / p90 / max), and the distinct lines
// of 8 consecutive workgroups (what one CU's 32 KB L1 holds at k_closest's occupancy).  Per wave it
// also counts what a material-keyed sort (optixReorder(materialId), RayGen.cu:63) could regroup:
// waves mixing hits and misses (sky), their minority lanes, and the distinct block ids of a wave's
// hits.
// Usage: tile_working_set ids.bin CX CY CZ cam.bin W H   (cam.bin: the oracle's camera_info, 32 f32)
#include <climits>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <unordered_set>
#include <vector>

#include "vx_device.hpp"

using namespace vx;

namespace {

struct Stats {
    std::vector<double> iters, reads, distinct, cu8;
    void print(const char *what) {
        auto pct = [](std::vector<double> v, double q) {
            std::sort(v.begin(), v.end());
            return v.empty() ? 0.0 : v[std::min(v.size() - 1, (size_t)(q * (double)v.size()))];
        };
        auto mean = [](const std::vector<double> &v) {
            double s = 0;
            for (double x : v) s += x;
            return v.empty() ? 0.0 : s / (double)v.size();
        };
        std::printf("%s: workgroups %zu | iterations mean %.0f | line reads mean %.0f | distinct lines mean %.1f "
                    "p90 %.0f max %.0f (%.1f KB mean) | reads per distinct line %.1f | 8 workgroups: distinct "
                    "lines mean %.0f max %.0f (%.1f KB mean, L1 32 KB)\n",
                    what, distinct.size(), mean(iters), mean(reads), mean(distinct), pct(distinct, 0.9),
                    pct(distinct, 1.0), mean(distinct) * 128 / 1024, mean(reads) / std::max(1.0, mean(distinct)),
                    mean(cu8), pct(cu8, 1.0), mean(cu8) * 128 / 1024);
    }
};

}  // namespace

int main(int argc, char **argv) {
    if (argc < 8) return 2;
    const int CX = atoi(argv[2]), CY = atoi(argv[3]), CZ = atoi(argv[4]), W = atoi(argv[6]), H = atoi(argv[7]);
    const int wx = CX * 32, wy = CY * 32, wz = CZ * 32, BX = wx / 4, BY = wy / 4, BZ = wz / 4;
    std::vector<uint8_t> ids((size_t)wx * wy * wz);
    FILE *f = fopen(argv[1], "rb");
    if (!f || fread(ids.data(), 1, ids.size(), f) != ids.size()) return 1;
    fclose(f);
    float cam[32];
    f = fopen(argv[5], "rb");
    if (!f || fread(cam, 4, 32, f) != 32) return 1;
    fclose(f);
    M3 uvToWorld;
    std::memcpy(&uvToWorld, cam + 6, 36);
    const V3 pos(cam[0], cam[1], cam[2]);
    const size_t nB = (size_t)BX * BY * BZ;
    auto blin = [&](int bx, int by, int bz) {  // vx_device.hpp brick_index
        const size_t m = (size_t)(bx >> 2) + (size_t)(CX * 2) * ((bz >> 2) + (size_t)(CZ * 2) * (by >> 2));
        return m * 64 + (size_t)((bx & 3) + 4 * ((bz & 3) + 4 * (by & 3)));
    };
    std::vector<uint8_t> bricks(nB * 64, 0);
    std::vector<uint64_t> cellMask(nB, 0);
    for (int y = 0; y < wy; ++y)
        for (int z = 0; z < wz; ++z)
            for (int x = 0; x < wx; ++x) {
                const size_t ch = (x >> 5) + (size_t)CX * ((z >> 5) + (size_t)CZ * (y >> 5));
                const uint8_t id = ids[ch * 32768 + (x & 31) + 32 * ((z & 31) + 32 * (y & 31))];
                if (!id) continue;
                const size_t b = blin(x >> 2, y >> 2, z >> 2);
                const int lc = (x & 3) + 4 * ((z & 3) + 4 * (y & 3));
                bricks[b * 64 + lc] = id;
                if (id >= 1 && id <= 12) cellMask[b] |= 1ull << lc;
            }
    std::vector<uint8_t> od(8 * nB, 0);  // the cube tables (vxpt_host.cpp octant_fill's recurrence)
    for (int oct = 0; oct < 8; ++oct) {
        uint8_t *S = od.data() + oct * nB;
        const int sx = (oct & 1) ? 1 : -1, sy = (oct & 2) ? 1 : -1, sz = (oct & 4) ? 1 : -1;
        auto get = [&](int x, int y, int z) -> int {
            if (x < 0 || y < 0 || z < 0 || x >= BX || y >= BY || z >= BZ) return 255;
            return S[blin(x, y, z)];
        };
        for (int iy = 0; iy < BY; ++iy)
            for (int iz = 0; iz < BZ; ++iz)
                for (int ix = 0; ix < BX; ++ix) {
                    const int x = sx > 0 ? BX - 1 - ix : ix, y = sy > 0 ? BY - 1 - iy : iy, z = sz > 0 ? BZ - 1 - iz : iz;
                    int v = 0;
                    if (!cellMask[blin(x, y, z)]) {
                        int mn = 255;
                        for (int k = 1; k < 8; ++k)
                            mn = std::min(mn, get(x + ((k & 1) ? sx : 0), y + ((k & 2) ? sy : 0), z + ((k & 4) ? sz : 0)));
                        v = std::min(255, 1 + mn);
                    }
                    S[blin(x, y, z)] = (uint8_t)v;
                }
    }
    WorldDev w{};
    w.bricks = bricks.data();
    w.cellMask = cellMask.data();
    w.bdist = od.data();
    w.nBricks = (int)nB;
    w.cx = CX; w.cy = CY; w.cz = CZ;
    w.wx = wx; w.wy = wy; w.wz = wz;
    w.mx = wx / 16; w.my = wy / 16; w.mz = wz / 16;

    // line ids: table tag in the top bits, 128-byte line below
    auto odLine = [&](const Dda &s) { return (1ull << 60) | ((size_t)(s.od - od.data()) + (size_t)s.nb) >> 7; };
    auto cmLine = [&](int nb) { return (2ull << 60) | (((size_t)nb * 8) >> 7); };
    auto idLine = [&](const Hit &h) {
        const size_t b = blin(h.x >> 2, h.y >> 2, h.z >> 2);
        return (3ull << 60) | ((b * 64 + (size_t)((h.x & 3) + 4 * ((h.z & 3) + 4 * (h.y & 3)))) >> 7);
    };
    // one ray's walk; its line reads go to `lines`, returns the hit
    auto walk = [&](V3 o, V3 d, std::vector<uint64_t> &lines, long &iters) {
        Hit h{0, 0, 0, 0, -1, 0, kRayMax};
        Dda s;
        int rc = dda_begin<false>(w, o, d, 0.0f, kRayMax, s, h);
        int lastNb = -1;
        auto visit = [&]() {
            if (s.nb == lastNb || s.nb < 0) return;
            lastNb = s.nb;
            lines.push_back(odLine(s));
            if (s.dist == 0) lines.push_back(cmLine(s.nb));
        };
        if (rc != DdaNone) visit();
        while (rc == DdaRun) {
            rc = dda_iter<false>(w, s, h);
            ++iters;
            visit();
        }
        if (rc != DdaEvent) return Hit{0, 0, 0, 0, -1, 0, kRayMax};
        lines.push_back(idLine(h));
        return h;
    };
    const V3 normals[6] = {V3(0, -1, 0), V3(0, 1, 0), V3(-1, 0, 0), V3(1, 0, 0), V3(0, 0, -1), V3(0, 0, 1)};
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    Stats cam1, sec;
    // per wave (camera, bounce): waves, mixed hit / miss waves, minority lanes of the mixed ones,
    // sum of distinct hit block ids
    long wv[2] = {0, 0}, mixed[2] = {0, 0}, minority[2] = {0, 0}, idsum[2] = {0, 0};
    int hitW[2][4][64], idW[2][4][64];
    std::vector<std::unordered_set<uint64_t>> cuCam, cuSec;
    const int tilesX = (W + 7) / 8, tilesY = (H + 7) / 8, nWg = (tilesX * tilesY * 64 + 255) / 256;
    for (int wg = 0; wg < nWg; ++wg)
        {
            std::vector<uint64_t> lc, ls;
            long ic = 0, is = 0;
            for (int p2 = 0; p2 < 2; ++p2)
                for (int q = 0; q < 4; ++q)
                    for (int l = 0; l < 64; ++l) hitW[p2][q][l] = -1, idW[p2][q][l] = 0;
            for (int k = 0; k < 256; ++k) {
                const int slot = wg * 256 + k, tile = slot >> 6, lane = slot & 63;
                const int x = (tile % tilesX) * 8 + (lane & 7), y = (tile / tilesX) * 8 + (lane >> 3);
                if (tile >= tilesX * tilesY || x >= W || y >= H) continue;
                const V2 uv(((float)x + 0.5f) / (float)W, ((float)y + 0.5f) / (float)H);
                const V3 d = normalize(m3_apply(uvToWorld, V3(uv.x, uv.y, 1.0f)));
                const Hit h = walk(pos, d, lc, ic);
                hitW[0][k >> 6][k & 63] = h.hit;
                idW[0][k >> 6][k & 63] = h.id;
                if (!h.hit) continue;
                // one diffuse bounce: cosine-distributed about the entered face's outward normal
                // (the face the ray crossed, seen from the ray: against d)
                V3 n = normals[h.face];
                if (dot(n, d) > 0.0f) n = V3(-n.x, -n.y, -n.z);
                const float r1 = U(rng), r2 = U(rng), phi = 6.2831853f * r1, sr = sqrtf(r2);
                const V3 a = fabsf(n.x) > 0.5f ? V3(0, 1, 0) : V3(1, 0, 0);
                const V3 t = normalize(cross(a, n)), b = cross(n, t);
                const V3 dd = normalize(t * (cosf(phi) * sr) + b * (sinf(phi) * sr) + n * sqrtf(1.0f - r2));
                const V3 hp = pos + d * h.t + n * 1e-3f;
                const Hit h2 = walk(hp, dd, ls, is);
                hitW[1][k >> 6][k & 63] = h2.hit;
                idW[1][k >> 6][k & 63] = h2.id;
            }
            for (int p2 = 0; p2 < 2; ++p2)
                for (int q = 0; q < 4; ++q) {
                    int nh = 0, nm = 0;
                    uint32_t seen = 0;
                    for (int l = 0; l < 64; ++l) {
                        if (hitW[p2][q][l] < 0) continue;
                        if (hitW[p2][q][l]) { ++nh; seen |= 1u << (idW[p2][q][l] & 31); } else ++nm;
                    }
                    if (nh + nm == 0) continue;
                    ++wv[p2];
                    if (nh && nm) { ++mixed[p2]; minority[p2] += std::min(nh, nm); }
                    idsum[p2] += __builtin_popcount(seen);
                }
            for (int pass = 0; pass < 2; ++pass) {
                const std::vector<uint64_t> &L = pass ? ls : lc;
                Stats &S = pass ? sec : cam1;
                std::unordered_set<uint64_t> u(L.begin(), L.end());
                S.iters.push_back((double)(pass ? is : ic));
                S.reads.push_back((double)L.size());
                S.distinct.push_back((double)u.size());
                auto &cu = pass ? cuSec : cuCam;
                cu.push_back(std::move(u));
                if (cu.size() == 8) {
                    std::unordered_set<uint64_t> all;
                    for (auto &s : cu) all.insert(s.begin(), s.end());
                    S.cu8.push_back((double)all.size());
                    cu.clear();
                }
            }
        }
    cam1.print("camera rays");
    sec.print("diffuse bounce rays");
    const char *names[2] = {"camera rays", "diffuse bounce rays"};
    for (int p2 = 0; p2 < 2; ++p2)
        std::printf("%s: waves %ld | mixing hits and misses %.1f %% (minority lanes %.1f %% of those waves' lanes) | "
                    "distinct block ids per wave %.2f\n", names[p2], wv[p2], 100.0 * mixed[p2] / std::max(1L, wv[p2]),
                    100.0 * minority[p2] / std::max(1.0, 64.0 * mixed[p2]), (double)idsum[p2] / std::max(1L, wv[p2]));
    return 0;
}
