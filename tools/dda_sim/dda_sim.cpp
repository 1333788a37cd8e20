// Traversal-structure study on the CPU (not product code): outer iterations per ray of the
// brick-level walk over a voxel world with (S1) the library's per-octant empty CUBE tables and
// (S2) per-octant anisotropic empty BOXES (greedy extents from the cube), for camera rays and
// secondary rays from their hits.  One outer iteration = one occupied-brick walk or one skip, as
// in dda_iter (vx_device.hpp).  Input: chunk-major u8 ids (the library's upload layout).
// Usage: dda_sim ids.bin CX CY CZ [subsample]
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

struct World {
    int W, H, D, BX, BY, BZ;
    std::vector<uint8_t> solid;     // per cell (x + W*(z + D*y))
    std::vector<uint8_t> bocc;      // per brick occupied
    std::vector<int> pre;           // 3D prefix sums of occupied bricks, (BX+1)(BY+1)(BZ+1)
    int cell(int x, int y, int z) const { return solid[(size_t)x + (size_t)W * (z + (size_t)D * y)]; }
    int bi(int bx, int by, int bz) const { return bx + BX * (bz + BZ * by); }
    int P(int x, int y, int z) const { return pre[(size_t)x + (BX + 1) * ((size_t)z + (BZ + 1) * y)]; }
    // occupied bricks in [x0,x1) x [y0,y1) x [z0,z1)
    int occ(int x0, int y0, int z0, int x1, int y1, int z1) const {
        return P(x1, y1, z1) - P(x0, y1, z1) - P(x1, y0, z1) - P(x1, y1, z0) + P(x0, y0, z1) + P(x0, y1, z0) +
               P(x1, y0, z0) - P(x0, y0, z0);
    }
};

struct Box { uint8_t e[3]; };  // extents in bricks along the octant's x, y, z directions

// empty box of extents e cornered at brick b, extending into octant sgn (clamped to the world)
static bool box_empty(const World &w, int bx, int by, int bz, const int sg[3], int ex, int ey, int ez) {
    int lo[3], hi[3];
    const int b[3] = {bx, by, bz}, e[3] = {ex, ey, ez}, n[3] = {w.BX, w.BY, w.BZ};
    for (int a = 0; a < 3; ++a) {
        if (sg[a] > 0) { lo[a] = b[a]; hi[a] = std::min(n[a], b[a] + e[a]); }
        else { lo[a] = std::max(0, b[a] - e[a] + 1); hi[a] = b[a] + 1; }
    }
    return w.occ(lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]) == 0;
}

int main(int argc, char **argv) {
    if (argc < 5) { std::fprintf(stderr, "usage: dda_sim ids.bin CX CY CZ [subsample] [cap] [orders]\n"); return 2; }
    const int cap = argc > 6 ? std::atoi(argv[6]) : 64, nOrders = argc > 7 ? std::atoi(argv[7]) : 2;
    const int CX = std::atoi(argv[2]), CY = std::atoi(argv[3]), CZ = std::atoi(argv[4]);
    const int sub = argc > 5 ? std::atoi(argv[5]) : 4;
    World w;
    w.W = CX * 32; w.H = CY * 32; w.D = CZ * 32;
    w.BX = w.W / 4; w.BY = w.H / 4; w.BZ = w.D / 4;
    std::vector<uint8_t> ids((size_t)CX * CY * CZ * 32768);
    FILE *f = std::fopen(argv[1], "rb");
    if (!f || std::fread(ids.data(), 1, ids.size(), f) != ids.size()) { std::fprintf(stderr, "bad ids\n"); return 1; }
    std::fclose(f);
    w.solid.assign((size_t)w.W * w.H * w.D, 0);
    for (int y = 0; y < w.H; ++y)
        for (int z = 0; z < w.D; ++z)
            for (int x = 0; x < w.W; ++x) {
                const size_t ch = (x >> 5) + (size_t)CX * ((z >> 5) + (size_t)CZ * (y >> 5));
                const int id = ids[ch * 32768 + (x & 31) + 32 * ((z & 31) + 32 * (y & 31))];
                w.solid[(size_t)x + (size_t)w.W * (z + (size_t)w.D * y)] = (id >= 1 && id <= 12) ? 1 : 0;
            }
    w.bocc.assign((size_t)w.BX * w.BY * w.BZ, 0);
    for (int y = 0; y < w.H; ++y)
        for (int z = 0; z < w.D; ++z)
            for (int x = 0; x < w.W; ++x)
                if (w.cell(x, y, z)) w.bocc[w.bi(x >> 2, y >> 2, z >> 2)] = 1;
    w.pre.assign((size_t)(w.BX + 1) * (w.BY + 1) * (w.BZ + 1), 0);
    for (int y = 1; y <= w.BY; ++y)
        for (int z = 1; z <= w.BZ; ++z)
            for (int x = 1; x <= w.BX; ++x)
                w.pre[(size_t)x + (w.BX + 1) * ((size_t)z + (w.BZ + 1) * y)] =
                    w.bocc[w.bi(x - 1, y - 1, z - 1)] + w.P(x - 1, y, z) + w.P(x, y - 1, z) + w.P(x, y, z - 1) -
                    w.P(x - 1, y - 1, z) - w.P(x - 1, y, z - 1) - w.P(x, y - 1, z - 1) + w.P(x - 1, y - 1, z - 1);
    // per octant: the cube (S1) and the greedy anisotropic box (S2) of every empty brick
    const size_t nb = (size_t)w.BX * w.BY * w.BZ;
    std::vector<Box> cube(8 * nb), aniso(8 * nb);
    for (int oct = 0; oct < 8; ++oct) {
        const int sg[3] = {(oct & 1) ? 1 : -1, (oct & 2) ? 1 : -1, (oct & 4) ? 1 : -1};
        for (int by = 0; by < w.BY; ++by)
            for (int bz = 0; bz < w.BZ; ++bz)
                for (int bx = 0; bx < w.BX; ++bx) {
                    const size_t k = oct * nb + w.bi(bx, by, bz);
                    if (w.bocc[w.bi(bx, by, bz)]) { cube[k] = {{0, 0, 0}}; aniso[k] = {{0, 0, 0}}; continue; }
                    int S = 1;
                    while (S < 64 && box_empty(w, bx, by, bz, sg, S + 1, S + 1, S + 1)) ++S;
                    cube[k] = {{(uint8_t)S, (uint8_t)S, (uint8_t)S}};
                    // greedy: grow x, z, then y one brick at a time while empty (cap 64), best of two orders
                    Box best{{(uint8_t)S, (uint8_t)S, (uint8_t)S}};
                    long bestV = (long)S * S * S;
                    const int orders[2][3] = {{0, 2, 1}, {1, 0, 2}};
                    for (int oi = 0; oi < nOrders; ++oi) {
                        const auto &ord = orders[oi];
                        int e[3] = {S, S, S};
                        for (int a : ord)
                            while (e[a] < cap) {
                                int t[3] = {e[0], e[1], e[2]};
                                ++t[a];
                                if (!box_empty(w, bx, by, bz, sg, t[0], t[1], t[2])) break;
                                e[a] = t[a];
                            }
                        const long v = (long)e[0] * e[1] * e[2];
                        if (v > bestV) { bestV = v; best = {{(uint8_t)e[0], (uint8_t)e[1], (uint8_t)e[2]}}; }
                    }
                    aniso[k] = best;
                }
    }
    // camera of bench.py (C1 x4) at 1920x1080 / sub; secondary rays from the hits: the sun direction
    // and cosine-distributed directions about the face normal
    const double pos[3] = {35.6184 * 4, 11.8733 * 4, 42.0387 * 4};
    double dir[3] = {-0.321564, -0.0129988, -0.946799};
    const double dl = std::sqrt(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    for (double &v : dir) v /= dl;
    double right[3] = {-dir[2], 0.0, dir[0]};  // dir x up
    const double rl = std::sqrt(right[0] * right[0] + right[2] * right[2]);
    right[0] /= rl; right[2] /= rl;
    const double up[3] = {right[1] * dir[2] - right[2] * dir[1], right[2] * dir[0] - right[0] * dir[2],
                          right[0] * dir[1] - right[1] * dir[0]};
    const int RW = 1920 / sub, RH = 1080 / sub;
    const double tanX = 1.0, tanY = tanX * RH / RW;
    double sun[3] = {0.35, 0.7, 0.45};
    const double sl = std::sqrt(sun[0] * sun[0] + sun[1] * sun[1] + sun[2] * sun[2]);
    for (double &v : sun) v /= sl;
    std::mt19937 rng(5);
    std::uniform_real_distribution<double> U(0.0, 1.0);

    // one walk: returns outer iterations; *hit / face / hit point for radiance rays
    auto walk = [&](const std::vector<Box> &tab, const double o[3], const double d[3], bool occl, int &iters,
                    double hp[3], int &face) -> bool {
        int c[3] = {(int)std::floor(o[0]), (int)std::floor(o[1]), (int)std::floor(o[2])};
        const int n[3] = {w.W, w.H, w.D};
        for (int a = 0; a < 3; ++a)
            if (c[a] < 0 || c[a] >= n[a]) return false;
        int s[3];
        double inv[3], tn[3];
        for (int a = 0; a < 3; ++a) {
            s[a] = d[a] > 0 ? 1 : -1;
            inv[a] = d[a] != 0 ? 1.0 / d[a] : 1e300;
            tn[a] = d[a] != 0 ? ((s[a] > 0 ? c[a] + 1 : c[a]) - o[a]) * inv[a] : 1e300;
        }
        const int oct = (s[0] > 0 ? 1 : 0) | (s[1] > 0 ? 2 : 0) | (s[2] > 0 ? 4 : 0);
        iters = 0;
        for (int guard = 0; guard < 4000; ++guard) {
            ++iters;
            const int b[3] = {c[0] >> 2, c[1] >> 2, c[2] >> 2};
            const size_t bk = w.bi(b[0], b[1], b[2]);
            if (!w.bocc[bk]) {
                const Box &bx = tab[oct * nb + bk];
                // box in cells; jump to its exit crossing
                double Te = 1e300;
                int ea = 0;
                int lo[3], hi[3];
                for (int a = 0; a < 3; ++a) {
                    const int e = 4 * (bx.e[a] - 1);
                    if (s[a] > 0) { lo[a] = b[a] * 4; hi[a] = std::min(b[a] * 4 + 3 + e, n[a] - 1); }
                    else { lo[a] = std::max(b[a] * 4 - e, 0); hi[a] = b[a] * 4 + 3; }
                    if (d[a] == 0) continue;
                    const double t = ((s[a] > 0 ? hi[a] + 1 : lo[a]) - o[a]) * inv[a];
                    if (t < Te) { Te = t; ea = a; }
                }
                for (int a = 0; a < 3; ++a) {
                    if (a == ea) c[a] = s[a] > 0 ? hi[a] : lo[a];
                    else if (d[a] != 0) c[a] = std::clamp((int)std::floor(o[a] + Te * d[a]), lo[a], hi[a]);
                    tn[a] = d[a] != 0 ? ((s[a] > 0 ? c[a] + 1 : c[a]) - o[a]) * inv[a] : 1e300;
                }
                tn[ea] = Te;
            } else {
                // cell walk inside the brick
                bool inBrick = true;
                while (inBrick) {
                    if (w.cell(c[0], c[1], c[2]) && !(occl && false)) {
                        face = 0;
                        hp[0] = c[0]; hp[1] = c[1]; hp[2] = c[2];
                        return true;
                    }
                    int a = tn[0] < tn[1] ? (tn[0] < tn[2] ? 0 : 2) : (tn[1] < tn[2] ? 1 : 2);
                    const int nc = c[a] + s[a];
                    if ((nc >> 2) != (c[a] >> 2)) break;  // leaves the brick: next outer iteration
                    c[a] = nc;
                    tn[a] += std::fabs(inv[a]);
                }
            }
            // step across the next plane
            int a = tn[0] < tn[1] ? (tn[0] < tn[2] ? 0 : 2) : (tn[1] < tn[2] ? 1 : 2);
            const double tHit = tn[a];
            c[a] += s[a];
            tn[a] += std::fabs(inv[a]);
            if (c[a] < 0 || c[a] >= n[a]) return false;
            if (w.cell(c[0], c[1], c[2])) {
                face = a * 2 + (s[a] > 0 ? 0 : 1);
                for (int k = 0; k < 3; ++k) hp[k] = o[k] + tHit * d[k];
                return true;
            }
        }
        iters = -1;  // stuck (the study's float walk, not the library's exact one): excluded
        return false;
    };

    struct Stat { std::vector<int> v; };
    Stat st[2][3];  // structure x {camera, sun, hemisphere}
    for (int py = 0; py < RH; ++py)
        for (int px = 0; px < RW; ++px) {
            const double u = ((px + 0.5) / RW * 2 - 1) * tanX, v = (1 - (py + 0.5) / RH * 2) * tanY;
            double d[3];
            for (int k = 0; k < 3; ++k) d[k] = dir[k] + u * right[k] + v * up[k];
            const double l = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
            for (double &x : d) x /= l;
            double hp[3];
            int face = 0;
            for (int S = 0; S < 2; ++S) {
                int it;
                const bool hit = walk(S ? aniso : cube, pos, d, false, it, hp, face);
                if (it >= 0) st[S][0].v.push_back(it);
                if (!hit) continue;
                // secondary rays from just outside the hit face
                double o2[3] = {hp[0], hp[1], hp[2]};
                const int a = face / 2;
                const double nrm = (face & 1) ? 1.0 : -1.0;  // back toward the ray origin side
                double nvec[3] = {0, 0, 0};
                nvec[a] = nrm;
                for (int k = 0; k < 3; ++k) o2[k] += nvec[k] * 1e-3;
                if (S == 0 && a == 0 && false) {}
                int it2;
                double hp2[3];
                int f2;
                walk(S ? aniso : cube, o2, sun, true, it2, hp2, f2);
                if (it2 >= 0) st[S][1].v.push_back(it2);
                // cosine hemisphere about the face normal
                std::mt19937 r2(px * 7919 + py);
                const double r1 = U(r2), rr = U(r2), phi = 2 * M_PI * r1, sr = std::sqrt(rr);
                double t1[3] = {0, 0, 0}, t2[3] = {0, 0, 0};
                t1[(a + 1) % 3] = 1; t2[(a + 2) % 3] = 1;
                double hd[3];
                for (int k = 0; k < 3; ++k)
                    hd[k] = std::cos(phi) * sr * t1[k] + std::sin(phi) * sr * t2[k] + std::sqrt(1 - rr) * nvec[k];
                walk(S ? aniso : cube, o2, hd, false, it2, hp2, f2);
                if (it2 >= 0) st[S][2].v.push_back(it2);
            }
        }
    const char *names[3] = {"camera", "sun", "hemisphere"};
    for (int k = 0; k < 3; ++k)
        for (int S = 0; S < 2; ++S) {
            auto v = st[S][k].v;
            std::sort(v.begin(), v.end());
            double mean = 0;
            for (int x : v) mean += x;
            mean /= std::max<size_t>(1, v.size());
            std::printf("%-10s %-6s n=%zu mean=%.2f p50=%d p90=%d p99=%d max=%d\n", names[k], S ? "aniso" : "cube",
                        v.size(), mean, v[v.size() / 2], v[v.size() * 9 / 10], v[v.size() * 99 / 100], v.back());
        }
    return 0;
}
