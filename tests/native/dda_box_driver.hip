// CPU test driver (host code only, no kernel launch): the library's voxel walk (vx_device.hpp, host +
// device) over a world read from a chunk-major id file, once with the default empty-cube skip
// tables and once with the empty-box tables of box_tables.hpp.  Prints the number of rays whose
// results differ (hit, cell, face, id, t bits; occlusion) and the mean outer iterations of both.
// Usage: dda_box_driver ids.bin CX CY CZ nrays seed
//        dda_box_driver ids.bin CX CY CZ --rays rays.bin out.bin   (rays: 8 f32 each, o d tmin tmax;
//        out per ray: 16 i32 = cube closest (hit x y z face id, t bits), box closest (same, through
//        save / resume), cube occluded, box occluded -- the probe kernels' modes 0 and 2)
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <random>
#include <vector>

#include "box_tables.hpp"
#include "vx_device.hpp"

using namespace vx;

// A walk through the straggler hand-over and then cut into up to G pieces (vx_device.hpp seg_plan /
// seg_bound / dda_seg_start, k_resume's resume_split), the pieces walked one after another: the
// result of the first piece with an event.  Must equal the whole walk's.
template <bool OCC>
static int split_walk(const WorldDev &w, V3 o, V3 d, float tmin, float tmax, int cap, int G, Hit &out) {
    Hit h{0, 0, 0, 0, -1, 0, kRayMax};
    Dda s;
    int rc = dda_begin<OCC, true>(w, o, d, tmin, tmax, s, h);
    for (int k = 0; rc == DdaRun && k < cap; ++k) rc = dda_iter<OCC, true, GlobalBricks, true>(w, s, h);
    if (rc != DdaRun) { out = h; return rc; }
    const DdaSaved sv = dda_save(s, 0);
    Dda s0;
    dda_resume<true>(w, o, d, tmin, tmax, sv, s0);
    int D, n;
    float te;
    const int pieces = seg_plan(w, s0, G, D, n, te);
    for (int k = 0; k < pieces; ++k) {
        Dda sk;
        dda_resume<true>(w, o, d, tmin, tmax, sv, sk);
        int P0 = 0, P1 = 0;
        const float T0 = k > 0 ? seg_bound(sk, D, k, pieces, n, P0) : 0.0f;
        const float T1 = k + 1 < pieces ? seg_bound(sk, D, k + 1, pieces, n, P1) : tmax;
        if (k > 0 && !(T0 < te)) break;  // past the walk's end: the pieces before covered it
        if (k > 0) dda_seg_start<true>(w, sk, D, P0, T0);
        sk.tmax = fminf(T1, tmax);
        Hit hk{0, 0, 0, 0, -1, 0, kRayMax};
        int r = DdaRun;
        while (r == DdaRun) r = dda_iter<OCC, true, GlobalBricks, true>(w, sk, hk);
        if (r == DdaEvent) { out = hk; return DdaEvent; }
    }
    out = Hit{0, 0, 0, 0, -1, 0, kRayMax};
    return DdaNone;
}

int main(int argc, char **argv) {
    if (argc < 7) return 2;
    const int CX = atoi(argv[2]), CY = atoi(argv[3]), CZ = atoi(argv[4]), nrays = atoi(argv[5]);
    const unsigned seed = (unsigned)atoi(argv[6]);
    const int wx = CX * 32, wy = CY * 32, wz = CZ * 32, BX = wx / 4, BY = wy / 4, BZ = wz / 4;
    std::vector<uint8_t> ids((size_t)wx * wy * wz);
    FILE *f = fopen(argv[1], "rb");
    if (!f || fread(ids.data(), 1, ids.size(), f) != ids.size()) return 1;
    fclose(f);
    const size_t nB = (size_t)BX * BY * BZ;
    auto blin = [&](int bx, int by, int bz) {  // vxpt_host.cpp brick_lin / vx_device.hpp brick_index
        const size_t m = (size_t)(bx >> 2) + (size_t)(CX * 2) * ((bz >> 2) + (size_t)(CZ * 2) * (by >> 2));
        return m * 64 + (size_t)((bx & 3) + 4 * ((bz & 3) + 4 * (by & 3)));
    };
    std::vector<uint8_t> bricks(nB * 64, 0);
    std::vector<uint64_t> cellMask(nB, 0);
    // the box walks' sky exit (WorldDev::skyTop): 1 + the highest cube row per brick column, then its
    // suffix maxima per x / z direction quadrant (the library's upload_sky_top, restated)
    const int nbx = wx / 4, nbz = wz / 4;
    std::vector<uint16_t> colTop((size_t)nbx * nbz, 0), skyTop((size_t)4 * nbx * nbz, 0);
    for (int y = 0; y < wy; ++y)
        for (int z = 0; z < wz; ++z)
            for (int x = 0; x < wx; ++x) {
                const size_t ch = (x >> 5) + (size_t)CX * ((z >> 5) + (size_t)CZ * (y >> 5));
                const uint8_t id = ids[ch * 32768 + (x & 31) + 32 * ((z & 31) + 32 * (y & 31))];
                if (!id) continue;
                const size_t b = blin(x >> 2, y >> 2, z >> 2);
                const int lc = (x & 3) + 4 * ((z & 3) + 4 * (y & 3));
                bricks[b * 64 + lc] = id;
                if (id >= 1 && id <= 12) {
                    cellMask[b] |= 1ull << lc;
                    uint16_t &ct = colTop[(size_t)(z >> 2) * nbx + (x >> 2)];
                    if (ct < y + 1) ct = (uint16_t)(y + 1);
                }
            }
    // the default cube tables (vxpt_host.cpp octant_fill's recurrence, whole grid)
    std::vector<uint8_t> od(8 * nB, 0);
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
    // the box tables (the library's builder)
    BrickPrefix pre;
    pre.build(BX, BY, BZ, [&](int x, int y, int z) { return cellMask[blin(x, y, z)] != 0; });
    std::vector<uint32_t> box(8 * nB, 0);
    long growX = 0, empties = 0;
    for (int oct = 0; oct < 8; ++oct)
        for (int y = 0; y < BY; ++y)
            for (int z = 0; z < BZ; ++z)
                for (int x = 0; x < BX; ++x) {
                    const size_t b = blin(x, y, z);
                    box[oct * nB + b] = grow_box(pre, x, y, z, oct, od[oct * nB + b]);
                    if (od[oct * nB + b]) {
                        ++empties;
                        growX += (box[oct * nB + b] & 0xFF) + ((box[oct * nB + b] >> 8) & 0xFF) + (box[oct * nB + b] >> 16) -
                                 3 * od[oct * nB + b];
                    }
                }
    WorldDev w{};
    w.bricks = bricks.data();
    w.cellMask = cellMask.data();
    w.bdist = od.data();
    w.bbox = box.data();
    w.nBricks = (int)nB;
    w.cx = CX; w.cy = CY; w.cz = CZ;
    w.wx = wx; w.wy = wy; w.wz = wz;
    w.mx = wx / 16; w.my = wy / 16; w.mz = wz / 16;
    // the box-table walks also yield every 3 cell crossings inside a brick (WorldDev::brickSteps; the
    // cube-table walks take whole bricks): the same hits prove the yield and its save / resume exact
    for (int q = 0; q < 4; ++q)
        for (int kz = 0; kz < nbz; ++kz)
            for (int kx = 0; kx < nbx; ++kx) {
                const int bz = (q & 2) ? nbz - 1 - kz : kz, bx = (q & 1) ? nbx - 1 - kx : kx;
                const int fz = (q & 2) ? bz + 1 : bz - 1, fx = (q & 1) ? bx + 1 : bx - 1;
                uint16_t *t = skyTop.data() + (size_t)q * nbx * nbz;
                uint16_t m = colTop[(size_t)bz * nbx + bx];
                if (fz >= 0 && fz < nbz && t[(size_t)fz * nbx + bx] > m) m = t[(size_t)fz * nbx + bx];
                if (fx >= 0 && fx < nbx && t[(size_t)bz * nbx + fx] > m) m = t[(size_t)bz * nbx + fx];
                t[(size_t)bz * nbx + bx] = m;
            }
    // the cube-table walks: no sky exit (w.skyTop null, the reference walk)
    WorldDev wb = w;
    wb.brickSteps = 3;
    wb.skyTop = skyTop.data();  // the box walks end above every cube ahead when not heading down (sky_exit)
    if (std::string(argv[5]) == "--rays") {
        FILE *fr = fopen(argv[6], "rb");
        if (!fr) return 1;
        std::vector<float> rays;
        float buf[8];
        while (fread(buf, 4, 8, fr) == 8) rays.insert(rays.end(), buf, buf + 8);
        fclose(fr);
        const size_t n = rays.size() / 8;
        std::vector<int32_t> out(n * 16, 0);
        for (size_t i = 0; i < n; ++i) {
            const float *r = &rays[i * 8];
            const V3 o(r[0], r[1], r[2]), d(r[3], r[4], r[5]);
            int32_t *q = &out[i * 16];
            const Hit hc = dda_closest<false>(w, o, d, r[7]);
            Hit hb{0, 0, 0, 0, -1, 0, kRayMax};
            Dda sb;
            int rb = dda_begin<false, true>(wb, o, d, 0.0f, r[7], sb, hb);
            while (rb == DdaRun) {
                const DdaSaved sv = dda_save(sb, 0);
                dda_resume<true>(wb, o, d, 0.0f, r[7], sv, sb);
                rb = dda_iter<false, true, GlobalBricks, true>(wb, sb, hb);
            }
            if (rb != DdaEvent) hb = Hit{0, 0, 0, 0, -1, 0, kRayMax};
            const Hit hs[2] = {hc, hb};
            for (int k = 0; k < 2; ++k) {
                q[7 * k + 0] = hs[k].hit; q[7 * k + 1] = hs[k].x; q[7 * k + 2] = hs[k].y; q[7 * k + 3] = hs[k].z;
                q[7 * k + 4] = hs[k].face; q[7 * k + 5] = hs[k].id; q[7 * k + 6] = float_as_bits(hs[k].t);
            }
            q[14] = dda_occluded<false>(w, o, d, r[6], r[7]) ? 1 : 0;
            q[15] = dda_occluded<true, true>(wb, o, d, r[6], r[7]) ? 1 : 0;
        }
        FILE *fo = fopen(argv[7], "wb");
        if (!fo || fwrite(out.data(), 4, out.size(), fo) != out.size()) return 1;
        fclose(fo);
        return 0;
    }
    std::mt19937 rng(seed);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    long diff = 0, hits = 0, itCube = 0, itBox = 0, splitDiff = 0, splitRuns = 0;
    for (int i = 0; i < nrays; ++i) {
        const bool outside = i % 4 == 0;
        V3 o(U(rng) * wx, U(rng) * wy, U(rng) * wz);
        if (outside) o = V3(o.x * 3 - wx, o.y * 3 - wy, o.z * 3 - wz);
        V3 d(U(rng) * 2 - 1, U(rng) * 2 - 1, U(rng) * 2 - 1);
        if (i % 11 == 0) d.y = 0.0f;
        if (i % 13 == 0) d.x = 0.0f;
        if (i % 5 == 0) d.y = -fabsf(d.y) - 0.3f;  // toward the terrain
        const float len = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
        if (!(len > 0.0f)) continue;
        d = V3(d.x / len, d.y / len, d.z / len);
        const float tmax = (i % 7 == 0) ? 20.0f : 1e27f, tmin = (i % 3 == 0) ? 0.5f : 0.0f;
        Hit hc{0, 0, 0, 0, -1, 0, kRayMax}, hb{0, 0, 0, 0, -1, 0, kRayMax};
        Dda sc, sb;
        int rc = dda_begin<false, false>(w, o, d, 0.0f, tmax, sc, hc), n1 = 0;
        while (rc == DdaRun) { rc = dda_iter<false, false>(w, sc, hc); ++n1; }
        if (rc != DdaEvent) hc = Hit{0, 0, 0, 0, -1, 0, kRayMax};
        int rb = dda_begin<false, true>(wb, o, d, 0.0f, tmax, sb, hb), n2 = 0;
        while (rb == DdaRun) {
            // every other ray through the straggler hand-over (dda_save / dda_resume)
            if (i & 1) { const DdaSaved sv = dda_save(sb, 0); dda_resume<true>(wb, o, d, 0.0f, tmax, sv, sb); }
            rb = dda_iter<false, true, GlobalBricks, true>(wb, sb, hb);
            ++n2;
        }
        if (rb != DdaEvent) hb = Hit{0, 0, 0, 0, -1, 0, kRayMax};
        itCube += n1; itBox += n2;
        hits += hc.hit;
        const bool same = hc.hit == hb.hit && hc.x == hb.x && hc.y == hb.y && hc.z == hb.z && hc.face == hb.face &&
                          hc.id == hb.id && float_as_bits(hc.t) == float_as_bits(hb.t);
        const bool oc = dda_occluded<false>(w, o, d, tmin, tmax), ob = dda_occluded<true, true>(wb, o, d, tmin, tmax);
        for (int G : {2, 4, 8, 16}) {
            const int cap = i % 7;
            Hit hs;
            if (split_walk<false>(wb, o, d, 0.0f, tmax, cap, G, hs) != DdaEvent) hs = Hit{0, 0, 0, 0, -1, 0, kRayMax};
            Hit ho;
            const bool os = split_walk<true>(wb, o, d, tmin, tmax, cap, G, ho) == DdaEvent;
            const bool ss = hs.hit == hb.hit && hs.x == hb.x && hs.y == hb.y && hs.z == hb.z && hs.face == hb.face &&
                            hs.id == hb.id && float_as_bits(hs.t) == float_as_bits(hb.t);
            ++splitRuns;
            if (!ss || os != ob) {
                if (splitDiff < 5)
                    printf("split diff ray %d G %d cap %d: box hit %d (%d %d %d) f%d t %.9g | split hit %d (%d %d %d) f%d t %.9g | occ %d %d\n",
                           i, G, cap, hb.hit, hb.x, hb.y, hb.z, hb.face, hb.t, hs.hit, hs.x, hs.y, hs.z, hs.face, hs.t, ob, os);
                ++splitDiff;
            }
        }
        if (!same || oc != ob) {
            if (diff < 5)
                printf("diff ray %d: cube hit %d (%d %d %d) f%d t %.9g | box hit %d (%d %d %d) f%d t %.9g | occ %d %d\n", i,
                       hc.hit, hc.x, hc.y, hc.z, hc.face, hc.t, hb.hit, hb.x, hb.y, hb.z, hb.face, hb.t, oc, ob);
            ++diff;
        }
    }
    printf("rays %d hits %ld diff %ld split-runs %ld split-diff %ld iters cube %.3f box %.3f empty-entries %ld mean-growth %.3f\n",
           nrays, hits, diff, splitRuns, splitDiff, (double)itCube / nrays, (double)itBox / nrays, empties,
           empties ? (double)growX / empties : 0.0);
    return 0;
}
