// vxpt -- the optional empty-box skip tables of the voxel DDA (host only, no HIP).  Shared by
// vxpt_host.cpp and the CPU test driver (tests/native/box_tables_driver.cpp).
//
// For every empty brick and octant the walk may jump over an empty box of bricks that starts at
// the brick and extends in the octant's directions.  The default tables hold the largest such
// CUBE (octant_fill).  The box tables grow that cube along x, then z, then y, one brick at a time
// while the box stays empty, up to max(cube, cap) bricks per axis -- a flat terrain's empty space
// above it is wide and low, which a cube cannot follow (tools/dda_sim: a quarter fewer camera-ray
// iterations on the C3 world).  Bricks outside the world count as empty, as for the cubes; growth
// stops at the world's edge.  Entry = x | y << 8 | z << 16 extents in bricks, 0 = occupied.
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

namespace vx {

// 3-D prefix counts of occupied bricks on a BX x BY x BZ grid
struct BrickPrefix {
    int BX = 0, BY = 0, BZ = 0;
    std::vector<int> p;  // (BX + 1) x (BZ + 1) x (BY + 1), index x + (BX + 1) * (z + (BZ + 1) * y)
    int at(int x, int y, int z) const { return p[(size_t)x + (size_t)(BX + 1) * ((size_t)z + (size_t)(BZ + 1) * y)]; }
    template <class Occ>
    void build(int bx, int by, int bz, Occ occ) {
        BX = bx; BY = by; BZ = bz;
        p.assign((size_t)(BX + 1) * (BY + 1) * (BZ + 1), 0);
        for (int y = 1; y <= BY; ++y)
            for (int z = 1; z <= BZ; ++z)
                for (int x = 1; x <= BX; ++x)
                    p[(size_t)x + (size_t)(BX + 1) * ((size_t)z + (size_t)(BZ + 1) * y)] =
                        (occ(x - 1, y - 1, z - 1) ? 1 : 0) + at(x - 1, y, z) + at(x, y - 1, z) + at(x, y, z - 1) -
                        at(x - 1, y - 1, z) - at(x - 1, y, z - 1) - at(x, y - 1, z - 1) + at(x - 1, y - 1, z - 1);
    }
    // occupied bricks in [x0, x1) x [y0, y1) x [z0, z1), clamped to the grid
    int count(int x0, int y0, int z0, int x1, int y1, int z1) const {
        x0 = std::max(x0, 0); y0 = std::max(y0, 0); z0 = std::max(z0, 0);
        x1 = std::min(x1, BX); y1 = std::min(y1, BY); z1 = std::min(z1, BZ);
        if (x0 >= x1 || y0 >= y1 || z0 >= z1) return 0;
        return at(x1, y1, z1) - at(x0, y1, z1) - at(x1, y0, z1) - at(x1, y1, z0) + at(x0, y0, z1) + at(x0, y1, z0) +
               at(x1, y0, z0) - at(x0, y0, z0);
    }
};

constexpr int kBoxCap = 8;  // growth limit in bricks per axis (past the cube)

// the box of brick (x, y, z) in octant oct (bit a set: the ray moves + along axis a), grown from its
// cube edge S (0 = occupied)
// capUp: the growth limit along y in the upward octants (the empty space above a terrain is tall)
inline uint32_t grow_box(const BrickPrefix &P, int x, int y, int z, int oct, int S, int cap = kBoxCap,
                         int capUp = kBoxCap) {
    if (S <= 0) return 0u;
    const int b[3] = {x, y, z}, n[3] = {P.BX, P.BY, P.BZ};
    const int sg[3] = {(oct & 1) ? 1 : -1, (oct & 2) ? 1 : -1, (oct & 4) ? 1 : -1};
    int e[3] = {S, S, S};
    const int lim = std::min(255, std::max(S, cap));
    const int limUp = std::min(255, std::max(S, capUp));
    auto empty = [&](const int *ext) {
        int lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = sg[a] > 0 ? b[a] : b[a] - ext[a] + 1;
            hi[a] = sg[a] > 0 ? b[a] + ext[a] : b[a] + 1;
        }
        return P.count(lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]) == 0;
    };
    static const int order[3] = {0, 2, 1};
    for (int a : order)
        while (e[a] < (a == 1 && sg[1] > 0 ? limUp : lim)) {
            // the box already reaches the world's edge on this axis: growing adds nothing
            if (sg[a] > 0 ? b[a] + e[a] >= n[a] : b[a] - e[a] + 1 <= 0) break;
            int t[3] = {e[0], e[1], e[2]};
            ++t[a];
            if (!empty(t)) break;
            e[a] = t[a];
        }
    return (uint32_t)e[0] | ((uint32_t)e[1] << 8) | ((uint32_t)e[2] << 16);
}

}  // namespace vx
