// vxpt -- device-side building blocks of the trace pass (included by trace.hip only):
// voxel DDA, safe spawn, Disney BSDF, blue-noise sampler, light sampling,
// reservoirs, sky lookup.  See trace.hip for the pass structure.
#pragma once
#include <climits>
#include "vx_mesh.hpp"

namespace vx {
namespace {

constexpr uint32_t kValidBit = 0x80000000u, kIndexMask = 0x7FFFFFFFu;
constexpr uint32_t kInvalidLight = 0x7FFFFFFFu, kSkyLight = 0x7FFFFFFEu, kSunLight = 0x7FFFFFFDu;
enum { LtInvalid = 0, LtSky = 1, LtSun = 2, LtLocal = 3 };
constexpr float kRoughThresh = 0.00001f, kTranslThresh = 0.001f;
constexpr float kMinPdf = 1e-5f, kMaxThroughput = 32.0f, kMinLobe = 0.05f;

// ----------------------------------------------------------------- voxel DDA
// host + device bit casts (the walk also runs on the host in the CPU tests)
VX_HD float bits_as_float(int v) { return __builtin_bit_cast(float, v); }
VX_HD int float_as_bits(float v) { return __builtin_bit_cast(int, v); }
VX_HD bool is_cube(int id) { return id >= 1 && id <= 12; }

struct Hit { int hit, x, y, z, face, id; float t; };

VX_HD int entry_face(int a, int s) {
    return a == 0 ? (s > 0 ? 2 : 3) : (a == 1 ? (s > 0 ? 1 : 0) : (s > 0 ? 5 : 4));
}

// The walk keeps every per-axis quantity in named scalars (no runtime-indexed
// arrays: those would live in scratch on gfx950).
struct Ray3 {
    float ox, oy, oz, dx, dy, dz, ix, iy, iz;
    int sx, sy, sz;
    bool mx, my, mz;
};
struct Cell {
    int x, y, z;
    float tx, ty, tz;  // t of the next plane crossing on each axis (INF if the axis does not move)
};

// t of the next plane after cell c along one axis; the only formula for plane t,
// so skipped and stepped walks produce identical values.
VX_HD float next_t(int c, int s, float o, float inv, bool mv) {
    if (!mv) return INFINITY;
    return ((float)(s > 0 ? c + 1 : c) - o) * inv;
}
// axis order of the reference tie rule (VoxelEngine.cu:1040-1166 strict '<'):
// smallest t first, ties to Z, then Y, then X
VX_HD int pick3(float tx, float ty, float tz) {
    if (tx < ty) return tx < tz ? 0 : 2;
    return ty < tz ? 1 : 2;
}
VX_HD bool before(float t1, int a1, float t2, int a2) { return t1 < t2 || (t1 == t2 && a1 > a2); }

// brick index shared by bdist / cellMask / bricks (macro-major: a 16^3 macro
// cell's 64 bricks are contiguous) and the cell inside the brick
VX_HD int brick_index(const WorldDev &w, int x, int y, int z) {
    const int m = (x >> 4) + w.mx * ((z >> 4) + w.mz * (y >> 4));
    return m * 64 + (((x >> 2) & 3) + 4 * (((z >> 2) & 3) + 4 * ((y >> 2) & 3)));
}
VX_HD int cell_of(int x, int y, int z) { return (x & 3) + 4 * ((z & 3) + 4 * (y & 3)); }

// Advance one axis to the cell it occupies when the walk leaves the box through
// the crossing (Te, ea): exactly the planes the cell-by-cell walk would cross first.
VX_HD void skip_axis(int &cb, float &tb, int s, float o, float d, float inv, int lo, int hi, int ab, float Te, int ea) {
    int est = clampi((int)floorf(o + Te * d), lo, hi);
    est = s > 0 ? max(est, cb) : min(est, cb);
    while (est != cb) {
        const float te = ((float)(s > 0 ? est : est + 1) - o) * inv;  // plane entering est
        if (before(te, ab, Te, ea)) break;
        est -= s;
    }
    float tn = ((float)(s > 0 ? est + 1 : est) - o) * inv;
    while (before(tn, ab, Te, ea)) {
        est += s;
        tn = ((float)(s > 0 ? est + 1 : est) - o) * inv;
    }
    cb = est;
    tb = tn;
}
// Jump from the current cell to the last cell, inside the empty box of Sx x Sy x Sz
// bricks that starts at the current brick and extends in the ray's octant
// (clamped to the world), that the ray visits; the box's exit crossing is
// then the walk's next step.  The landing is exact per axis (skip_axis), so any
// empty box gives the cell-by-cell walk's result.
VX_HD void skip_box(const WorldDev &w, const Ray3 &r, Cell &c, int Sx, int Sy, int Sz) {
    const int ex = 4 * (Sx - 1), ey = 4 * (Sy - 1), ez = 4 * (Sz - 1);
    const int lx = r.sx > 0 ? (c.x & ~3) : max((c.x & ~3) - ex, 0), hx = r.sx > 0 ? min((c.x | 3) + ex, w.wx - 1) : (c.x | 3);
    const int ly = r.sy > 0 ? (c.y & ~3) : max((c.y & ~3) - ey, 0), hy = r.sy > 0 ? min((c.y | 3) + ey, w.wy - 1) : (c.y | 3);
    const int lz = r.sz > 0 ? (c.z & ~3) : max((c.z & ~3) - ez, 0), hz = r.sz > 0 ? min((c.z | 3) + ez, w.wz - 1) : (c.z | 3);
    const float Tx = r.mx ? ((float)(r.sx > 0 ? hx + 1 : lx) - r.ox) * r.ix : INFINITY;
    const float Ty = r.my ? ((float)(r.sy > 0 ? hy + 1 : ly) - r.oy) * r.iy : INFINITY;
    const float Tz = r.mz ? ((float)(r.sz > 0 ? hz + 1 : lz) - r.oz) * r.iz : INFINITY;
    const int ea = pick3(Tx, Ty, Tz);
    const float Te = ea == 0 ? Tx : (ea == 1 ? Ty : Tz);
    if (ea == 0) { c.x = r.sx > 0 ? hx : lx; c.tx = Tx; }
    else if (r.mx) skip_axis(c.x, c.tx, r.sx, r.ox, r.dx, r.ix, lx, hx, 0, Te, ea);
    if (ea == 1) { c.y = r.sy > 0 ? hy : ly; c.ty = Ty; }
    else if (r.my) skip_axis(c.y, c.ty, r.sy, r.oy, r.dy, r.iy, ly, hy, 1, Te, ea);
    if (ea == 2) { c.z = r.sz > 0 ? hz : lz; c.tz = Tz; }
    else if (r.mz) skip_axis(c.z, c.tz, r.sz, r.oz, r.dz, r.iz, lz, hz, 2, Te, ea);
}
// the empty cube of S bricks (the default tables)
VX_HD void skip_cube(const WorldDev &w, const Ray3 &r, Cell &c, int S) { skip_box(w, r, c, S, S, S); }

VX_HD bool slab(float o, float d, float W, int a, float &t0, float &t1, int &ax) {
    if (d == 0.0f) return !(o < 0.0f || o >= W);
    const float inv = 1.0f / d;
    const float ta = (0.0f - o) * inv, tb = (W - o) * inv;
    const float lo = ta < tb ? ta : tb, hi = ta < tb ? tb : ta;
    if (lo > t0) { t0 = lo; ax = a; }
    if (hi < t1) t1 = hi;
    return true;
}

// Start a walk; returns false if the ray never meets the world box.  For an
// origin outside the box, `outside` is set and the entry crossing (axis `ax`,
// t `tEnter`) is already taken.
VX_HD void ray_setup(V3 o, V3 d, Ray3 &r) {
    r.ox = o.x; r.oy = o.y; r.oz = o.z;
    r.dx = d.x; r.dy = d.y; r.dz = d.z;
    r.mx = d.x != 0.0f; r.my = d.y != 0.0f; r.mz = d.z != 0.0f;
    r.sx = d.x > 0.0f ? 1 : -1; r.sy = d.y > 0.0f ? 1 : -1; r.sz = d.z > 0.0f ? 1 : -1;
    r.ix = r.mx ? 1.0f / d.x : 0.0f; r.iy = r.my ? 1.0f / d.y : 0.0f; r.iz = r.mz ? 1.0f / d.z : 0.0f;
}
VX_HD bool walk_begin(const WorldDev &w, V3 o, V3 d, Ray3 &r, Cell &c, bool &outside, int &ax, float &tEnter) {
    ray_setup(o, d, r);
    c.x = (int)floorf(o.x); c.y = (int)floorf(o.y); c.z = (int)floorf(o.z);
    outside = !(c.x >= 0 && c.x < w.wx && c.y >= 0 && c.y < w.wy && c.z >= 0 && c.z < w.wz);
    if (outside) {
        // slab test against the world box, axes in x, y, z order
        float t0 = -INFINITY, t1 = INFINITY;
        ax = -1;
        if (!slab(o.x, d.x, (float)w.wx, 0, t0, t1, ax) || !slab(o.y, d.y, (float)w.wy, 1, t0, t1, ax) ||
            !slab(o.z, d.z, (float)w.wz, 2, t0, t1, ax))
            return false;
        if (ax < 0 || t0 > t1 || t1 <= 0.0f) return false;
        c.x = ax == 0 ? (d.x > 0.0f ? 0 : w.wx - 1) : clampi((int)floorf(o.x + t0 * d.x), 0, w.wx - 1);
        c.y = ax == 1 ? (d.y > 0.0f ? 0 : w.wy - 1) : clampi((int)floorf(o.y + t0 * d.y), 0, w.wy - 1);
        c.z = ax == 2 ? (d.z > 0.0f ? 0 : w.wz - 1) : clampi((int)floorf(o.z + t0 * d.z), 0, w.wz - 1);
        tEnter = t0;
    }
    c.tx = next_t(c.x, r.sx, r.ox, r.ix, r.mx);
    c.ty = next_t(c.y, r.sy, r.oy, r.iy, r.my);
    c.tz = next_t(c.z, r.sz, r.oz, r.iz, r.mz);
    return true;
}

// One step of the walk: cross the nearest plane.  Returns the crossed plane's
// t and coordinate and the face of the entered cell the crossing goes through.
VX_HD void walk_step(const Ray3 &r, Cell &c, float &t, int &planeCoord, int &face) {
    const int a = pick3(c.tx, c.ty, c.tz);
    if (a == 0) {
        t = c.tx; planeCoord = r.sx > 0 ? c.x + 1 : c.x; face = r.sx > 0 ? 2 : 3;
        c.x += r.sx; c.tx = next_t(c.x, r.sx, r.ox, r.ix, true);
    } else if (a == 1) {
        t = c.ty; planeCoord = r.sy > 0 ? c.y + 1 : c.y; face = r.sy > 0 ? 1 : 0;
        c.y += r.sy; c.ty = next_t(c.y, r.sy, r.oy, r.iy, true);
    } else {
        t = c.tz; planeCoord = r.sz > 0 ? c.z + 1 : c.z; face = r.sz > 0 ? 5 : 4;
        c.z += r.sz; c.tz = next_t(c.z, r.sz, r.oz, r.iz, true);
    }
}
VX_HD bool in_world(const WorldDev &w, const Cell &c) {
    return (unsigned)c.x < (unsigned)w.wx && (unsigned)c.y < (unsigned)w.wy && (unsigned)c.z < (unsigned)w.wz;
}
// face through which a ray entering the world box along axis ax enters the cell
VX_HD int entry_face_of(int ax, V3 d) {
    return ax == 0 ? (d.x > 0.0f ? 2 : 3) : (ax == 1 ? (d.y > 0.0f ? 1 : 0) : (d.z > 0.0f ? 5 : 4));
}

// Resumable walk state (dda_begin + dda_iter).  Block ids are read lazily:
// the face rule needs an id only when a crossing joins two cube cells (or for
// the hit record), so `prevId` is 0 (empty cell), the cube's id, or -1 (a
// cube whose id has not been read; its byte is bricks[prevLoc]).
struct Dda {
    Ray3 r;
    Cell c;
    const uint8_t *od;  // the ray octant's empty-cube table
    const uint32_t *ob; // the ray octant's empty-box table (BOX walks only)
    int nb;        // brick of the current cell
    int dist;      // its empty-cube edge in bricks (0 = occupied: walk its cells); BOX: the box's x extent
    uint32_t box;  // BOX walks: the box's packed extents
    uint64_t cm;   // its cube-cell mask (dist == 0)
    int prevId, prevLoc, steps;
    float tmin, tmax;
};
enum { DdaRun = 0, DdaEvent = 1, DdaNone = 2 };

// Where a walk reads a brick's skip-table entry and cube mask: global memory (every kernel but the
// LDS-cached camera walk of k_closest, trace.hip LdsBricks).  Sets s.box / s.dist; returns the mask.
struct GlobalBricks {
    template <bool BOX>
    VX_HD uint64_t fetch(const WorldDev &w, Dda &s, int nb) const {
        // the brick's cube mask is fetched beside its table entry, not behind it: one memory
        // round trip per new brick (8 wasted bytes for an empty one) instead of two
        const uint64_t m = w.cellMask[nb];
        if constexpr (BOX) {
            s.box = s.ob[nb];
            s.dist = (int)(s.box & 0xFFu);
        } else {
            s.dist = s.od[nb];
        }
        return m;
    }
};

// brick data of the walk's current cell (cached per brick); returns the cube bit
template <bool BOX = false, class F = GlobalBricks>
VX_HD bool locate(const WorldDev &w, Dda &s, const F &f = F()) {
    const int nb = brick_index(w, s.c.x, s.c.y, s.c.z);
    if (nb != s.nb) {
        s.nb = nb;
        const uint64_t m = f.template fetch<BOX>(w, s, nb);
        s.cm = s.dist ? 0ull : m;
    }
    return (s.cm >> cell_of(s.c.x, s.c.y, s.c.z)) & 1ull;
}
VX_HD int octant_of(const Ray3 &r) { return (r.sx > 0 ? 1 : 0) | (r.sy > 0 ? 2 : 0) | (r.sz > 0 ? 4 : 0); }
VX_HD int prev_id(const WorldDev &w, const Dda &s) { return s.prevId > 0 ? s.prevId : (int)w.bricks[s.prevLoc]; }

// The face rule at one crossing into a cell with cube bit `solid` (byte index
// `loc`).  Radiance rays (OCC = false): entering cube b from cell a hits iff
// a is empty, b != a, or the plane is a chunk boundary.  Visibility rays
// (OCC = true, t >= tmin): any crossing that enters or leaves a cube face
// (no culling).  Returns true on an event; otherwise updates prevId/prevLoc.
template <bool OCC>
VX_HD bool cross(const WorldDev &w, Dda &s, bool solid, int loc, bool chunkPlane, float t, int face, Hit &h) {
    if (OCC) {
        if (t >= s.tmin) {
            if (solid != (s.prevId != 0)) return true;
            if (solid) {
                if (chunkPlane) return true;
                const int bid = w.bricks[loc];
                if (bid != prev_id(w, s)) return true;
                s.prevId = bid;
            }
            return false;
        }
        s.prevId = solid ? -1 : 0;
        s.prevLoc = loc;
        return false;
    }
    if (!solid) { s.prevId = 0; return false; }
    const int bid = w.bricks[loc];
    if (s.prevId == 0 || chunkPlane || bid != prev_id(w, s)) {
        h = {1, s.c.x, s.c.y, s.c.z, face, bid, t};
        return true;
    }
    s.prevId = bid;
    return false;
}

// Walk the crossings that stay inside the current occupied 4^3 brick (cube
// bits in s.cm).  Inside a brick no crossing is a chunk plane or leaves the
// world.  Returns 0 when the next crossing leaves the brick (state = last cell
// inside), 1 on an event (h filled for radiance rays), 2 when t exceeds tmax,
// 3 after w.brickSteps crossings inside the brick (the walk continues there).
template <bool OCC>
VX_HD int brick_walk(const WorldDev &w, Dda &s, Hit &h, int *cnt = nullptr) {
    const Ray3 &r = s.r;
    Cell &c = s.c;
    int lc = cell_of(c.x, c.y, c.z);
    const uint64_t cm = s.cm;
    const int base = s.nb * 64;
    const int lim = w.brickSteps > 0 ? w.brickSteps : 10;
    for (int k = 0; k < 10; ++k) {  // at most 9 crossings stay inside a 4^3 brick
        if (k == lim) return 3;
        const int a = pick3(c.tx, c.ty, c.tz);
        if (cnt) ++*cnt;
        // per-axis choices as bit blends, not selects between struct fields (a
        // select of two loads becomes a load through a selected pointer, which
        // pins the walk state in scratch)
        const int mx = -(int)(a == 0), my = -(int)(a == 1), mz = -(int)(a == 2);
        const int sa = (r.sx & mx) | (r.sy & my) | (r.sz & mz);
        const int la = ((c.x & mx) | (c.y & my) | (c.z & mz)) & 3;
        if (sa > 0 ? la == 3 : la == 0) return 0;
        const float t = bits_as_float((float_as_bits(c.tx) & mx) | (float_as_bits(c.ty) & my) |
                                       (float_as_bits(c.tz) & mz));
        if (!(t <= s.tmax)) return 2;
        c.x += sa & mx;
        c.y += sa & my;
        c.z += sa & mz;
        const int ca = (c.x & mx) | (c.y & my) | (c.z & mz);
        const float oa = bits_as_float((float_as_bits(r.ox) & mx) | (float_as_bits(r.oy) & my) |
                                        (float_as_bits(r.oz) & mz));
        const float ia = bits_as_float((float_as_bits(r.ix) & mx) | (float_as_bits(r.iy) & my) |
                                        (float_as_bits(r.iz) & mz));
        const float nt = ((float)(sa > 0 ? ca + 1 : ca) - oa) * ia;
        c.tx = mx ? nt : c.tx;
        c.ty = my ? nt : c.ty;
        c.tz = mz ? nt : c.tz;
        lc += sa * ((1 & mx) | (16 & my) | (4 & mz));
        const bool solid = (cm >> lc) & 1ull;
        if (solid || s.prevId != 0) {
            const int face = (mx & (sa > 0 ? 2 : 3)) | (my & (sa > 0 ? 1 : 0)) | (mz & (sa > 0 ? 5 : 4));
            if (cross<OCC>(w, s, solid, base + lc, false, t, face, h)) return 1;
        }
    }
    return 0;
}

// Radiance rays (OCC = false): closest front-facing cube face, t <= tmax.
// Contract A4': entering cube cell b from a hits iff b != a, or the crossed
// plane is a chunk boundary, or a is outside the world.
// Visibility rays (OCC = true): any face crossing with tmin <= t <= tmax (no
// culling, so leaving a cube cell counts too).
template <bool OCC, bool BOX = false, class F = GlobalBricks>
VX_HD int dda_begin(const WorldDev &w, V3 o, V3 d, float tmin, float tmax, Dda &s, Hit &h, const F &f = F()) {
    bool outside;
    int ax = -1;
    float tEnter = 0;
    s.tmin = tmin;
    s.tmax = tmax;
    s.steps = 0;
    if (!walk_begin(w, o, d, s.r, s.c, outside, ax, tEnter)) return DdaNone;
    if constexpr (BOX) s.ob = w.bbox + (size_t)w.nBricks * octant_of(s.r);
    else s.od = w.bdist + (size_t)w.nBricks * octant_of(s.r);
    s.nb = -1;
    const bool solid = locate<BOX>(w, s, f);
    s.prevId = solid ? -1 : 0;
    s.prevLoc = s.nb * 64 + cell_of(s.c.x, s.c.y, s.c.z);
    if (outside) {
        if (tEnter > tmax) return DdaNone;
        if (solid && tEnter >= (OCC ? tmin : 0.0f)) {
            if (!OCC) h = {1, s.c.x, s.c.y, s.c.z, entry_face_of(ax, d), (int)w.bricks[s.prevLoc], tEnter};
            return DdaEvent;
        }
    }
    return DdaRun;
}

// Walk state as saved between launches (straggler continuation): the cell
// and its plane crossings, the face-rule state and the step count; the rest
// is rebuilt from the ray exactly as dda_begin builds it.
struct DdaSaved { int4 cell; float4 t; int2 face; };
VX_HD DdaSaved dda_save(const Dda &s, int entry) {
    return DdaSaved{make_int4(s.c.x, s.c.y, s.c.z, entry), make_float4(s.c.tx, s.c.ty, s.c.tz, 0.0f),
                    make_int2(s.prevLoc, (s.prevId + 1) | (s.steps << 16))};
}
template <bool BOX = false>
VX_HD void dda_resume(const WorldDev &w, V3 o, V3 d, float tmin, float tmax, const DdaSaved &v, Dda &s) {
    ray_setup(o, d, s.r);
    s.c.x = v.cell.x; s.c.y = v.cell.y; s.c.z = v.cell.z;
    s.c.tx = v.t.x; s.c.ty = v.t.y; s.c.tz = v.t.z;
    s.tmin = tmin;
    s.tmax = tmax;
    if constexpr (BOX) s.ob = w.bbox + (size_t)w.nBricks * octant_of(s.r);
    else s.od = w.bdist + (size_t)w.nBricks * octant_of(s.r);
    s.nb = -1;
    locate<BOX>(w, s);
    s.prevLoc = v.face.x;
    s.prevId = (v.face.y & 0xFFFF) - 1;
    s.steps = v.face.y >> 16;
}

// Segmented walks (k_resume, tuning resume_split): the rest of a walk cut into G pieces along the
// ray's dominant axis D, one lane each.  The walk's crossings are the per-axis plane crossings merged
// in the order `before` (t, then Z before Y before X), so the state after every crossing before D's
// plane P (t = T) is known without walking: axis D stands in the cell before P, every other axis in
// the cell skip_axis computes for (T, D).  A piece starts there (its cell's id state as dda_begin
// sets it: prevId always describes the walk's current cell) and ends at the next piece's T as its
// tmax, so the pieces together process every crossing of the walk.  A piece's first event is the
// walk's first event after the piece's start; the walk's result is that of the first piece with an
// event -- the cell-by-cell walk's, bit for bit.
//
// The dominant axis D and the number n of its cells between the walk's cell and where the walk
// ends (te: tmax, or the world box's exit); returns the pieces, min(G, n) (at least 1).  A piece
// whose boundary t is not before te (a rounding case at the last cell) is empty: the piece before it
// walks to the end.
// (per-axis choices as bit blends, as in brick_walk: a select between fields pins the walk in scratch)
VX_HD int blend_i(int D, int x, int y, int z) { return (x & -(int)(D == 0)) | (y & -(int)(D == 1)) | (z & -(int)(D == 2)); }
VX_HD float blend_f(int D, float x, float y, float z) {
    return bits_as_float(blend_i(D, float_as_bits(x), float_as_bits(y), float_as_bits(z)));
}
VX_HD int seg_plan(const WorldDev &w, const Dda &s, int G, int &D, int &n, float &te) {
    const Ray3 &r = s.r;
    const float ax = fabsf(r.dx), ay = fabsf(r.dy), az = fabsf(r.dz);
    D = (ax >= ay && ax >= az) ? 0 : (ay >= az ? 1 : 2);
    te = s.tmax;
    if (r.mx) te = fminf(te, ((float)(r.sx > 0 ? w.wx : 0) - r.ox) * r.ix);
    if (r.my) te = fminf(te, ((float)(r.sy > 0 ? w.wy : 0) - r.oy) * r.iy);
    if (r.mz) te = fminf(te, ((float)(r.sz > 0 ? w.wz : 0) - r.oz) * r.iz);
    const int c = blend_i(D, s.c.x, s.c.y, s.c.z), sd = blend_i(D, r.sx, r.sy, r.sz);
    const float o = blend_f(D, r.ox, r.oy, r.oz), d = blend_f(D, r.dx, r.dy, r.dz);
    const int wd = blend_i(D, w.wx, w.wy, w.wz);
    const int e = clampi((int)floorf(o + te * d), 0, wd - 1);
    n = sd > 0 ? e - c : c - e;
    return n < 1 ? 1 : (n < G ? n : G);
}
// piece k's boundary (1 <= k < pieces): D's plane P entering the piece's first D-cell
// (k * n / pieces cells ahead of the walk's cell), and its t by next_t's formula
VX_HD float seg_bound(const Dda &s, int D, int k, int pieces, int n, int &P) {
    const Ray3 &r = s.r;
    const int c = blend_i(D, s.c.x, s.c.y, s.c.z), sd = blend_i(D, r.sx, r.sy, r.sz);
    const float o = blend_f(D, r.ox, r.oy, r.oz), inv = blend_f(D, r.ix, r.iy, r.iz);
    const int q = c + sd * (k * n / pieces);
    P = sd > 0 ? q : q + 1;
    return ((float)P - o) * inv;
}
template <bool BOX = false>
VX_HD void dda_seg_start(const WorldDev &w, Dda &s, int D, int P, float T) {
    const Ray3 &r = s.r;
    Cell &c = s.c;
    if (D == 0) { c.x = r.sx > 0 ? P - 1 : P; c.tx = T; }
    else if (r.mx) skip_axis(c.x, c.tx, r.sx, r.ox, r.dx, r.ix, 0, w.wx - 1, 0, T, D);
    if (D == 1) { c.y = r.sy > 0 ? P - 1 : P; c.ty = T; }
    else if (r.my) skip_axis(c.y, c.ty, r.sy, r.oy, r.dy, r.iy, 0, w.wy - 1, 1, T, D);
    if (D == 2) { c.z = r.sz > 0 ? P - 1 : P; c.tz = T; }
    else if (r.mz) skip_axis(c.z, c.tz, r.sz, r.oz, r.dz, r.iz, 0, w.wz - 1, 2, T, D);
    s.nb = -1;
    const bool solid = locate<BOX>(w, s);
    s.prevId = solid ? -1 : 0;
    s.prevLoc = s.nb * 64 + cell_of(c.x, c.y, c.z);
}

// SKY: the walk may end above the cubes it can still reach (WorldDev::skyTop, below); a compile-time
// switch so that the walks without it (camera rays, a queue's first iterations) keep their code
template <bool OCC, bool BOX = false, class F = GlobalBricks, bool SKY = false>
VX_HD int dda_iter(const WorldDev &w, Dda &s, Hit &h, int *cnt = nullptr, const F &f = F()) {
    if (++s.steps > w.wx + w.wy + w.wz + 3) return DdaNone;
    if (cnt) ++cnt[s.dist == 0 ? 3 : (s.dist == 1 ? 2 : 1)];
    if (s.dist == 0) {
        const int rc = brick_walk<OCC>(w, s, h, cnt ? cnt + 4 : nullptr);
        if (rc == 1) return DdaEvent;
        if (rc == 2) return DdaNone;
        if (rc == 3) {  // a continuation of the same brick: not a new step of the step bound
            --s.steps;
            return DdaRun;
        }
    } else {
        if constexpr (BOX) skip_box(w, s.r, s.c, (int)(s.box & 0xFFu), (int)((s.box >> 8) & 0xFFu), (int)((s.box >> 16) & 0xFFu));
        else skip_cube(w, s.r, s.c, s.dist);
    }
    // sky exit, after an empty box (not per cell step): see below
    const bool skyCheck = SKY && s.dist != 0 && w.skyTop && !(s.r.dy < 0.0f);
    // the next crossing leaves the brick (or the skipped box)
    float t;
    int planeCoord, face;
    walk_step(s.r, s.c, t, planeCoord, face);
    if (!(t <= s.tmax)) return DdaNone;
    const bool chunkPlane = (planeCoord & 31) == 0;
    const bool out = !in_world(w, s.c);
    if (out) {
        // leaving the world: only a visibility ray leaving a cube cell sees a face
        return (OCC && t >= s.tmin && s.prevId != 0) ? DdaEvent : DdaNone;
    }
    // sky exit: the walk left an empty box (prevId 0: no cube left behind) into a cell at or above every
    // cube cell of the brick columns it can still reach (x and z only move with the ray, y does not
    // fall), so this cell is empty and no crossing ahead joins or leaves a cube -- the cell-by-cell walk
    // would reach the world's edge without an event.  The table entry is fetched beside the brick's.
    int top = INT_MAX;
    if constexpr (SKY)
        if (skyCheck)
            top = (int)w.skyTop[((size_t)((s.r.sx > 0 ? 1 : 0) | (s.r.sz > 0 ? 2 : 0)) * (w.wz >> 2) + (s.c.z >> 2)) *
                                    (w.wx >> 2) + (s.c.x >> 2)];
    const bool solid = locate<BOX>(w, s, f);
    if constexpr (SKY)
        if (s.c.y >= top) return DdaNone;
    if (solid || s.prevId != 0) {
        if (cross<OCC>(w, s, solid, s.nb * 64 + cell_of(s.c.x, s.c.y, s.c.z), chunkPlane, t, face, h))
            return DdaEvent;
    }
    return DdaRun;
}

template <bool BOX = false, class F = GlobalBricks, bool SKY = false>
VX_HD Hit dda_closest(const WorldDev &w, V3 o, V3 d, float tmax, int *iters = nullptr, const F &f = F()) {
    Hit h{0, 0, 0, 0, -1, 0, kRayMax};
    Dda s;
    int rc = dda_begin<false, BOX>(w, o, d, 0.0f, tmax, s, h, f);
    while (rc == DdaRun) rc = dda_iter<false, BOX, F, SKY>(w, s, h, iters, f);
    if (rc != DdaEvent) h = Hit{0, 0, 0, 0, -1, 0, kRayMax};
    return h;
}

template <bool BOX = false, bool SKY = false>
VX_HD bool dda_occluded(const WorldDev &w, V3 o, V3 d, float tmin, float tmax, int *iters = nullptr) {
    Hit h;
    Dda s;
    int rc = dda_begin<true, BOX>(w, o, d, tmin, tmax, s, h);
    while (rc == DdaRun) rc = dda_iter<true, BOX, GlobalBricks, SKY>(w, s, h, iters);
    return rc == DdaEvent;
}

VX_D V3 face_normal(int f) {
    return f == 0 ? V3(0, 1, 0) : f == 1 ? V3(0, -1, 0) : f == 2 ? V3(-1, 0, 0) : f == 3 ? V3(1, 0, 0)
         : f == 4 ? V3(0, 0, 1) : V3(0, 0, -1);
}

// Hit point on the face plane + self-intersection-safe spawn points
// (SelfHit.h:539-656 specialised to unit quads under one translation instance).
VX_D void hit_frame(const Hit &h, V3 o, V3 d, V3 &front, V3 &back, V3 &ng) {
    V3 p = o + d * h.t;
    const bool ax0 = h.face == 2 || h.face == 3, ax1 = h.face < 2;  // else z (faces 4, 5)
    // blend instead of selecting a field by index: keeps h and p in registers
    const int cell = (ax0 ? h.x : 0) + (ax1 ? h.y : 0) + ((!ax0 && !ax1) ? h.z : 0);
    const bool high = (h.face == 0 || h.face == 3 || h.face == 4);
    const int plane = cell + (high ? 1 : 0);
    const float pa = (float)plane;
    ng = face_normal(h.face);
    const int T = (cell >> 5) * 32;
    const float planeLocal = (float)(plane - T), planeWorld = (float)plane, Tf = (float)T;
    const float c0t = 5.9604648328104529e-08f, c1t = 1.1920930376163769e-07f;
    const float eps = mul_ru(c1t, 2.0f);
    const float triErr = fma_ru(c0t, planeLocal, eps);
    const float cI = 1.19209317972490680404007434844970703125E-7f;
    const float wldErr = fma_ru(cI, planeLocal, mul_ru(cI, Tf));
    const float objErr = fma_ru(cI, planeWorld, mul_ru(cI, Tf));
    float off = add_ru(objErr, triErr);
    off = off + wldErr;
    // outward normal component along the axis is +1 for the high faces, -1 otherwise
    const float n = high ? 1.0f : -1.0f;
    const float fa = high ? fma_ru(off, n, pa) : fma_rd(off, n, pa);
    const float ba = high ? fma_rd(-off, n, pa) : fma_ru(-off, n, pa);
    front = V3(ax0 ? fa : p.x, ax1 ? fa : p.y, (!ax0 && !ax1) ? fa : p.z);
    back = V3(ax0 ? ba : p.x, ax1 ? ba : p.y, (!ax0 && !ax1) ? ba : p.z);
}

// ----------------------------------------------------------------- BSDF
VX_D V3 clamp_throughput(V3 v) {
    const float l = luminance(v), a = fabsf(l);
    if (a > kMaxThroughput && a > 0.0f) return v * (kMaxThroughput / a);
    return v;
}
VX_D float disney_diffuse_fresnel(float cwo, float cwi, float r) {
    const float eb = lerpf(0.0f, 0.5f, r), ef = lerpf(1.0f, 1.0f / 1.51f, r);
    const float fd90 = eb + 2.0f * r * cwi * cwi;
    const float ls = 1.0f + (fd90 - 1.0f) * pow5(1.0f - cwo);
    const float vs = 1.0f + (fd90 - 1.0f) * pow5(1.0f - cwi);
    return ls * vs * ef;
}
VX_D float gtr2(float ch, float sh, float a) {  // GTR2Aniso(ch, sh, 0, 1, a, a)
    const float a2 = a * a;
    const float s = (1.0f * 1.0f) / a2 + (0.0f * 0.0f) / a2;
    const float t = sh * sh * s + ch * ch;
    return 1.0f / (kPi * a * a * t * t);
}
VX_D float smith_g(float c, float a) {
    const float a2 = a * a, c2 = c * c;
    return 2.0f / (1.0f + sqrtf(1.0f + a2 * (1.0f - c2) / c2));
}

struct Lobes { V3 C0; float sp, dp; };
VX_D bool lobes(V3 albedo, float metalness, float cosForF, Lobes &L) {
    const float lum = 0.299f * albedo.x + 0.587f * albedo.y + 0.114f * albedo.z;
    const V3 tint = lum > 0.0f ? albedo / lum : V3(1.0f);
    const V3 specColor = lerp3(V3(1.0f), tint, 0.0f);
    L.C0 = lerp3(0.08f * 0.5f * specColor, albedo, metalness);
    const V3 F = L.C0 + (V3(1.0f) - L.C0) * pow5(1.0f - cosForF);
    const float avgF = (F.x + F.y + F.z) / 3.0f;
    const float sw = avgF, dw = (1.0f - metalness) * (1.0f - avgF), tw = sw + dw;
    if (tw < kSafeCos) return false;
    float sp = sw / tw;
    if (dw > kSafeCos && sw > kSafeCos) sp = clampf(sp, kMinLobe, 1.0f - kMinLobe);
    L.sp = clampf(sp, 0.0f, 1.0f);
    L.dp = fmaxf(0.0f, 1.0f - L.sp);
    return true;
}

// EvaluateFresnelDielectric (Bsdf.h:40-65)
VX_D float fresnel_dielectric(float et, float cosIn) {
    const float cosi = fabsf(cosIn);
    float sint = 1.0f - cosi * cosi;
    sint = (0.0f < sint) ? sqrtf(sint) / et : 0.0f;
    if (1.0f < sint) return 1.0f;
    float cost = 1.0f - sint * sint;
    cost = (0.0f < cost) ? sqrtf(cost) : 0.0f;
    const float ec = et * cosi, ect = et * cost;
    const float rPerp = (cosi - ect) / (cosi + ect);
    const float rPar = (ec - cost) / (ec + cost);
    const float r = (rPar * rPar + rPerp * rPerp) * 0.5f;
    return r <= 1.0f ? r : 1.0f;
}
// refract (LinearMath.h:1483-1513): false on total internal reflection
VX_D bool refract3(V3 &r, V3 i, V3 n, float ior) {
    float neg = dot(i, n), eta;
    if (neg > 0.0f) { eta = ior; n = -n; neg = -neg; } else eta = 1.0f / ior;
    const float k = 1.0f - eta * eta * (1.0f - neg * neg);
    if (k < 0.0f) { r = V3(0.0f); return false; }
    r = normalize(eta * i - (eta * neg + sqrtf(k)) * n);
    return true;
}
// SpecularReflectionTransmissionSample (Bsdf.h:218-245), ior 1.4; the
// transmission flag only matters for thin films (closesthit.cu:293)
VX_D void spec_refl_trans_sample(float u, V3 n, V3 ng, V3 wo, V3 albedo, V3 &wi, V3 &bop, float &pdf) {
    const float ior = 1.4f;
    const float eta = dot(wo, ng) > 0.0f ? ior / 1.0f : 1.0f / ior;
    const V3 wr = reflect3(-wo, n);
    V3 wt;
    float R = 1.0f;
    if (refract3(wt, -wo, n, eta)) R = fresnel_dielectric(eta, dot(wo, n));
    if (u <= R) { wi = wr; pdf = R; } else { wi = wt; pdf = 1.0f - R; }
    bop = albedo / pdf;
}

// DisneyBSDFSample for rough surfaces (Bsdf.h:401-534); specular branch of
// the reference only for roughness < 1e-5 (:403-425).
VX_D void disney_sample(float u0, float u1, float u2, float u3, V3 n, V3 ng, V3 wo, V3 albedo, bool metallic,
                        float translucency, float roughness, V3 &wi, V3 &bop, float &pdf) {
    if (roughness < kRoughThresh) {
        if (translucency < kTranslThresh) {
            wi = reflect3(-wo, n);
            if (dot(wi, n) <= 0.0f || dot(wi, ng) <= 0.0f) { bop = V3(0.0f); pdf = 0.0f; }
            else { bop = albedo; pdf = 1.0f; }
            pdf = fmaxf(pdf, kMinPdf);
            bop = clamp_throughput(bop);
        } else if (translucency > 1.0f - kTranslThresh) {
            spec_refl_trans_sample(u0, n, ng, wo, albedo, wi, bop, pdf);
            pdf = fmaxf(pdf, kMinPdf);
            bop = clamp_throughput(bop);
        } else {
            bop = V3(0.0f);
            pdf = 0.0f;
        }
        return;
    }
    const float metalness = metallic ? 1.0f : 0.0f;
    const float alpha = fmaxf(roughness * roughness, kRoughThresh);
    const float cwo = fmaxf(kSafeCos, dot(n, wo));
    Lobes L;
    if (!lobes(albedo, metalness, cwo, L)) { bop = V3(0.0f); pdf = 0.0f; return; }
    if (u3 < L.sp) {
        float ct = sqrtf((1.0f - u0) / (1.0f + (alpha * alpha - 1.0f) * u0));
        ct = clampf(ct, kSafeCos, 1.0f);
        const float st = sqrtf(fmaxf(0.0f, 1.0f - ct * ct));
        const float phi = kTwoPi * u1;
        V3 wh(st * cosf(phi), st * sinf(phi), ct);
        align_vector(n, wh);
        wi = normalize(reflect3(-wo, wh));
        if (dot(wi, n) <= 0.0f || dot(wi, ng) <= 0.0f) { bop = V3(0.0f); pdf = 0.0f; return; }
        const float cwi = dot(wi, n);
        const float cwh = fmaxf(kSafeCos, fabsf(dot(wh, n)));
        const float cwowh = fmaxf(kSafeCos, fabsf(dot(wo, wh)));
        const float swh = sqrtf(fmaxf(0.0f, 1.0f - cwh * cwh));
        const float D = gtr2(cwh, swh, alpha);
        const V3 Fs = L.C0 + (V3(1.0f) - L.C0) * pow5(1.0f - cwowh);
        const float G = smith_g(cwo, alpha) * smith_g(cwi, alpha);
        const V3 brdf = Fs * D * G / (4.0f * cwo * cwi);
        float mpdf = fmaxf(D * cwh / (4.0f * cwowh), kMinPdf);
        pdf = fmaxf(mpdf * fmaxf(L.sp, kMinPdf), kMinPdf);
        bop = clamp_throughput(brdf * cwi / pdf);
    } else {
        const float ct = sqrtf(u0);
        const float st = sqrtf(fmaxf(0.0f, 1.0f - ct * ct));
        const float phi = kTwoPi * u1;
        wi = V3(st * cosf(phi), st * sinf(phi), ct);
        align_vector(n, wi);
        if (dot(wi, ng) <= 0.0f) { bop = V3(0.0f); pdf = 0.0f; return; }
        const float cwi = fmaxf(kSafeCos, dot(wi, n));
        const float fl = disney_diffuse_fresnel(cwo, cwi, roughness);
        const V3 db = albedo * (1.0f - metalness) * fl / kPi;
        float dpdf = fmaxf(cwi / kPi, kMinPdf);
        pdf = fmaxf(dpdf * fmaxf(L.dp, kMinPdf), kMinPdf);
        bop = clamp_throughput(db * cwi / pdf);
    }
}

VX_D void disney_eval(V3 n, V3 ng, V3 wi, V3 wo, V3 albedo, bool metallic, float roughness, V3 &bsdf, float &pdf) {
    bsdf = V3(0.0f);
    if (roughness < kRoughThresh) { pdf = 0.0f; return; }
    if (dot(wo, n) <= 0.0f || dot(wi, n) <= 0.0f || dot(wo, ng) <= 0.0f || dot(wi, ng) <= 0.0f) { pdf = 0.0f; return; }
    const float metalness = metallic ? 1.0f : 0.0f;
    const float alpha = fmaxf(roughness * roughness, kRoughThresh);
    const float cwo = dot(wo, n), cwi = dot(wi, n);
    const V3 wh = normalize(wi + wo);
    const float cwh = fmaxf(kSafeCos, fabsf(dot(wh, n)));
    const float cwowh = fmaxf(kSafeCos, fabsf(dot(wo, wh)));
    Lobes L;
    const bool ok = lobes(albedo, metalness, cwowh, L);
    const V3 F = L.C0 + (V3(1.0f) - L.C0) * pow5(1.0f - cwowh);
    V3 diffuse(0.0f);
    if (!metallic) diffuse = albedo * (1.0f - metalness) * disney_diffuse_fresnel(cwo, cwi, roughness) / kPi;
    const float swh = sqrtf(fmaxf(0.0f, 1.0f - cwh * cwh));
    const float D = gtr2(cwh, swh, alpha);
    const float G = smith_g(cwo, alpha) * smith_g(cwi, alpha);
    const V3 spec = F * D * G / (4.0f * cwo * cwi);
    bsdf = clamp_throughput(diffuse + spec);
    if (!ok) { pdf = 0.0f; return; }
    const float dpdf = fmaxf(cwi / kPi, kMinPdf);
    const float spdf = fmaxf(D * cwh / (4.0f * cwowh), kMinPdf);
    pdf = fmaxf(dpdf * fmaxf(L.dp, kMinPdf) + spdf * fmaxf(L.sp, kMinPdf), kMinPdf);
}

// ----------------------------------------------------------------- sampling
struct Rng {
    const BlueNoiseDev *bn;
    int px, py, it, idx;
    VX_D float next() {  // BlueNoiseRandGenerator::rand (RandGen.h:21-45)
        const int i = px & 127, j = py & 127, s = it & 255, d = idx++;
        const int rk = s ^ bn->rank[(d + (i + j * 128) * 8) & (128 * 128 * 8 - 1)];
        int v = bn->sobol[d + rk * 256];
        v ^= bn->scramble[(d % 8) + (i + j * 128) * 8];
        return v / 256.0f;
    }
};
VX_D float bn_rand(const BlueNoiseDev &bn, int px, int py, int it, int d) {
    const int i = px & 127, j = py & 127, s = it & 255;
    const int rk = s ^ bn.rank[(d + (i + j * 128) * 8) & (128 * 128 * 8 - 1)];
    int v = bn.sobol[d + rk * 256];
    v ^= bn.scramble[(d % 8) + (i + j * 128) * 8];
    return v / 256.0f;
}

VX_D unsigned alias_sample(const AliasBin *b, int len, float u, float &pmf) {
    const int offset = min(int(u * len), int(len - 1));
    const float up = fminf(u * len - offset, 0.999999f);
    const AliasBin e = b[offset];
    if (up < e.q) { pmf = e.p; return offset; }
    pmf = b[e.alias].p;
    return e.alias;
}

struct LSample { V3 position, radiance; float solidAnglePdf; int type; };

VX_D V3 ld3(const float4 *p, size_t i) { const float4 v = p[i]; return V3(v.x, v.y, v.z); }

VX_D LSample sun_ls(const SkyDev &k, int idx) {
    const int sx = idx % k.sunW, sy = idx / k.sunW;
    LSample s;
    s.solidAnglePdf = (k.sunW * k.sunH) / (kTwoPi * (1.0f - k.sunCosMax));
    s.position = eq_area_cone_dir(k.sunDir, (sx + 0.5f) / float(k.sunW), (sy + 0.5f) / float(k.sunH), k.sunCosMax);
    s.radiance = ld3(k.sun, (size_t)clampi(sy, 0, k.sunH - 1) * k.sunW + clampi(sx, 0, k.sunW - 1));
    s.type = LtSun;
    return s;
}
VX_D LSample sky_ls(const SkyDev &k, int idx) {
    const int sx = idx % k.skyW, sy = idx / k.skyW;
    LSample s;
    s.solidAnglePdf = (k.skyW * k.skyH) / (4.0f * kPi);
    s.position = eq_area_sphere_dir((sx + 0.5f) / float(k.skyW), (sy + 0.5f) / float(k.skyH));
    s.radiance = ld3(k.sky, (size_t)sy * k.skyW + sx);
    s.type = LtSky;
    return s;
}

// the same samples with the position given (a stored light sample's direction, trace.hip load_ls)
VX_D LSample sun_ls_at(const SkyDev &k, int idx, V3 dir) {
    const int sx = idx % k.sunW, sy = idx / k.sunW;
    LSample s;
    s.solidAnglePdf = (k.sunW * k.sunH) / (kTwoPi * (1.0f - k.sunCosMax));
    s.position = dir;
    s.radiance = ld3(k.sun, (size_t)clampi(sy, 0, k.sunH - 1) * k.sunW + clampi(sx, 0, k.sunW - 1));
    s.type = LtSun;
    return s;
}
VX_D LSample sky_ls_at(const SkyDev &k, int idx, V3 dir) {
    LSample s;
    s.solidAnglePdf = (k.skyW * k.skyH) / (4.0f * kPi);
    s.position = dir;
    s.radiance = ld3(k.sky, (size_t)idx);
    s.type = LtSky;
    return s;
}

struct SurfS {
    V3 pos, normal, geoNormal, albedo, wo;
    float depth, roughness, translucency;
    bool metallic;
};

// the direction a light sample is seen in from p: local lights by position (closesthit.cu:610,
// Restir.h:201), environment samples carry it
VX_D V3 light_dir(const LSample &ls, V3 p) { return ls.type == LtLocal ? normalize(ls.position - p) : ls.position; }
VX_D float target_pdf(const LSample &ls, const SurfS &sf) {  // Restir.h:194-211
    if (ls.solidAnglePdf <= 0 || ls.type == LtInvalid) return 0.0f;
    const V3 wi = light_dir(ls, sf.pos);
    V3 fr;
    float pdf;
    disney_eval(sf.normal, sf.geoNormal, wi, sf.wo, sf.albedo, sf.metallic, sf.roughness, fr, pdf);
    return luminance(ls.radiance * fr * fabsf(dot(wi, sf.normal)) / ls.solidAnglePdf);
}
VX_D float mis_weight(const SurfS &sf, const LSample &ls, float selPdf, float lightMis, float brdfMis) {
    const float sa = ls.solidAnglePdf;  // Restir.h:286-328 (brdfCutoff 0)
    if (brdfMis == 0.0f || sa <= 0.0f || isinf(sa) || isnan(sa)) return lightMis * selPdf;
    V3 dir = ls.position;
    if (ls.type == LtLocal) {
        const V3 toLight = ls.position - sf.pos;
        dir = toLight / length(toLight);
    }
    V3 fr;
    float bp;
    disney_eval(sf.normal, sf.geoNormal, dir, sf.wo, sf.albedo, sf.metallic, sf.roughness, fr, bp);
    return (lightMis * (selPdf * sa) + brdfMis * bp) / sa;
}
// TriangleLight::calcSample (Light.h:54-82; SampleTriangle LinearMath.h:2048-2056, PdfAtoW :2125)
VX_D LSample tri_sample(const TriL &t, V2 uv, V3 viewer) {
    const float sx = sqrtf(uv.x);
    LSample r;
    r.position = t.base + t.e1 * (sx * (1.0f - uv.y)) + t.e2 * (sx * uv.y);
    V3 L = r.position - viewer;
    const float Ld = length(L);
    L /= Ld;
    const float areaPdf = 1.0f / t.area;
    const float cosT = saturate(dot(L, -t.n));
    r.solidAnglePdf = areaPdf * (Ld * Ld) / cosT;
    r.radiance = t.rad;
    r.type = LtLocal;
    return r;
}
VX_D V2 inverse_tri_sample(float u, float v) {  // InverseTriangleSample (LinearMath.h:2059-2064)
    const float b0 = 1.0f - u - v, sx = 1 - b0;
    return V2(sx * sx, v / sx);
}
// mis_weight and target_pdf of one environment candidate with a single BSDF evaluation (both
// evaluate the same Disney lobe for the same surface and direction; results identical to the
// two calls).  Local lights normalise their direction two ways and go through the two calls.
VX_D void mis_and_target(const SurfS &sf, const LSample &ls, float selPdf, float lightMis, float brdfMis,
                         float &blended, float &tp) {
    if (ls.type == LtLocal) {
        blended = mis_weight(sf, ls, selPdf, lightMis, brdfMis);
        tp = target_pdf(ls, sf);
        return;
    }
    const float sa = ls.solidAnglePdf;
    const bool tpEval = !(sa <= 0 || ls.type == LtInvalid);
    const bool misEval = !(brdfMis == 0.0f || sa <= 0.0f || isinf(sa) || isnan(sa));
    V3 fr(0.0f);
    float bp = 0.0f;
    if (tpEval || misEval)
        disney_eval(sf.normal, sf.geoNormal, ls.position, sf.wo, sf.albedo, sf.metallic, sf.roughness, fr, bp);
    blended = misEval ? (lightMis * (selPdf * sa) + brdfMis * bp) / sa : lightMis * selPdf;
    tp = tpEval ? luminance(ls.radiance * fr * fabsf(dot(ls.position, sf.normal)) / ls.solidAnglePdf) : 0.0f;
}
VX_D bool stream_sample(Reservoir &r, uint32_t light, V2 uv, float rnd, float target, float invSrc) {
    const float w = target * invSrc;
    r.M += 1;
    r.weightSum += w;
    const bool sel = (rnd * r.weightSum < w);
    if (sel) {
        r.lightData = light | kValidBit;
        r.uvData = (uint32_t)(saturate(uv.x) * 0xffff) | ((uint32_t)(saturate(uv.y) * 0xffff) << 16);
        r.targetPdf = target;
    }
    return sel;
}
VX_D bool combine(Reservoir &r, const Reservoir &n, float rnd, float target) {
    const float w = target * (n.weightSum * n.M);
    r.M += n.M;
    r.weightSum += w;
    const bool sel = (rnd * r.weightSum < w);
    if (sel) { r.lightData = n.lightData; r.uvData = n.uvData; r.targetPdf = target; }
    return sel;
}
VX_D void finalize(Reservoir &r, float num, float den) {
    const float d = r.targetPdf * den;
    r.weightSum = (d == 0.0f) ? 0.0f : (r.weightSum * num) / d;
}
VX_D Reservoir empty_res() { return Reservoir{0u, 0u, 0.0f, 0.0f, 0.0f}; }

// GetLightSampleFromReservoir (Restir.h:383-415); local lights are sampled as seen from `pos`
VX_D bool light_from_res(const TraceArgs &a, LSample &ls, const Reservoir &r, V3 pos, bool hasLocal) {
    const SkyDev &k = a.sky;
    const uint32_t li = r.lightData & kIndexMask;
    const float ux = (float)(r.uvData & 0xffff) / float(0xffff), uy = (float)(r.uvData >> 16) / float(0xffff);
    if (li == kSkyLight) {
        const int x = clampi(int(ux * k.skyW), 0, k.skyW - 1), y = clampi(int(uy * k.skyH), 0, k.skyH - 1);
        ls = sky_ls(k, y * k.skyW + x);
    } else if (li == kSunLight) {
        const int x = clampi(int(ux * k.sunW), 0, k.sunW - 1), y = clampi(int(uy * k.sunH), 0, k.sunH - 1);
        ls = sun_ls(k, y * k.sunW + x);
    } else if (hasLocal && li < (uint32_t)a.numLights) {
        ls = tri_sample(tri_light(a.lights[li]), V2(ux, uy), pos);
        return true;
    }
    return li < kInvalidLight;
}
// light_from_res in two steps, so that several reservoirs' table reads are in flight together:
// env_entry issues the environment light's radiance read (the sky or sun table entry; for any other
// light sky entry 0, unused), light_from_entry finishes with it -- light_from_res's values exactly
VX_D float4 env_entry(const SkyDev &k, const Reservoir &r) {
    const uint32_t li = r.lightData & kIndexMask;
    const float ux = (float)(r.uvData & 0xffff) / float(0xffff), uy = (float)(r.uvData >> 16) / float(0xffff);
    const bool sun = li == kSunLight;
    const int w = sun ? k.sunW : k.skyW, h = sun ? k.sunH : k.skyH;
    const int x = clampi(int(ux * w), 0, w - 1), y = clampi(int(uy * h), 0, h - 1);
    return (sun ? k.sun : k.sky)[(sun || li == kSkyLight) ? (size_t)y * w + x : 0];
}
VX_D bool light_from_entry(const TraceArgs &a, LSample &ls, const Reservoir &r, V3 pos, bool hasLocal, float4 e) {
    const SkyDev &k = a.sky;
    const uint32_t li = r.lightData & kIndexMask;
    const float ux = (float)(r.uvData & 0xffff) / float(0xffff), uy = (float)(r.uvData >> 16) / float(0xffff);
    if (li == kSkyLight) {
        const int x = clampi(int(ux * k.skyW), 0, k.skyW - 1), y = clampi(int(uy * k.skyH), 0, k.skyH - 1);
        ls.solidAnglePdf = (k.skyW * k.skyH) / (4.0f * kPi);  // sky_ls at y * skyW + x
        ls.position = eq_area_sphere_dir((x + 0.5f) / float(k.skyW), (y + 0.5f) / float(k.skyH));
        ls.radiance = V3(e.x, e.y, e.z);
        ls.type = LtSky;
    } else if (li == kSunLight) {
        const int x = clampi(int(ux * k.sunW), 0, k.sunW - 1), y = clampi(int(uy * k.sunH), 0, k.sunH - 1);
        ls.solidAnglePdf = (k.sunW * k.sunH) / (kTwoPi * (1.0f - k.sunCosMax));  // sun_ls at y * sunW + x
        ls.position = eq_area_cone_dir(k.sunDir, (x + 0.5f) / float(k.sunW), (y + 0.5f) / float(k.sunH), k.sunCosMax);
        ls.radiance = V3(e.x, e.y, e.z);
        ls.type = LtSun;
    } else if (hasLocal && li < (uint32_t)a.numLights) {
        ls = tri_sample(tri_light(a.lights[li]), V2(ux, uy), pos);
        return true;
    }
    return li < kInvalidLight;
}

VX_D int reflect_view(int p, int n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - p - 1;
    return p;
}

// GetPrevSurface (Restir.h): the previous pass's G-buffer at (x, y).  j = the previous pass's
// camera jitter of the shading pixel (bn_rand(px, py, iterationIndex - 1, 0 / 1): the same for
// every tap); vd = the tap's view direction, computed when vdIn is null and returned in vdOut.
// the surface of a tap record (nr, b) seen along vd
VX_D void rec_surface(const TraceArgs &a, float4 nr, float4 b, V3 vd, SurfS &sf) {
    sf.depth = b.w;
    sf.pos = a.prevCam.pos + vd * sf.depth;
    sf.wo = -vd;
    sf.normal = V3(nr.x, nr.y, nr.z);
    sf.geoNormal = sf.normal;
    sf.albedo = V3(b.x, b.y, b.z);
    const int rb = float_as_bits(nr.w);
    sf.roughness = bits_as_float(rb & 0x7FFFFFFF);
    sf.metallic = rb < 0;
    sf.translucency = 0.0f;  // not read by the taps' target pdf (disney_eval)
}

VX_D V3 sky_emission(const SkyDev &k, V3 dir) {  // miss.cu:53-77
    V3 emission(0.0f);
    V2 uv = eq_area_sphere_uv(dir);
    {
        const V2 UV(uv.x * (float)k.skyW, uv.y * (float)k.skyH);
        const float fx0 = floorf(UV.x - 0.5f), fy0 = floorf(UV.y - 0.5f);
        const V2 fr = UV - V2(fx0 + 0.5f, fy0 + 0.5f);
        const V2 f2 = fr * fr, f3 = f2 * fr;
        const V2 w1 = -2.0f * f3 + 3.0f * f2;
        const V2 w0 = 1.0f - w1;
        const int tx0 = (int)fx0, ty0 = (int)fy0;
        const float wt[4] = {w0.x * w0.y, w1.x * w0.y, w0.x * w1.y, w1.x * w1.y};
        V3 out(0.0f);
        float sum = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int x = tx0 + (i & 1), y = ty0 + (i >> 1);
            if (x >= k.skyW) x %= k.skyW;
            if (x < 0) x = k.skyW - (-x) % k.skyW;
            y = clampi(y, 0, k.skyH - 1);
            sum += wt[i];
            out += ld3(k.sky, (size_t)y * k.skyW + x) * wt[i];
        }
        out /= sum;
        emission += out;
    }
    if (eq_area_cone_uv(uv, k.sunDir, dir, k.sunCosMax)) {
        int x = (int)(uv.x * k.sunW), y = (int)(uv.y * k.sunH);
        if (x >= k.sunW) x %= k.sunW;
        if (x < 0) x = k.sunW - (-x) % k.sunW;
        emission += ld3(k.sun, (size_t)clampi(y, 0, k.sunH - 1) * k.sunW + clampi(x, 0, k.sunW - 1));
    }
    return emission;
}

// ---------------------------------------------------------------- textures
// tex2DLod on an RGBA8 mip chain (TextureManager.cu:228-246: wrap addressing, linear filter,
// linear mip filter, normalized coordinates, unorm reads, lod clamped to [0, maxLod]).  The
// hardware's 8-bit fixed-point filter weights are float weights here (the oracle does the same).
VX_D float4 texel_f(const uchar4 *t, unsigned off, int S, int x, int y) {
    const uchar4 v = t[off + (unsigned)(y * S + x)];
    return make_float4(v.x / 255.0f, v.y / 255.0f, v.z / 255.0f, v.w / 255.0f);
}
VX_D int wrap_i(int i, int S) {
    const int m = i % S;
    return m < 0 ? m + S : m;
}
VX_D V4 tex_bilinear(const uchar4 *t, const TexInfo &ti, int l, float u, float v) {
    const int S = ti.size >> l;
    const float x = u * (float)S - 0.5f, y = v * (float)S - 0.5f;
    const float fx = floorf(x), fy = floorf(y);
    const float ax = x - fx, ay = y - fy;
    const int x0 = wrap_i((int)fx, S), x1 = wrap_i((int)fx + 1, S);
    const int y0 = wrap_i((int)fy, S), y1 = wrap_i((int)fy + 1, S);
    const unsigned o = ti.off[l];
    const float4 a = texel_f(t, o, S, x0, y0), b = texel_f(t, o, S, x1, y0);
    const float4 c = texel_f(t, o, S, x0, y1), d = texel_f(t, o, S, x1, y1);
    const float w00 = (1.0f - ax) * (1.0f - ay), w10 = ax * (1.0f - ay), w01 = (1.0f - ax) * ay, w11 = ax * ay;
    return V4(a.x * w00 + b.x * w10 + c.x * w01 + d.x * w11, a.y * w00 + b.y * w10 + c.y * w01 + d.y * w11,
              a.z * w00 + b.z * w10 + c.z * w01 + d.z * w11, a.w * w00 + b.w * w10 + c.w * w01 + d.w * w11);
}
VX_D V4 tex_lod(const uchar4 *t, const TexInfo &ti, float u, float v, float lod) {
    lod = fminf(fmaxf(lod, 0.0f), (float)ti.maxLod);
    const int l0 = (int)floorf(lod);
    const float fl = lod - (float)l0;
    const V4 c0 = tex_bilinear(t, ti, l0, u, v);
    if (!(fl > 0.0f)) return c0;
    const V4 c1 = tex_bilinear(t, ti, min(l0 + 1, ti.maxLod), u, v);
    return c0 * (1.0f - fl) + c1 * fl;
}

// Camera::getRayConeWidth (Camera.h:133-149): the angle one pixel subtends
VX_D float ray_cone_spread(const CamDev &cam, int px, int py) {
    const V2 pc = (V2((float)px, (float)py) + 0.5f) - cam.res / 2.0f;
    const V2 po(copysignf(0.5f, pc.x), copysignf(0.5f, pc.y));
    const V2 uvN = (pc - po) * cam.invRes * 2.0f, uvF = (pc + po) * cam.invRes * 2.0f;
    const V2 pN = uvN * cam.tanHalfFov, pF = uvF * cam.tanHalfFov;
    return atanf(sqrtf(pF.x * pF.x + pF.y * pF.y)) - atanf(sqrtf(pN.x * pN.x + pN.y * pN.y));
}

// Textured MaterialState (closesthit.cu:167-254): world-grid uv of the front position, ray-cone
// lod, albedo x texture, roughness / metallic from textures, tangent-space normal map aligned to
// the face and blended at strength 0.2.  coneWidth = the ray cone's width at this hit.
// vertexTc: the mesh triangle's interpolated texcoords (closesthit.cu:189; useVertexTc = a mesh hit)
VX_D void apply_textures(const uchar4 *texels, const TexInfo *tex, const MatDev &m, V3 pos, V3 ng, V3 wo,
                         float coneWidth, V3 &albedo, float &roughness, bool &metallic, V3 &normal,
                         bool useVertexTc = false, V2 vertexTc = V2(0.0f, 0.0f)) {
    V2 tc(0.0f, 0.0f);
    if (m.worldGridUV) {
        if (fabsf(ng.x) > 0.9f) tc = V2(fmodf(pos.z, m.uvScale), fmodf(pos.y, m.uvScale));
        else if (fabsf(ng.y) > 0.9f) tc = V2(fmodf(pos.x, m.uvScale), fmodf(pos.z, m.uvScale));
        else if (fabsf(ng.z) > 0.9f) tc = V2(fmodf(pos.x, m.uvScale), fmodf(pos.y, m.uvScale));
    } else if (useVertexTc) {
        tc = vertexTc;
    }
    tc = tc / m.uvScale;
    const float mip0 = sqrtf(1024.0f * 1024.0f + 1024.0f * 1024.0f);  // MaterialParameter::texSize (1024, 1024)
    const float lod = log2f(coneWidth / fmaxf(dot(ng, wo), 0.2f) / m.uvScale * 2.0f * mip0) - 3.0f;
    if (m.tex[0] >= 0) {
        const V4 c = tex_lod(texels, tex[m.tex[0]], tc.x, tc.y, lod);
        albedo = albedo * V3(c.x, c.y, c.z);
    }
    albedo = max3(albedo, V3(0.001f));
    if (m.tex[2] >= 0) roughness = tex_lod(texels, tex[m.tex[2]], tc.x, tc.y, lod).x;
    if (m.tex[3] >= 0) metallic = tex_lod(texels, tex[m.tex[3]], tc.x, tc.y, lod).x > 0.5f;
    if (m.tex[1] >= 0) {
        const V4 c = tex_lod(texels, tex[m.tex[1]], tc.x, tc.y, lod);
        V3 n = normalize(V3(c.x - 0.5f, c.y - 0.5f, c.z - 0.5f));
        n.x = -n.x;
        n.y = -n.y;
        align_vector(ng, n);
        normal = n;
    } else {
        normal = ng;
    }
    normal = lerp3(ng, normal, 0.2f);
}

}  // namespace
}  // namespace vx
