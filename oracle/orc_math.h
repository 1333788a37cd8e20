// ORACLE (test infrastructure only) -- CPU restatement of the reference's
// vector/matrix semantics, renderer/shaders/LinearMath.h.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// link this code, and only as the checker.  Nothing in the product links it.
//
// Every operator below reproduces the reference's arithmetic *including its
// quirks* (SURVEY.md §8a-Z(1)):
//   * Float4 binary operators compute w from z (LinearMath.h:866-874)
//   * Float4 -=, *=, /= by a scalar do `w += a` (LinearMath.h:917-940)
//   * dot(Float3) / length / Mat3*Float3 use the compensated InnerProduct
//     (LinearMath.h:114-138, 1017, 1103-1108)
//   * cross() uses the difference-of-products form (LinearMath.h:87-93, 980)
//   * normalize(Float3) returns (0,0,1) for |v|<1e-8 or NaN (LinearMath.h:962-973)
// Build with -ffp-contract=off: the reference's explicit FMA() calls are the
// only fused operations.
#pragma once
#include <cmath>
#include <cstdint>
#include <cfloat>

namespace orc {

static constexpr float kPi = 3.1415926535897932384626422832795028841971f;  // LinearMath.h:17
static constexpr float kTwoPi = 6.2831853071795864769252867665590057683943f;
static constexpr float kPiOver2 = 1.5707963267948966192313216916397514420985f;
static constexpr float kPiOver4 = 0.7853981633974483096156608458198757210492f;
static constexpr float kPiOver180 = 0.01745329251f;
static constexpr float kInvTwoPi = 0.15915494309f;
static constexpr float kSafeCos = 1e-5f;        // SAFE_COSINE_EPSI
static constexpr float kRayMax = 1.0e27f;       // Common.h:27

inline float fmaf_(float a, float b, float c) { return std::fmaf(a, b, c); }

// --- compensated arithmetic (LinearMath.h:87-146) ---
inline float dop(float a, float b, float c, float d) {
    float cd = c * d;
    float err = fmaf_(-c, d, cd);
    float r = fmaf_(a, b, -cd);
    return r + err;
}
struct CF { float v, err; };
inline CF two_prod(float a, float b) { float ab = a * b; return {ab, fmaf_(a, b, -ab)}; }
inline CF two_sum(float a, float b) {
    float s = a + b, delta = s - a;
    return {s, (a - (s - delta)) + (b - delta)};
}
// InnerProduct(a,b,c,d,e,f) expanded exactly as the variadic recursion does
inline float inner3(float a, float b, float c, float d, float e, float f) {
    CF ef = two_prod(e, f);
    CF cd = two_prod(c, d);
    CF s1 = two_sum(cd.v, ef.v);
    CF tp = {s1.v, cd.err + (ef.err + s1.err)};
    CF ab = two_prod(a, b);
    CF s2 = two_sum(ab.v, tp.v);
    CF r = {s2.v, ab.err + (tp.err + s2.err)};
    return r.v + r.err;
}

struct F2 {
    float x = 0, y = 0;
    F2() = default;
    F2(float a, float b) : x(a), y(b) {}
    explicit F2(float a) : x(a), y(a) {}
    F2 operator+(const F2 &o) const { return {x + o.x, y + o.y}; }
    F2 operator-(const F2 &o) const { return {x - o.x, y - o.y}; }
    F2 operator*(const F2 &o) const { return {x * o.x, y * o.y}; }
    F2 operator/(const F2 &o) const { return {x / o.x, y / o.y}; }
    F2 operator+(float a) const { return {x + a, y + a}; }
    F2 operator-(float a) const { return {x - a, y - a}; }
    F2 operator*(float a) const { return {x * a, y * a}; }
    F2 operator/(float a) const { return {x / a, y / a}; }
    float length() const { return std::sqrt(x * x + y * y); }
};
inline F2 operator*(float a, const F2 &v) { return {v.x * a, v.y * a}; }
inline F2 operator-(float a, const F2 &v) { return {a - v.x, a - v.y}; }
inline F2 operator/(float a, const F2 &v) { return {a / v.x, a / v.y}; }

struct F3 {
    float x = 0, y = 0, z = 0;
    F3() = default;
    F3(float a, float b, float c) : x(a), y(b), z(c) {}
    explicit F3(float a) : x(a), y(a), z(a) {}
    float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    F3 operator+(const F3 &o) const { return {x + o.x, y + o.y, z + o.z}; }
    F3 operator-(const F3 &o) const { return {x - o.x, y - o.y, z - o.z}; }
    F3 operator*(const F3 &o) const { return {x * o.x, y * o.y, z * o.z}; }
    F3 operator/(const F3 &o) const { return {x / o.x, y / o.y, z / o.z}; }
    F3 operator+(float a) const { return {x + a, y + a, z + a}; }
    F3 operator-(float a) const { return {x - a, y - a, z - a}; }
    F3 operator*(float a) const { return {x * a, y * a, z * a}; }
    F3 operator/(float a) const { return {x / a, y / a, z / a}; }
    F3 &operator+=(const F3 &o) { x += o.x; y += o.y; z += o.z; return *this; }
    F3 &operator-=(const F3 &o) { x -= o.x; y -= o.y; z -= o.z; return *this; }
    F3 &operator*=(const F3 &o) { x *= o.x; y *= o.y; z *= o.z; return *this; }
    F3 &operator/=(const F3 &o) { x /= o.x; y /= o.y; z /= o.z; return *this; }
    F3 &operator*=(float a) { x *= a; y *= a; z *= a; return *this; }
    F3 &operator/=(float a) { x /= a; y /= a; z /= a; return *this; }
    F3 operator-() const { return {-x, -y, -z}; }
    float length2() const { return inner3(x, x, y, y, z, z); }
    float length() const { return std::sqrt(length2()); }
    F3 normalized() const { float n = length(); return {x / n, y / n, z / n}; }
};
inline F3 operator*(float a, const F3 &v) { return {v.x * a, v.y * a, v.z * a}; }
inline F3 operator-(float a, const F3 &v) { return {a - v.x, a - v.y, a - v.z}; }
inline F3 operator+(float a, const F3 &v) { return {v.x + a, v.y + a, v.z + a}; }
inline F3 operator/(float a, const F3 &v) { return {a / v.x, a / v.y, a / v.z}; }

// Float4 with the reference's operator semantics (LinearMath.h:834-954)
struct F4 {
    float x = 0, y = 0, z = 0, w = 0;
    F4() = default;
    F4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
    explicit F4(float a) : x(a), y(a), z(a), w(a) {}
    F4(const F3 &v, float a) : x(v.x), y(v.y), z(v.z), w(a) {}
    F3 xyz() const { return {x, y, z}; }
    void set_xyz(const F3 &v) { x = v.x; y = v.y; z = v.z; }
    float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : (i == 2 ? z : w)); }
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : (i == 2 ? z : w)); }
    // quirk: w computed from z
    F4 operator+(const F4 &v) const { return {x + v.x, y + v.y, z + v.z, z + v.z}; }
    F4 operator-(const F4 &v) const { return {x - v.x, y - v.y, z - v.z, z - v.z}; }
    F4 operator*(const F4 &v) const { return {x * v.x, y * v.y, z * v.z, z * v.z}; }
    F4 operator/(const F4 &v) const { return {x / v.x, y / v.y, z / v.z, z / v.z}; }
    F4 operator+(float a) const { return {x + a, y + a, z + a, z + a}; }
    F4 operator-(float a) const { return {x - a, y - a, z - a, z - a}; }
    F4 operator*(float a) const { return {x * a, y * a, z * a, z * a}; }
    F4 operator/(float a) const { return {x / a, y / a, z / a, z / a}; }
    F4 &operator+=(const F4 &v) { x += v.x; y += v.y; z += v.z; w += v.w; return *this; }
    F4 &operator-=(const F4 &v) { x -= v.x; y -= v.y; z -= v.z; w -= v.w; return *this; }
    F4 &operator*=(const F4 &v) { x *= v.x; y *= v.y; z *= v.z; w *= v.w; return *this; }
    F4 &operator/=(const F4 &v) { x /= v.x; y /= v.y; z /= v.z; w /= v.w; return *this; }
    F4 &operator+=(float a) { x += a; y += a; z += a; w += a; return *this; }
    // quirk: w += a
    F4 &operator-=(float a) { x -= a; y -= a; z -= a; w += a; return *this; }
    F4 &operator*=(float a) { x *= a; y *= a; z *= a; w += a; return *this; }
    F4 &operator/=(float a) { x /= a; y /= a; z /= a; w += a; return *this; }
};
inline F4 operator*(float a, const F4 &v) { return {v.x * a, v.y * a, v.z * a, v.w * a}; }
inline F4 operator+(float a, const F4 &v) { return {v.x + a, v.y + a, v.z + a, v.w + a}; }
inline F4 operator-(float a, const F4 &v) { return {a - v.x, a - v.y, a - v.z, a - v.w}; }

inline float dot(const F3 &a, const F3 &b) { return inner3(a.x, b.x, a.y, b.y, a.z, b.z); }
inline float dot(const F4 &a, const F4 &b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
inline float length(const F3 &v) { return std::sqrt(dot(v, v)); }
inline F3 cross(const F3 &a, const F3 &b) {
    return {dop(a.y, b.z, a.z, b.y), dop(a.z, b.x, a.x, b.z), dop(a.x, b.y, a.y, b.x)};
}
inline F3 normalize(const F3 &v) {
    float n = std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
    if (n < 1e-8f || std::isnan(n)) return {0.f, 0.f, 1.f};
    return {v.x / n, v.y / n, v.z / n};
}
inline F2 normalize(const F2 &v) { float n = std::sqrt(v.x * v.x + v.y * v.y); return {v.x / n, v.y / n}; }
// Device code resolves max/min(float,float) to CUDA's fmaxf/fminf (non-template
// exact match beats LinearMath.h:69's template); ints use the template.
inline float mymax(float a, float b) { return std::fmax(a, b); }
inline float mymin(float a, float b) { return std::fmin(a, b); }
inline int mymax(int a, int b) { return a > b ? a : b; }
inline int mymin(int a, int b) { return a < b ? a : b; }
inline F3 max3f(const F3 &a, const F3 &b) { return {mymax(a.x, b.x), mymax(a.y, b.y), mymax(a.z, b.z)}; }
inline F3 min3f(const F3 &a, const F3 &b) { return {mymin(a.x, b.x), mymin(a.y, b.y), mymin(a.z, b.z)}; }
inline F4 max4f(const F4 &a, const F4 &b) { return {mymax(a.x, b.x), mymax(a.y, b.y), mymax(a.z, b.z), mymax(a.w, b.w)}; }
inline float clampf(float a, float lo = 0.f, float hi = 1.f) { return a < lo ? lo : (a > hi ? hi : a); }
inline int clampi(int a, int lo, int hi) { return a < lo ? lo : (a > hi ? hi : a); }
inline F3 clamp3f(const F3 &a, const F3 &lo, const F3 &hi) {
    return {clampf(a.x, lo.x, hi.x), clampf(a.y, lo.y, hi.y), clampf(a.z, lo.z, hi.z)};
}
inline float saturate(float x) { return std::fmin(std::fmax(x, 0.0f), 1.0f); }
inline float lerpf(float a, float b, float w) { return a + w * (b - a); }
inline F3 lerp3(const F3 &a, const F3 &b, float w) { return a + w * (b - a); }
inline F4 lerp4(const F4 &a, const F4 &b, float w) { return a + w * (b - a); }  // quirky w
inline F3 reflect3f(const F3 &i, const F3 &n) { return i - 2.0f * n * dot(n, i); }
inline float pow5(float e) { float e2 = e * e; return e2 * e2 * e; }
inline F3 abs3(const F3 &v) { return {std::fabs(v.x), std::fabs(v.y), std::fabs(v.z)}; }
inline F3 sqrt3f(const F3 &v) { return {std::sqrt(v.x), std::sqrt(v.y), std::sqrt(v.z)}; }
inline F3 smoothstep3f(const F3 &a, const F3 &b, float w) { return a + (w * w * (3.0f - 2.0f * w)) * (b - a); }
inline float luminance(const F3 &c) { return dot(c, F3(0.2126f, 0.7152f, 0.0722f)); }
inline bool is_null(const F3 &v) { return v.x == 0.0f && v.y == 0.0f && v.z == 0.0f; }

// Mat3, column-major storage; 9-float ctor takes row-major arguments
// (LinearMath.h:1040-1108)
struct M3 {
    float m00 = 0, m10 = 0, m20 = 0, m01 = 0, m11 = 0, m21 = 0, m02 = 0, m12 = 0, m22 = 0;
    M3() = default;
    M3(const F3 &c0, const F3 &c1, const F3 &c2)
        : m00(c0.x), m10(c0.y), m20(c0.z), m01(c1.x), m11(c1.y), m21(c1.z), m02(c2.x), m12(c2.y), m22(c2.z) {}
    M3(float a00, float a01, float a02, float a10, float a11, float a12, float a20, float a21, float a22)
        : m00(a00), m10(a10), m20(a20), m01(a01), m11(a11), m21(a21), m02(a02), m12(a12), m22(a22) {}
    void transpose() { std::swap(m01, m10); std::swap(m20, m02); std::swap(m21, m12); }
};
inline M3 operator*(const M3 &A, const M3 &B) {
    return M3(A.m00 * B.m00 + A.m01 * B.m10 + A.m02 * B.m20, A.m00 * B.m01 + A.m01 * B.m11 + A.m02 * B.m21,
              A.m00 * B.m02 + A.m01 * B.m12 + A.m02 * B.m22, A.m10 * B.m00 + A.m11 * B.m10 + A.m12 * B.m20,
              A.m10 * B.m01 + A.m11 * B.m11 + A.m12 * B.m21, A.m10 * B.m02 + A.m11 * B.m12 + A.m12 * B.m22,
              A.m20 * B.m00 + A.m21 * B.m10 + A.m22 * B.m20, A.m20 * B.m01 + A.m21 * B.m11 + A.m22 * B.m21,
              A.m20 * B.m02 + A.m21 * B.m12 + A.m22 * B.m22);
}
inline F3 operator*(const M3 &m, const F3 &v) {
    return {inner3(m.m00, v.x, m.m01, v.y, m.m02, v.z), inner3(m.m10, v.x, m.m11, v.y, m.m12, v.z),
            inner3(m.m20, v.x, m.m21, v.y, m.m22, v.z)};
}

// Quaternion (LinearMath.h:1311-1366)
struct Q {
    F3 v; float w = 0;
    Q() = default;
    Q(const F3 &a, float b) : v(a), w(b) {}
    Q conj() const { return {-v, w}; }
    float norm2() const { return v.x * v.x + v.y * v.y + v.z * v.z + w * w; }
    Q normalized() const { float n = std::sqrt(norm2()); return {v / n, w / n}; }
    Q operator*(const Q &q) const { return {w * q.v + q.w * v + cross(v, q.v), w * q.w - dot(v, q.v)}; }
};
inline Q rotate(const Q &q, const Q &v) { return q * v * q.conj(); }
inline Q rotation_between(const Q &p, const Q &q) {
    return Q(cross(p.v, q.v), std::sqrt(p.v.length2() * q.v.length2()) + dot(p.v, q.v)).normalized();
}
inline Q axis_angle(const F3 &axis, float angle) {
    return Q(axis.normalized() * std::sin(angle / 2), std::cos(angle / 2));
}
inline F3 rotate3f(const F3 &axis, float angle, const F3 &v) { return rotate(axis_angle(axis, angle), Q(v, 0.f)).v; }

// alignVector (LinearMath.h:1806-1814)
inline void align_vector(const F3 &axis, F3 &w) {
    const float s = std::copysign(1.0f, axis.z);
    w.z *= s;
    const F3 h(axis.x, axis.y, axis.z + s);
    const float k = dot(w, h) / (1.0f + std::fabs(axis.z));
    w = k * h - w;
}

// LocalizeSample / equal-area maps (LinearMath.h:1449-1461, 1857-1913)
inline void localize_sample(const F3 &n, F3 &u, F3 &v) {
    F3 w(1, 0, 0);
    if (std::fabs(n.x) > 0.707f) w = F3(0, 1, 0);
    u = cross(n, w);
    v = cross(n, u);
}
inline F3 equal_area_sphere_dir(float u, float v) {
    float y = 2.0f * v - 1.0f;
    float r = std::sqrt(1.0f - y * y);
    float phi = kTwoPi * u;
    return {r * std::cos(phi), y, r * std::sin(phi)};
}
inline F2 equal_area_sphere_uv(const F3 &d) {
    float u = std::atan2(-d.z, -d.x) / kTwoPi + 0.5f;
    float v = (d.y + 1.0f) * 0.5f;
    return {u, v};
}
inline F3 equal_area_hemisphere_dir(float u, float v) {
    float z = v;
    float r = std::sqrt(1.0f - v * v);
    float phi = kTwoPi * u;
    return {r * std::cos(phi), z, r * std::sin(phi)};
}
inline F3 equal_area_cone_dir(const F3 &sunDir, float u, float v, float cosThetaMax) {
    float cosTheta = (1.0f - u) + u * cosThetaMax;
    float sinTheta = std::sqrt(1.0f - cosTheta * cosTheta);
    float phi = v * kTwoPi;
    F3 t, b;
    localize_sample(sunDir, t, b);
    M3 trans(t, sunDir, b);
    F3 coords(std::cos(phi) * sinTheta, cosTheta, std::sin(phi) * sinTheta);
    return trans * coords;
}
inline bool equal_area_cone_uv(F2 &uv, const F3 &sunDir, const F3 &rayDir, float cosThetaMax) {
    F3 t, b;
    localize_sample(sunDir, t, b);
    M3 trans(t, sunDir, b);
    trans.transpose();
    F3 c = trans * rayDir;
    float cosTheta = c.y;
    if (cosTheta < cosThetaMax) return false;
    float u = (1.0f - cosTheta) / (1.0f - cosThetaMax);
    float sinTheta = std::sqrt(1.0f - cosTheta * cosTheta);
    if (sinTheta < 1e-5f || (c.x / sinTheta) < -1.0f || (c.x / sinTheta) > 1.0f) return false;
    float v = std::acos(c.x / sinTheta) * kInvTwoPi;
    uv = F2(u, v);
    return true;
}
inline F2 concentric_disk(F2 u) {
    // LinearMath.h:1658-1685; note `2.0 * u - 1.0` is double*Float2 -> float ops
    F2 o = F2(u.x * 2.0f - 1.0f, u.y * 2.0f - 1.0f);
    if (std::fabs(o.x) < 1e-10f && std::fabs(o.y) < 1e-10f) return F2(0, 0);
    float theta, r;
    if (std::fabs(o.x) > std::fabs(o.y)) {
        r = o.x;
        theta = kPiOver4 * (o.y / o.x);
    } else {
        r = o.y;
        theta = kPiOver2 - kPiOver4 * (o.x / o.y);
    }
    return F2(std::cos(theta) * r, std::sin(theta) * r);
}

// Directed-rounding helpers for the self-intersection offset (SelfHit.h:124-190).
// Emulated through binary64, which is exact for the operand ranges used here
// (integer-valued voxel coordinates <= 2^16, error terms ~2^-23).
inline float round_up_f(double d) {
    float r = (float)d;
    if ((double)r < d) r = std::nextafter(r, INFINITY);
    return r;
}
inline float round_dn_f(double d) {
    float r = (float)d;
    if ((double)r > d) r = std::nextafter(r, -INFINITY);
    return r;
}
inline float fma_ru(float a, float b, float c) { return round_up_f((double)a * (double)b + (double)c); }
inline float fma_rd(float a, float b, float c) { return round_dn_f((double)a * (double)b + (double)c); }
inline float mul_ru(float a, float b) { return round_up_f((double)a * (double)b); }
inline float add_ru(float a, float b) { return round_up_f((double)a + (double)b); }

}  // namespace orc
