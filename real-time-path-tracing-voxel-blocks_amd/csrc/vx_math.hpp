// vxpt -- vector math shared by the host set-up code and the gfx950 kernels.
//
// Arithmetic follows renderer/shaders/LinearMath.h operation for operation so
// that results are reproducible, including the reference's Float4 operator
// behaviour (binary ops take w from z, LinearMath.h:866-874; `-=,*=,/=` by a
// scalar add to w, :917-940) which the denoiser's second-moment channel
// depends on.  The translation units are built with -ffp-contract=off; every
// fused multiply-add below is spelled out with fmaf where the reference
// spells FMA().
#pragma once
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>

#define VX_HD __host__ __device__ __forceinline__
#define VX_D __device__ __forceinline__

namespace vx {

constexpr float kPi = 3.1415926535897932384626422832795028841971f;
constexpr float kTwoPi = 6.2831853071795864769252867665590057683943f;
constexpr float kPiOver2 = 1.5707963267948966192313216916397514420985f;
constexpr float kPiOver4 = 0.7853981633974483096156608458198757210492f;
constexpr float kPiOver180 = 0.01745329251f;
constexpr float kInvTwoPi = 0.15915494309f;
constexpr float kSafeCos = 1e-5f;
constexpr float kRayMax = 1.0e27f;

VX_HD float fmx(float a, float b) { return fmaxf(a, b); }
VX_HD float fmn(float a, float b) { return fminf(a, b); }
VX_HD float clampf(float a, float lo = 0.f, float hi = 1.f) { return a < lo ? lo : (a > hi ? hi : a); }
VX_HD int clampi(int a, int lo, int hi) { return a < lo ? lo : (a > hi ? hi : a); }
VX_HD float saturate(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }
VX_HD float lerpf(float a, float b, float w) { return a + w * (b - a); }
VX_HD float pow5(float e) { float e2 = e * e; return e2 * e2 * e; }

// difference of products / compensated inner product (LinearMath.h:87-146)
VX_HD float dop(float a, float b, float c, float d) {
    float cd = c * d;
    float err = fmaf(-c, d, cd);
    return fmaf(a, b, -cd) + err;
}
VX_HD float inner3(float a, float b, float c, float d, float e, float f) {
    float ef = e * f, efE = fmaf(e, f, -ef);
    float cd = c * d, cdE = fmaf(c, d, -cd);
    float s1 = cd + ef, d1 = s1 - cd, s1E = (cd - (s1 - d1)) + (ef - d1);
    float tpE = cdE + (efE + s1E);
    float ab = a * b, abE = fmaf(a, b, -ab);
    float s2 = ab + s1, d2 = s2 - ab, s2E = (ab - (s2 - d2)) + (s1 - d2);
    return s2 + (abE + (tpE + s2E));
}

struct V2 {
    float x, y;
    VX_HD V2() : x(0), y(0) {}
    VX_HD V2(float a, float b) : x(a), y(b) {}
    VX_HD explicit V2(float a) : x(a), y(a) {}
    VX_HD V2 operator+(V2 o) const { return {x + o.x, y + o.y}; }
    VX_HD V2 operator-(V2 o) const { return {x - o.x, y - o.y}; }
    VX_HD V2 operator*(V2 o) const { return {x * o.x, y * o.y}; }
    VX_HD V2 operator+(float a) const { return {x + a, y + a}; }
    VX_HD V2 operator-(float a) const { return {x - a, y - a}; }
    VX_HD V2 operator*(float a) const { return {x * a, y * a}; }
    VX_HD V2 operator/(float a) const { return {x / a, y / a}; }
};
VX_HD V2 operator*(float a, V2 v) { return {v.x * a, v.y * a}; }
VX_HD V2 operator-(float a, V2 v) { return {a - v.x, a - v.y}; }

struct V3 {
    float x, y, z;
    VX_HD V3() : x(0), y(0), z(0) {}
    VX_HD V3(float a, float b, float c) : x(a), y(b), z(c) {}
    VX_HD explicit V3(float a) : x(a), y(a), z(a) {}
    VX_HD float get(int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    VX_HD void set(int i, float v) { if (i == 0) x = v; else if (i == 1) y = v; else z = v; }
    VX_HD V3 operator+(V3 o) const { return {x + o.x, y + o.y, z + o.z}; }
    VX_HD V3 operator-(V3 o) const { return {x - o.x, y - o.y, z - o.z}; }
    VX_HD V3 operator*(V3 o) const { return {x * o.x, y * o.y, z * o.z}; }
    VX_HD V3 operator/(V3 o) const { return {x / o.x, y / o.y, z / o.z}; }
    VX_HD V3 operator*(float a) const { return {x * a, y * a, z * a}; }
    VX_HD V3 operator/(float a) const { return {x / a, y / a, z / a}; }
    VX_HD V3 &operator+=(V3 o) { x += o.x; y += o.y; z += o.z; return *this; }
    VX_HD V3 &operator*=(V3 o) { x *= o.x; y *= o.y; z *= o.z; return *this; }
    VX_HD V3 &operator*=(float a) { x *= a; y *= a; z *= a; return *this; }
    VX_HD V3 &operator/=(float a) { x /= a; y /= a; z /= a; return *this; }
    VX_HD V3 operator-() const { return {-x, -y, -z}; }
};
VX_HD V3 operator*(float a, V3 v) { return {v.x * a, v.y * a, v.z * a}; }
VX_HD V3 operator-(float a, V3 v) { return {a - v.x, a - v.y, a - v.z}; }

// Float4 with the reference's operator semantics
struct alignas(16) V4 {
    float x, y, z, w;
    VX_HD V4() : x(0), y(0), z(0), w(0) {}
    VX_HD V4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
    VX_HD explicit V4(float a) : x(a), y(a), z(a), w(a) {}
    VX_HD V4(V3 v, float a) : x(v.x), y(v.y), z(v.z), w(a) {}
    VX_HD V3 xyz() const { return {x, y, z}; }
    VX_HD void set_xyz(V3 v) { x = v.x; y = v.y; z = v.z; }
    VX_HD float get(int i) const { return i == 0 ? x : (i == 1 ? y : (i == 2 ? z : w)); }
    VX_HD V4 operator+(V4 v) const { return {x + v.x, y + v.y, z + v.z, z + v.z}; }
    VX_HD V4 operator-(V4 v) const { return {x - v.x, y - v.y, z - v.z, z - v.z}; }
    VX_HD V4 operator*(V4 v) const { return {x * v.x, y * v.y, z * v.z, z * v.z}; }
    VX_HD V4 operator/(V4 v) const { return {x / v.x, y / v.y, z / v.z, z / v.z}; }
    VX_HD V4 operator*(float a) const { return {x * a, y * a, z * a, z * a}; }
    VX_HD V4 operator/(float a) const { return {x / a, y / a, z / a, z / a}; }
    VX_HD V4 &operator+=(V4 v) { x += v.x; y += v.y; z += v.z; w += v.w; return *this; }
    VX_HD V4 &operator*=(V4 v) { x *= v.x; y *= v.y; z *= v.z; w *= v.w; return *this; }
    VX_HD V4 &operator-=(float a) { x -= a; y -= a; z -= a; w += a; return *this; }
    VX_HD V4 &operator/=(float a) { x /= a; y /= a; z /= a; w += a; return *this; }
};
VX_HD V4 operator*(float a, V4 v) { return {v.x * a, v.y * a, v.z * a, v.w * a}; }

VX_HD float dot(V3 a, V3 b) { return inner3(a.x, b.x, a.y, b.y, a.z, b.z); }
VX_HD float length(V3 v) { return sqrtf(dot(v, v)); }
VX_HD V3 cross(V3 a, V3 b) { return {dop(a.y, b.z, a.z, b.y), dop(a.z, b.x, a.x, b.z), dop(a.x, b.y, a.y, b.x)}; }
VX_HD V3 normalize(V3 v) {
    float n = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z);
    if (n < 1e-8f || n != n) return {0.f, 0.f, 1.f};
    return {v.x / n, v.y / n, v.z / n};
}
VX_HD V3 normalized_c(V3 v) {  // Float3::normalized(): compensated length, no guard
    float n = sqrtf(inner3(v.x, v.x, v.y, v.y, v.z, v.z));
    return {v.x / n, v.y / n, v.z / n};
}
VX_HD V3 max3(V3 a, V3 b) { return {fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)}; }
VX_HD V3 lerp3(V3 a, V3 b, float w) { return a + w * (b - a); }
VX_HD V4 lerp4(V4 a, V4 b, float w) { return a + w * (b - a); }
VX_HD V3 reflect3(V3 i, V3 n) { return i - 2.0f * n * dot(n, i); }
VX_HD V3 abs3(V3 v) { return {fabsf(v.x), fabsf(v.y), fabsf(v.z)}; }
VX_HD float luminance(V3 c) { return dot(c, V3(0.2126f, 0.7152f, 0.0722f)); }
// Plain FMA inner product for smooth per-tap weights in the denoiser's inner
// loops (normal-angle and luminance weights): within ~2 ulp of the compensated
// dot above (LinearMath.h:1017) at a tenth of its ~30 instructions.  Threshold
// tests (plane distance) keep the compensated form.
VX_HD float dot_fast(V3 a, V3 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, a.z * b.z)); }
VX_HD float luminance_fast(V3 c) { return dot_fast(c, V3(0.2126f, 0.7152f, 0.0722f)); }
VX_HD bool is_null(V3 v) { return v.x == 0.0f && v.y == 0.0f && v.z == 0.0f; }

// 3x3 matrix, column-major (LinearMath.h:1040-1108)
struct M3 {
    float m00, m10, m20, m01, m11, m21, m02, m12, m22;
};
VX_HD M3 m3_cols(V3 c0, V3 c1, V3 c2) { return {c0.x, c0.y, c0.z, c1.x, c1.y, c1.z, c2.x, c2.y, c2.z}; }
VX_HD M3 m3_rows(float a00, float a01, float a02, float a10, float a11, float a12, float a20, float a21, float a22) {
    return {a00, a10, a20, a01, a11, a21, a02, a12, a22};
}
VX_HD M3 m3_zero() { return {0, 0, 0, 0, 0, 0, 0, 0, 0}; }
VX_HD M3 m3_transpose(M3 m) { return {m.m00, m.m01, m.m02, m.m10, m.m11, m.m12, m.m20, m.m21, m.m22}; }
VX_HD M3 m3_mul(const M3 &A, const M3 &B) {
    return m3_rows(A.m00 * B.m00 + A.m01 * B.m10 + A.m02 * B.m20, A.m00 * B.m01 + A.m01 * B.m11 + A.m02 * B.m21,
                   A.m00 * B.m02 + A.m01 * B.m12 + A.m02 * B.m22, A.m10 * B.m00 + A.m11 * B.m10 + A.m12 * B.m20,
                   A.m10 * B.m01 + A.m11 * B.m11 + A.m12 * B.m21, A.m10 * B.m02 + A.m11 * B.m12 + A.m12 * B.m22,
                   A.m20 * B.m00 + A.m21 * B.m10 + A.m22 * B.m20, A.m20 * B.m01 + A.m21 * B.m11 + A.m22 * B.m21,
                   A.m20 * B.m02 + A.m21 * B.m12 + A.m22 * B.m22);
}
VX_HD V3 m3_apply(const M3 &m, V3 v) {
    return {inner3(m.m00, v.x, m.m01, v.y, m.m02, v.z), inner3(m.m10, v.x, m.m11, v.y, m.m12, v.z),
            inner3(m.m20, v.x, m.m21, v.y, m.m22, v.z)};
}

// quaternion (LinearMath.h:1311-1370)
struct Qt { V3 v; float w; };
VX_HD Qt q_mul(Qt p, Qt q) { return {p.w * q.v + q.w * p.v + cross(p.v, q.v), p.w * q.w - dot(p.v, q.v)}; }
VX_HD Qt q_conj(Qt q) { return {-q.v, q.w}; }
VX_HD Qt q_normalized(Qt q) {
    float n = sqrtf(q.v.x * q.v.x + q.v.y * q.v.y + q.v.z * q.v.z + q.w * q.w);
    return {q.v / n, q.w / n};
}
VX_HD Qt q_rotation_between(V3 p, V3 q) {
    float lp = inner3(p.x, p.x, p.y, p.y, p.z, p.z), lq = inner3(q.x, q.x, q.y, q.y, q.z, q.z);
    return q_normalized({cross(p, q), sqrtf(lp * lq) + dot(p, q)});
}
VX_HD V3 q_rotate(Qt q, V3 v) { return q_mul(q_mul(q, {v, 0.f}), q_conj(q)).v; }

VX_HD void align_vector(V3 axis, V3 &w) {  // LinearMath.h:1806-1814
    const float s = copysignf(1.0f, axis.z);
    w.z *= s;
    const V3 h(axis.x, axis.y, axis.z + s);
    const float k = dot(w, h) / (1.0f + fabsf(axis.z));
    w = k * h - w;
}
VX_HD void localize_sample(V3 n, V3 &u, V3 &v) {
    V3 w(1, 0, 0);
    if (fabsf(n.x) > 0.707f) w = V3(0, 1, 0);
    u = cross(n, w);
    v = cross(n, u);
}
VX_HD V3 eq_area_sphere_dir(float u, float v) {
    float y = 2.0f * v - 1.0f;
    float r = sqrtf(1.0f - y * y);
    float phi = kTwoPi * u;
    return {r * cosf(phi), y, r * sinf(phi)};
}
VX_HD V2 eq_area_sphere_uv(V3 d) { return {atan2f(-d.z, -d.x) / kTwoPi + 0.5f, (d.y + 1.0f) * 0.5f}; }
VX_HD V3 eq_area_cone_dir(V3 sunDir, float u, float v, float cosThetaMax) {
    float ct = (1.0f - u) + u * cosThetaMax;
    float st = sqrtf(1.0f - ct * ct);
    float phi = v * kTwoPi;
    V3 t, b;
    localize_sample(sunDir, t, b);
    return m3_apply(m3_cols(t, sunDir, b), V3(cosf(phi) * st, ct, sinf(phi) * st));
}
VX_HD bool eq_area_cone_uv(V2 &uv, V3 sunDir, V3 rayDir, float cosThetaMax) {
    V3 t, b;
    localize_sample(sunDir, t, b);
    V3 c = m3_apply(m3_transpose(m3_cols(t, sunDir, b)), rayDir);
    float ct = c.y;
    if (ct < cosThetaMax) return false;
    float u = (1.0f - ct) / (1.0f - cosThetaMax);
    float st = sqrtf(1.0f - ct * ct);
    if (st < 1e-5f || (c.x / st) < -1.0f || (c.x / st) > 1.0f) return false;
    uv = V2(u, acosf(c.x / st) * kInvTwoPi);
    return true;
}

// Directed rounding for the self-intersection offsets (SelfHit.h:124-190),
// emulated through binary64 (exact for the operand ranges of voxel faces).
VX_HD float round_up_d(double d) {
    float r = (float)d;
    if ((double)r < d) r = nextafterf(r, INFINITY);
    return r;
}
VX_HD float round_dn_d(double d) {
    float r = (float)d;
    if ((double)r > d) r = nextafterf(r, -INFINITY);
    return r;
}
VX_HD float fma_ru(float a, float b, float c) { return round_up_d((double)a * (double)b + (double)c); }
VX_HD float fma_rd(float a, float b, float c) { return round_dn_d((double)a * (double)b + (double)c); }
VX_HD float mul_ru(float a, float b) { return round_up_d((double)a * (double)b); }
VX_HD float add_ru(float a, float b) { return round_up_d((double)a + (double)b); }

}  // namespace vx
