// rsim_math.hpp -- ORACLE (test infrastructure only).
// Restatement of the Bullet LinearMath operations RocketSim relies on
// (GigaLearnCPP/RLGymCPP/RocketSim/libsrc/bullet3-3.24/LinearMath/btVector3.h,
//  btMatrix3x3.h, btQuaternion.h, btTransformUtil.h), keeping Bullet's operation order:
// division is multiplication by the reciprocal, vector*matrix dots with columns, etc.
// Which branch of the LinearMath headers the reference build compiles is g_arith (include/rlgpu_arith.h):
// the x86 builds define BT_USE_SSE_IN_API (btScalar.h:113-137, :217-223) and run the SSE branches
// restated below next to the scalar ones; rsqrtss is executed, not modelled (x86_rsqrtss).
#pragma once
#include <cfloat>
#include <cmath>
#include <xmmintrin.h>

#include "../include/rlgpu_arith.h"
#include "../include/rlgpu_detmath.h"

namespace orc {

// The reference build's arithmetic (RLGPU_ARITH_*), per thread: the env set sets it for every arena it
// steps (env_ref.cpp), a World for the edge records it builds.
inline thread_local int g_arith = RLGPU_ARITH_MSVC_X64;
inline bool sse_api() { return g_arith != RLGPU_ARITH_SCALAR; }
struct ArithScope {  // g_arith for a scope
    int saved;
    explicit ArithScope(int a) : saved(g_arith) { g_arith = a; }
    ~ArithScope() { g_arith = saved; }
};
// the instruction itself (the product's kernels look up this host's table of it)
__attribute__((noinline)) inline float x86_rsqrtss(float x) { return _mm_cvtss_f32(_mm_rsqrt_ss(_mm_set_ss(x))); }

constexpr float SIMD_EPSILON = FLT_EPSILON;
constexpr float SIMD_PI = 3.1415926535897932384626433832795029f;
constexpr float SIMD_HALF_PI = SIMD_PI * 0.5f;
constexpr float ANGULAR_MOTION_THRESHOLD = 0.5f * SIMD_HALF_PI;  // btRigidBody.h

struct V {
    float x = 0, y = 0, z = 0;
    V() = default;
    V(float a, float b, float c) : x(a), y(b), z(c) {}
    float& operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
};
inline V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V operator-(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V operator-(V a) { return {-a.x, -a.y, -a.z}; }
inline V operator*(V a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V operator*(float s, V a) { return {a.x * s, a.y * s, a.z * s}; }
inline V operator*(V a, V b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V operator/(V a, float s) { return a * (1.0f / s); }  // btVector3 operator/
inline V& operator+=(V& a, V b) { a = a + b; return a; }
inline V& operator-=(V& a, V b) { a = a - b; return a; }
inline V& operator*=(V& a, float s) { a = a * s; return a; }
inline float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline float len2(V a) { return dot(a, a); }
inline float len(V a) { return std::sqrt(len2(a)); }
// btVector3::normalize / normalized (btVector3.h:304-345,958-963).  SSE: d = (xx + yy) + zz (mul_ps, two
// add_ss), y0 = rsqrtss(d), one Newton step y0 * (1.5 - ((d * 0.5) * y0) * y0), the vector times it.
// Scalar: *this /= length().
inline V bt_normalize(V a) {
    if (!sse_api()) return a / len(a);
    const float d = (a.x * a.x + a.y * a.y) + a.z * a.z;
    const float y0 = x86_rsqrtss(d);
    float h = d * 0.5f;
    h = h * y0;
    h = h * y0;
    const float r = y0 * (1.5f - h);
    return {a.x * r, a.y * r, a.z * r};
}
inline V safe_normalized(V a) {  // btVector3::safeNormalize
    float l2 = len2(a);
    if (l2 >= SIMD_EPSILON * SIMD_EPSILON) return a / std::sqrt(l2);
    return {1, 0, 0};
}
// RocketSim Vec::Length / Normalized (MathTypes.h:35-41,88-95): true division, zero-safe.
inline float rs_len(V a) {
    float l2 = a.x * a.x + a.y * a.y + a.z * a.z;
    return l2 > 0 ? std::sqrt(l2) : 0.f;
}
inline V rs_div(V a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline V rs_norm(V a) {
    float l = rs_len(a);
    if (l > FLT_EPSILON * FLT_EPSILON) return rs_div(a, l);
    return V();
}
inline bool is_zero(V a) { return a.x == 0 && a.y == 0 && a.z == 0; }
inline bool fuzzy_zero(V a) { return len2(a) < SIMD_EPSILON * SIMD_EPSILON; }

// btMatrix3x3: rows.
struct M {
    V r[3];
    V col(int i) const { return {r[0][i], r[1][i], r[2][i]}; }
    static M ident() { M m; m.r[0] = {1, 0, 0}; m.r[1] = {0, 1, 0}; m.r[2] = {0, 0, 1}; return m; }
};
inline V operator*(const M& m, V v) { return {dot(m.r[0], v), dot(m.r[1], v), dot(m.r[2], v)}; }
// v * M (btMatrix3x3 operator*(const btVector3&, const btMatrix3x3&): tdotx/y/z)
inline V vmul(V v, const M& m) {
    return {m.r[0].x * v.x + m.r[1].x * v.y + m.r[2].x * v.z, m.r[0].y * v.x + m.r[1].y * v.y + m.r[2].y * v.z,
            m.r[0].z * v.x + m.r[1].z * v.y + m.r[2].z * v.z};
}
inline M operator*(const M& a, const M& b) {
    M o;
    for (int i = 0; i < 3; i++) {
        // btMatrix3x3 operator*: row i dot columns of b (tdotx/tdoty/tdotz)
        V ri = a.r[i];
        o.r[i] = {b.r[0].x * ri.x + b.r[1].x * ri.y + b.r[2].x * ri.z, b.r[0].y * ri.x + b.r[1].y * ri.y + b.r[2].y * ri.z,
                  b.r[0].z * ri.x + b.r[1].z * ri.y + b.r[2].z * ri.z};
    }
    return o;
}
inline M transpose(const M& m) {
    M o;
    o.r[0] = m.col(0);
    o.r[1] = m.col(1);
    o.r[2] = m.col(2);
    return o;
}
inline M scaled(const M& m, V s) {  // btMatrix3x3::scaled: columns scaled
    M o;
    for (int i = 0; i < 3; i++) o.r[i] = {m.r[i].x * s.x, m.r[i].y * s.y, m.r[i].z * s.z};
    return o;
}
inline float cofac(const M& m, int r1, int c1, int r2, int c2) { return m.r[r1][c1] * m.r[r2][c2] - m.r[r1][c2] * m.r[r2][c1]; }
inline M inverse(const M& m) {  // btMatrix3x3::inverse
    V co(cofac(m, 1, 1, 2, 2), cofac(m, 1, 2, 2, 0), cofac(m, 1, 0, 2, 1));
    float det = dot(m.r[0], co);
    float s = 1.0f / det;
    M o;
    o.r[0] = {co.x * s, cofac(m, 0, 2, 2, 1) * s, cofac(m, 0, 1, 1, 2) * s};
    o.r[1] = {co.y * s, cofac(m, 0, 0, 2, 2) * s, cofac(m, 0, 2, 1, 0) * s};
    o.r[2] = {co.z * s, cofac(m, 0, 1, 2, 0) * s, cofac(m, 0, 0, 1, 1) * s};
    return o;
}

struct Q {
    float x, y, z, w;
};
// btQuaternion operator* and *= (btQuaternion.h:253-334,617-704).  The SSE branch forms
// A0 = q1.w * q2 and the lane products A1 = q1(x y z x) * q2(w w w x), A2 = q1(y z x y) * q2(z x y y),
// B1 = q1(z x y z) * q2(y z x z); it returns (A0 - B1) + (A1 + A2) with the w lane of A1 + A2 negated.
inline Q qmul(Q a, Q b) {
    if (sse_api())
        return {(a.w * b.x - a.z * b.y) + (a.x * b.w + a.y * b.z), (a.w * b.y - a.x * b.z) + (a.y * b.w + a.z * b.x),
                (a.w * b.z - a.y * b.x) + (a.z * b.w + a.x * b.y), (a.w * b.w - a.z * b.z) + -(a.x * b.x + a.y * b.y)};
    return {a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
            a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
// btQuaternion::length2 = dot(*this) (btQuaternion.h:337-366).  SSE: products, movehl + add_ps, then add_ss
// of lane 1: (xx + zz) + (yy + ww).  Scalar: left to right.
inline float qlen2(Q q) {
    if (sse_api()) return (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w);
    return q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
}
// btQuaternion::safeNormalize (btQuaternion.h:374-382): normalize() when length2 > SIMD_EPSILON, i.e.
// times 1 / sqrt(length2) (SSE: sqrt_ss, div_ss, mul_ps, :385-405; scalar: /= length())
inline Q qsafe_normalize(Q q) {
    float l2 = qlen2(q);
    if (l2 > SIMD_EPSILON) {
        float s = 1.0f / std::sqrt(l2);
        return {q.x * s, q.y * s, q.z * s, q.w * s};
    }
    return q;
}
inline Q quat_axis_angle(V axis, float angle) {  // btQuaternion::setRotation
    float d = len(axis);
    float s = rs_sinf_at(angle * 0.5f, RS_SITE_AXIS_ANGLE) / d;
    return {axis.x * s, axis.y * s, axis.z * s, rs_cosf_at(angle * 0.5f, RS_SITE_AXIS_ANGLE)};
}
// btMatrix3x3::setRotation (btMatrix3x3.h:216-280), s = 2 / q.length2().  The SSE branch (:222-272)
// builds each row from unscaled products -- row 0 (-yy + -zz, xy + -wz, zx + yw), row 1 (xy + zw,
// -xx + -zz, yz + -wx), row 2 (zx + -wy, yz + wx, -xx + -yy) -- multiplies by s and adds the identity
// row (1 or +0).  The scalar branch scales one factor first and forms 1 - (yy + zz) on the diagonal.
inline M mat_from_quat(Q q) {
    float d = qlen2(q);
    float s = 2.0f / d;
    if (sse_api()) {
        const float x = q.x, y = q.y, z = q.z, w = q.w;
        M m;
        m.r[0] = {(-(y * y) + -(z * z)) * s + 1.0f, (x * y + -(w * z)) * s + 0.0f, (z * x + y * w) * s + 0.0f};
        m.r[1] = {(x * y + z * w) * s + 0.0f, (-(x * x) + -(z * z)) * s + 1.0f, (y * z + -(w * x)) * s + 0.0f};
        m.r[2] = {(z * x + -(w * y)) * s + 0.0f, (y * z + w * x) * s + 0.0f, (-(x * x) + -(y * y)) * s + 1.0f};
        return m;
    }
    float xs = q.x * s, ys = q.y * s, zs = q.z * s;
    float wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
    float xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
    float yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
    M m;
    m.r[0] = {1.0f - (yy + zz), xy - wz, xz + wy};
    m.r[1] = {xy + wz, 1.0f - (xx + zz), yz - wx};
    m.r[2] = {xz - wy, yz + wx, 1.0f - (xx + yy)};
    return m;
}
// btMatrix3x3::getRotation (btMatrix3x3.h:421-489).  The SSE branch (:423-474) stores x = trace + 1 (or
// m[i][i] - m[j][j] - m[k][k] + 1) unscaled in the leading component and multiplies all four by
// 0.5 / sqrt(x); the scalar branch stores sqrt(x) * 0.5 there.  Branches and sums are the same.
inline Q quat_from_mat(const M& m) {
    const bool sse = sse_api();
    float trace = m.r[0].x + m.r[1].y + m.r[2].z;
    float t[4];
    if (trace > 0.0f) {
        const float x = trace + 1.0f;
        float s = std::sqrt(x);
        t[3] = s * 0.5f;
        s = 0.5f / s;
        if (sse) t[3] = x * s;
        t[0] = (m.r[2].y - m.r[1].z) * s;
        t[1] = (m.r[0].z - m.r[2].x) * s;
        t[2] = (m.r[1].x - m.r[0].y) * s;
    } else {
        int i = m.r[0].x < m.r[1].y ? (m.r[1].y < m.r[2].z ? 2 : 1) : (m.r[0].x < m.r[2].z ? 2 : 0);
        int j = (i + 1) % 3, k = (i + 2) % 3;
        const float x = m.r[i][i] - m.r[j][j] - m.r[k][k] + 1.0f;
        float s = std::sqrt(x);
        t[i] = s * 0.5f;
        s = 0.5f / s;
        if (sse) t[i] = x * s;
        t[3] = (m.r[k][j] - m.r[j][k]) * s;
        t[j] = (m.r[j][i] + m.r[i][j]) * s;
        t[k] = (m.r[k][i] + m.r[i][k]) * s;
    }
    return {t[0], t[1], t[2], t[3]};
}
// btTransformUtil::integrateTransform (exponential map)
inline void integrate_transform(V pos, const M& rot, V linvel, V angvel, float dt, V& out_pos, M& out_rot) {
    out_pos = pos + linvel * dt;
    float fAngle2 = len2(angvel);
    float fAngle = 0;
    if (fAngle2 > SIMD_EPSILON) fAngle = std::sqrt(fAngle2);
    if (fAngle * dt > ANGULAR_MOTION_THRESHOLD) fAngle = ANGULAR_MOTION_THRESHOLD / dt;
    V axis;
    if (fAngle < 0.001f)
        axis = angvel * (0.5f * dt - (dt * dt * dt) * 0.020833333333f * fAngle * fAngle);
    else
        axis = angvel * (rs_sinf_at(0.5f * fAngle * dt, RS_SITE_INTEGRATE) / fAngle);
    Q dorn{axis.x, axis.y, axis.z, rs_cosf_at(fAngle * dt * 0.5f, RS_SITE_INTEGRATE)};
    Q orn0 = quat_from_mat(rot);
    Q pred = qmul(dorn, orn0);
    pred = qsafe_normalize(pred);
    if (qlen2(pred) > SIMD_EPSILON)
        out_rot = mat_from_quat(pred);
    else
        out_rot = rot;
}

// btMatrix3x3::setEulerYPR(yaw, pitch, roll) == setEulerZYX(roll, pitch, yaw).
// Host-only (spawn tables are precomputed with libm and uploaded as data).
inline M euler_ypr(float yaw, float pitch, float roll) {
    float ci = std::cos(roll), cj = std::cos(pitch), ch = std::cos(yaw);
    float si = std::sin(roll), sj = std::sin(pitch), sh = std::sin(yaw);
    float cc = ci * ch, cs = ci * sh, sc = si * ch, ss = si * sh;
    M m;
    m.r[0] = {cj * ch, sj * sc - cs, sj * cc + ss};
    m.r[1] = {cj * sh, sj * ss + cc, sj * cs - sc};
    m.r[2] = {-sj, cj * si, cj * ci};
    return m;
}

}  // namespace orc
