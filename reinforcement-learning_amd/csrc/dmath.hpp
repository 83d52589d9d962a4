// dmath.hpp -- float3 / 3x3 / quaternion arithmetic for the arena kernels, in the operation
// order of Bullet LinearMath (btVector3.h, btMatrix3x3.h, btQuaternion.h, btTransformUtil.h)
// that RocketSim runs on, so results agree bit for bit with the CPU oracle when both are built
// without FMA contraction.  Division is multiplication by the reciprocal (btVector3::operator/);
// v*M dots with columns; transcendentals come from include/rlgpu_detmath.h.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/rlgpu_detmath.h"

#define HD __host__ __device__ __forceinline__

namespace rl {

constexpr float kEps = 1.1920928955078125e-07f;  // FLT_EPSILON == SIMD_EPSILON
constexpr float kPi = 3.1415926535897932384626433832795029f;
constexpr float kHalfPi = kPi * 0.5f;
constexpr float kAngularMotionThreshold = 0.5f * kHalfPi;

struct v3 {
    float x, y, z;
};
HD v3 mk(float a, float b, float c) { return v3{a, b, c}; }
HD v3 zero3() { return v3{0.f, 0.f, 0.f}; }
HD v3 operator+(v3 a, v3 b) { return v3{a.x + b.x, a.y + b.y, a.z + b.z}; }
HD v3 operator-(v3 a, v3 b) { return v3{a.x - b.x, a.y - b.y, a.z - b.z}; }
HD v3 operator-(v3 a) { return v3{-a.x, -a.y, -a.z}; }
HD v3 operator*(v3 a, float s) { return v3{a.x * s, a.y * s, a.z * s}; }
HD v3 operator*(float s, v3 a) { return v3{a.x * s, a.y * s, a.z * s}; }
HD v3 operator*(v3 a, v3 b) { return v3{a.x * b.x, a.y * b.y, a.z * b.z}; }
HD v3 operator/(v3 a, float s) { return a * (1.0f / s); }
HD v3& operator+=(v3& a, v3 b) { a = a + b; return a; }
HD v3& operator-=(v3& a, v3 b) { a = a - b; return a; }
HD v3& operator*=(v3& a, float s) { a = a * s; return a; }
HD float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// one of three vectors by a runtime index, as selects (keeps small vector tables in registers)
HD v3 sel3(v3 a, v3 b, v3 c, int i) {  // per component (a select of lvalues would select addresses)
    return v3{i == 0 ? a.x : (i == 1 ? b.x : c.x), i == 0 ? a.y : (i == 1 ? b.y : c.y), i == 0 ? a.z : (i == 1 ? b.z : c.z)};
}
HD v3 cross(v3 a, v3 b) { return v3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
HD float len2(v3 a) { return dot(a, a); }
HD float len(v3 a) { return sqrtf(len2(a)); }
HD v3 normalized(v3 a) { return a / len(a); }
HD v3 safe_normalized(v3 a) {
    float l2 = len2(a);
    if (l2 >= kEps * kEps) return a / sqrtf(l2);
    return v3{1.f, 0.f, 0.f};
}
HD bool is_zero(v3 a) { return a.x == 0.f && a.y == 0.f && a.z == 0.f; }
HD bool fuzzy_zero(v3 a) { return len2(a) < kEps * kEps; }
HD float comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
HD void set_comp(v3& a, int i, float v) {
    if (i == 0) a.x = v;
    else if (i == 1) a.y = v;
    else a.z = v;
}
// RocketSim Vec (MathTypes.h): true division, zero-safe length / normalize
HD float rs_len(v3 a) {
    float l2 = a.x * a.x + a.y * a.y + a.z * a.z;
    return l2 > 0.f ? sqrtf(l2) : 0.f;
}
HD v3 rs_div(v3 a, float s) { return v3{a.x / s, a.y / s, a.z / s}; }
HD v3 rs_norm(v3 a) {
    float l = rs_len(a);
    if (l > kEps * kEps) return rs_div(a, l);
    return zero3();
}

struct m3 {
    v3 r0, r1, r2;
};
HD v3 row(const m3& m, int i) { return sel3(m.r0, m.r1, m.r2, i); }
HD v3 col(const m3& m, int i) { return v3{comp(m.r0, i), comp(m.r1, i), comp(m.r2, i)}; }
HD m3 ident3() { return m3{v3{1, 0, 0}, v3{0, 1, 0}, v3{0, 0, 1}}; }
HD v3 operator*(const m3& m, v3 v) { return v3{dot(m.r0, v), dot(m.r1, v), dot(m.r2, v)}; }
HD v3 vmul(v3 v, const m3& m) {
    return v3{m.r0.x * v.x + m.r1.x * v.y + m.r2.x * v.z, m.r0.y * v.x + m.r1.y * v.y + m.r2.y * v.z,
              m.r0.z * v.x + m.r1.z * v.y + m.r2.z * v.z};
}
HD v3 mrow_mul(v3 ri, const m3& b) {
    return v3{b.r0.x * ri.x + b.r1.x * ri.y + b.r2.x * ri.z, b.r0.y * ri.x + b.r1.y * ri.y + b.r2.y * ri.z,
              b.r0.z * ri.x + b.r1.z * ri.y + b.r2.z * ri.z};
}
HD m3 operator*(const m3& a, const m3& b) { return m3{mrow_mul(a.r0, b), mrow_mul(a.r1, b), mrow_mul(a.r2, b)}; }
HD m3 transpose(const m3& m) { return m3{col(m, 0), col(m, 1), col(m, 2)}; }
HD m3 scaled(const m3& m, v3 s) {
    return m3{v3{m.r0.x * s.x, m.r0.y * s.y, m.r0.z * s.z}, v3{m.r1.x * s.x, m.r1.y * s.y, m.r1.z * s.z},
              v3{m.r2.x * s.x, m.r2.y * s.y, m.r2.z * s.z}};
}
HD float mel(const m3& m, int r, int c) { return comp(row(m, r), c); }
HD float cofac(const m3& m, int r1, int c1, int r2, int c2) { return mel(m, r1, c1) * mel(m, r2, c2) - mel(m, r1, c2) * mel(m, r2, c1); }
HD m3 inverse(const m3& m) {
    v3 co = v3{cofac(m, 1, 1, 2, 2), cofac(m, 1, 2, 2, 0), cofac(m, 1, 0, 2, 1)};
    float det = dot(m.r0, co);
    float s = 1.0f / det;
    return m3{v3{co.x * s, cofac(m, 0, 2, 2, 1) * s, cofac(m, 0, 1, 1, 2) * s},
              v3{co.y * s, cofac(m, 0, 0, 2, 2) * s, cofac(m, 0, 2, 1, 0) * s},
              v3{co.z * s, cofac(m, 0, 1, 2, 0) * s, cofac(m, 0, 0, 1, 1) * s}};
}

struct quat {
    float x, y, z, w;
};
HD quat qmul(quat a, quat b) {
    return quat{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
                a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
HD float qlen2(quat q) { return q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w; }
HD quat qsafe_normalize(quat q) {
    float l2 = qlen2(q);
    if (l2 >= kEps) {
        float s = 1.0f / sqrtf(l2);
        return quat{q.x * s, q.y * s, q.z * s, q.w * s};
    }
    return q;
}
HD quat quat_axis_angle(v3 axis, float angle) {
    float d = len(axis);
    float sa, ca;
    rs_sincosf(angle * 0.5f, &sa, &ca);
    float s = sa / d;
    return quat{axis.x * s, axis.y * s, axis.z * s, ca};
}
HD m3 mat_from_quat(quat q) {
    float d = qlen2(q);
    float s = 2.0f / d;
    float xs = q.x * s, ys = q.y * s, zs = q.z * s;
    float wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
    float xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
    float yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
    return m3{v3{1.0f - (yy + zz), xy - wz, xz + wy}, v3{xy + wz, 1.0f - (xx + zz), yz - wx},
              v3{xz - wy, yz + wx, 1.0f - (xx + yy)}};
}
HD quat quat_from_mat(const m3& m) {
    float trace = m.r0.x + m.r1.y + m.r2.z;
    float t[4];
    if (trace > 0.0f) {
        float s = sqrtf(trace + 1.0f);
        t[3] = s * 0.5f;
        s = 0.5f / s;
        t[0] = (m.r2.y - m.r1.z) * s;
        t[1] = (m.r0.z - m.r2.x) * s;
        t[2] = (m.r1.x - m.r0.y) * s;
    } else {
        int i = m.r0.x < m.r1.y ? (m.r1.y < m.r2.z ? 2 : 1) : (m.r0.x < m.r2.z ? 2 : 0);
        // written out per i (j = i+1, k = i+2 mod 3): a runtime index would put m and t in scratch
        if (i == 0) {
            float s = sqrtf(m.r0.x - m.r1.y - m.r2.z + 1.0f);
            t[0] = s * 0.5f;
            s = 0.5f / s;
            t[3] = (m.r2.y - m.r1.z) * s;
            t[1] = (m.r1.x + m.r0.y) * s;
            t[2] = (m.r2.x + m.r0.z) * s;
        } else if (i == 1) {
            float s = sqrtf(m.r1.y - m.r2.z - m.r0.x + 1.0f);
            t[1] = s * 0.5f;
            s = 0.5f / s;
            t[3] = (m.r0.z - m.r2.x) * s;
            t[2] = (m.r2.y + m.r1.z) * s;
            t[0] = (m.r0.y + m.r1.x) * s;
        } else {
            float s = sqrtf(m.r2.z - m.r0.x - m.r1.y + 1.0f);
            t[2] = s * 0.5f;
            s = 0.5f / s;
            t[3] = (m.r1.x - m.r0.y) * s;
            t[0] = (m.r0.z + m.r2.x) * s;
            t[1] = (m.r1.z + m.r2.y) * s;
        }
    }
    return quat{t[0], t[1], t[2], t[3]};
}
HD void integrate_transform(v3 pos, const m3& rot, v3 linvel, v3 angvel, float dt, v3& out_pos, m3& out_rot) {
    out_pos = pos + linvel * dt;
    float a2 = len2(angvel);
    float a = 0.f;
    if (a2 > kEps) a = sqrtf(a2);
    if (a * dt > kAngularMotionThreshold) a = kAngularMotionThreshold / dt;
    v3 axis;
    float sh, ch;
    if (a < 0.001f) {
        axis = angvel * (0.5f * dt - (dt * dt * dt) * 0.020833333333f * a * a);
    } else {
        rs_sincosf(0.5f * a * dt, &sh, &ch);
        axis = angvel * (sh / a);
    }
    float cw = rs_cosf(a * dt * 0.5f);
    quat dorn{axis.x, axis.y, axis.z, cw};
    quat orn0 = quat_from_mat(rot);
    quat pred = qsafe_normalize(qmul(dorn, orn0));
    if (qlen2(pred) > kEps)
        out_rot = mat_from_quat(pred);
    else
        out_rot = rot;
}

}  // namespace rl
