// dmath.hpp -- float3 / 3x3 / quaternion arithmetic for the arena kernels, in the operation
// order of Bullet LinearMath (btVector3.h, btMatrix3x3.h, btQuaternion.h, btTransformUtil.h)
// that RocketSim runs on, so results agree bit for bit with the CPU oracle when both are built
// without FMA contraction.  Division is multiplication by the reciprocal (btVector3::operator/);
// v*M dots with columns; transcendentals come from include/rlgpu_detmath.h.
//
// Every operation whose arithmetic depends on the reference build's Bullet code path takes the set's
// arithmetic mode `ar` (include/rlgpu_arith.h): the x86 modes follow the BT_USE_SSE_IN_API branches
// (rsqrtss normalize, SSE quaternion dot / product, SSE setRotation / getRotation), RLGPU_ARITH_SCALAR
// Bullet's scalar code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rlgpu_arith.h"
#include "../../include/rlgpu_detmath.h"
#if !defined(__HIP_DEVICE_COMPILE__) && (defined(__x86_64__) || defined(__i386__))
#include <xmmintrin.h>
#endif

#define HD __host__ __device__ __forceinline__

namespace rl {

// This host's rsqrtss table (host/x86_arith.cpp, rlgpu_x86_rsqrt_table), uploaded by env.hip at create:
// one copy per translation unit, only env.hip's kernels read it.
struct RsqrtLut {
    const uint32_t* t;  // [2 << bits]
    int bits;
};
static __constant__ RsqrtLut kRsqrtLut;

// rsqrtss.  On the device the table lookup of rlgpu_x86_rsqrtss_emulated: zero / denormal -> +-inf,
// +inf -> 0, NaN -> quiet NaN, negative -> default NaN, a normal 2^(2q + p) * 1.m -> entry (p, top bits
// of m) scaled by 2^-q.  On the host the instruction itself (the library builds edge records with it).
HD float x86_rsqrtss(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    const uint32_t u = __float_as_uint(x);
    const uint32_t e = (u >> 23) & 0xffu, m = u & 0x7fffffu;
    if (e == 0u) return __uint_as_float((u & 0x80000000u) | 0x7f800000u);
    if (e == 0xffu) return m ? __uint_as_float(u | 0x400000u) : ((u >> 31) ? __uint_as_float(0xffc00000u) : 0.f);
    if (u >> 31) return __uint_as_float(0xffc00000u);
    const int E = (int)e - 127, p = E & 1, q = (E - p) / 2;
    const int bits = kRsqrtLut.bits;
    const uint32_t r = kRsqrtLut.t[((uint32_t)p << bits) | (m >> (23 - bits))];
    return __uint_as_float((uint32_t)((int32_t)r - q * (1 << 23)));
#elif defined(__x86_64__) || defined(__i386__)
    return _mm_cvtss_f32(_mm_rsqrt_ss(_mm_set_ss(x)));
#else
    return 1.f / sqrtf(x);  // no x86 host: the x86 modes are refused at create (rlgpu_x86_rsqrt_table)
#endif
}
HD bool sse_api(int ar) { return ar != RLGPU_ARITH_SCALAR; }

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
// btVector3::normalize (btVector3.h:304-345).  SSE: the squared length as mul_ps then add_ss (x + y) + z,
// rsqrtss, one Newton step y0 * (1.5 - ((d * 0.5) * y0) * y0), then the vector times it.  Scalar:
// *this /= length(), i.e. times 1 / sqrt.
HD v3 bt_normalize(v3 a, int ar) {
    if (!sse_api(ar)) return a / len(a);
    const float d = (a.x * a.x + a.y * a.y) + a.z * a.z;
    const float y0 = x86_rsqrtss(d);
    float h = d * 0.5f;
    h = h * y0;
    h = h * y0;
    const float r = y0 * (1.5f - h);
    return v3{a.x * r, a.y * r, a.z * r};
}
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
// btQuaternion operator* / *= (btQuaternion.h:253-284,619-650).  SSE: A0 = q1.w * q2, B1 = the (z x y z) x
// (y z x z) products, A1 = (x y z x) x (w w w x) + (y z x y) x (z x y y); result (A0 - B1) + A1 with A1's
// w negated.  Scalar: left to right.
HD quat qmul(quat a, quat b, int ar) {
    if (sse_api(ar))
        return quat{(a.w * b.x - a.z * b.y) + (a.x * b.w + a.y * b.z), (a.w * b.y - a.x * b.z) + (a.y * b.w + a.z * b.x),
                    (a.w * b.z - a.y * b.x) + (a.z * b.w + a.x * b.y), (a.w * b.w - a.z * b.z) + -(a.x * b.x + a.y * b.y)};
    return quat{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
                a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
// btQuaternion::length2 = dot(*this) (btQuaternion.h:337-366).  SSE: (xx + zz) + (yy + ww) (movehl, add_ps,
// add_ss); scalar: ((xx + yy) + zz) + ww.
HD float qlen2(quat q, int ar) {
    if (sse_api(ar)) return (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w);
    return q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
}
// btQuaternion::safeNormalize / normalize (btQuaternion.h:374-405): l2 > SIMD_EPSILON, then times
// 1 / sqrt(l2) (SSE: sqrt_ss, div_ss, mul_ps; scalar: /= length())
HD quat qsafe_normalize(quat q, int ar) {
    float l2 = qlen2(q, ar);
    if (l2 > kEps) {
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
// btMatrix3x3::setRotation (btMatrix3x3.h:216-280), s = 2 / q.length2().  SSE (:222-272): unscaled products
// summed per row, times s, plus the identity row: m00 = (-(yy) + -(zz)) s + 1, m01 = (xy + -(wz)) s + 0, ...
// Scalar: the products of q with q * s, 1 - (yy + zz) on the diagonal.
HD m3 mat_from_quat(quat q, int ar) {
    float d = qlen2(q, ar);
    float s = 2.0f / d;
    if (sse_api(ar)) {
        const float x = q.x, y = q.y, z = q.z, w = q.w;
        return m3{v3{(-(y * y) + -(z * z)) * s + 1.0f, (x * y + -(w * z)) * s + 0.0f, (z * x + y * w) * s + 0.0f},
                  v3{(x * y + z * w) * s + 0.0f, (-(x * x) + -(z * z)) * s + 1.0f, (y * z + -(w * x)) * s + 0.0f},
                  v3{(z * x + -(w * y)) * s + 0.0f, (y * z + w * x) * s + 0.0f, (-(x * x) + -(y * y)) * s + 1.0f}};
    }
    float xs = q.x * s, ys = q.y * s, zs = q.z * s;
    float wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
    float xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
    float yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
    return m3{v3{1.0f - (yy + zz), xy - wz, xz + wy}, v3{xy + wz, 1.0f - (xx + zz), yz - wx},
              v3{xz - wy, yz + wx, 1.0f - (xx + yy)}};
}
// btMatrix3x3::getRotation (btMatrix3x3.h:421-489).  Both paths pick the same branch and component sums;
// SSE (:423-474) keeps x = trace + 1 (or the diagonal sum) in the leading component and scales all four
// by 0.5 / sqrt(x), where scalar stores sqrt(x) * 0.5 there.
HD quat quat_from_mat(const m3& m, int ar) {
    const bool sse = sse_api(ar);
    float trace = m.r0.x + m.r1.y + m.r2.z;
    float t[4];
    if (trace > 0.0f) {
        float x = trace + 1.0f;
        float s = sqrtf(x);
        t[3] = sse ? x : s * 0.5f;
        s = 0.5f / s;
        if (sse) t[3] = t[3] * s;
        t[0] = (m.r2.y - m.r1.z) * s;
        t[1] = (m.r0.z - m.r2.x) * s;
        t[2] = (m.r1.x - m.r0.y) * s;
    } else {
        int i = m.r0.x < m.r1.y ? (m.r1.y < m.r2.z ? 2 : 1) : (m.r0.x < m.r2.z ? 2 : 0);
        // written out per i (j = i+1, k = i+2 mod 3): a runtime index would put m and t in scratch
        if (i == 0) {
            float x = m.r0.x - m.r1.y - m.r2.z + 1.0f;
            float s = sqrtf(x);
            t[0] = s * 0.5f;
            s = 0.5f / s;
            if (sse) t[0] = x * s;
            t[3] = (m.r2.y - m.r1.z) * s;
            t[1] = (m.r1.x + m.r0.y) * s;
            t[2] = (m.r2.x + m.r0.z) * s;
        } else if (i == 1) {
            float x = m.r1.y - m.r2.z - m.r0.x + 1.0f;
            float s = sqrtf(x);
            t[1] = s * 0.5f;
            s = 0.5f / s;
            if (sse) t[1] = x * s;
            t[3] = (m.r0.z - m.r2.x) * s;
            t[2] = (m.r2.y + m.r1.z) * s;
            t[0] = (m.r0.y + m.r1.x) * s;
        } else {
            float x = m.r2.z - m.r0.x - m.r1.y + 1.0f;
            float s = sqrtf(x);
            t[2] = s * 0.5f;
            s = 0.5f / s;
            if (sse) t[2] = x * s;
            t[3] = (m.r1.x - m.r0.y) * s;
            t[0] = (m.r0.z + m.r2.x) * s;
            t[1] = (m.r1.z + m.r2.y) * s;
        }
    }
    return quat{t[0], t[1], t[2], t[3]};
}
// btTransformUtil::integrateTransform (btTransformUtil.h:37-88), exponential map
HD void integrate_transform(v3 pos, const m3& rot, v3 linvel, v3 angvel, float dt, v3& out_pos, m3& out_rot, int ar) {
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
    quat orn0 = quat_from_mat(rot, ar);
    quat pred = qsafe_normalize(qmul(dorn, orn0, ar), ar);
    if (qlen2(pred, ar) > kEps)
        out_rot = mat_from_quat(pred, ar);
    else
        out_rot = rot;
}

}  // namespace rl
