/*
 * rlgpu_detmath.h -- deterministic float transcendentals shared by the HIP kernels and the
 * CPU oracle.
 *
 * The reference calls libm sinf/cosf/atan2f (btSin/btCos in btTransformUtil.h:71-73,
 * atan2f in Car.cpp:713, btAtan2/btAsin in btMatrix3x3.h:530-532).  libm and the device
 * math library differ in the last bits, and rigid-body simulation amplifies 1-ulp
 * differences over ticks.  Both sides of the parity test therefore use these Cephes-style
 * single-precision kernels, compiled with -ffp-contract=off on both sides, so the GPU and the oracle agree bit
 * for bit.  This is arithmetic infrastructure, not simulator logic.
 *
 * Measured against the float64 truth over the simulator's domains (tests/test_detmath_bound.py):
 * sin / cos <= 1 ulp, atan2 <= 3 ulp, asin <= 7 ulp (near |x| -> 1 only; glibc: <= 1 ulp each).
 * Swapping the host libm in moves one env step's obs / rewards by < 5e-5 relative, no mask or
 * terminal flips.
 */
#ifndef RLGPU_DETMATH_H
#define RLGPU_DETMATH_H

#if defined(__HIPCC__) || defined(__HIP__)
#define RLGPU_HD __host__ __device__ __forceinline__
#else
#define RLGPU_HD static inline
#endif

#define RLGPU_PI_F 3.14159265358979323846f

/* RLGPU_DETMATH_LIBM: the oracle's "libm" build variant (oracle/Makefile, build/liboracle_libm.so) swaps
 * the host libm in for sin / cos / atan / atan2 / asin to bound what these kernels change against the
 * reference's own libm calls (tests/test_detmath_bound.py).  Never defined for the product or the
 * default oracle. */
#if defined(RLGPU_DETMATH_LIBM) && !(defined(__HIPCC__) || defined(__HIP__))
#include <math.h>
#define RLGPU_LIBM_SWAP 1
#else
#define RLGPU_LIBM_SWAP 0
#endif

/* sin and cos of x (Cephes sinf/cosf, octant reduction with 3-part pi/4). */
RLGPU_HD void rs_sincosf(float xin, float* s_out, float* c_out) {
    const float FOPI = 1.27323954473516f;
    const float DP1 = 0.78515625f, DP2 = 2.4187564849853515625e-4f, DP3 = 3.77489497744594108e-8f;
#if RLGPU_LIBM_SWAP
    *s_out = sinf(xin);
    *c_out = cosf(xin);
    return;
#endif
    float x = xin;
    int ssign = 1, csign = 1;
    if (x < 0.0f) {
        x = -x;
        ssign = -1;
    }
    int j = (int)(FOPI * x);
    float y = (float)j;
    if (j & 1) {
        j += 1;
        y += 1.0f;
    }
    j &= 7;
    if (j > 3) {
        ssign = -ssign;
        csign = -csign;
        j -= 4;
    }
    if (j > 1) csign = -csign;
    x = ((x - y * DP1) - y * DP2) - y * DP3;
    float z = x * x;
    float sp = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * x + x;
    float cp = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z - 0.5f * z + 1.0f;
    float s, c;
    if (j == 1 || j == 2) {
        s = cp;
        c = sp;
    } else {
        s = sp;
        c = cp;
    }
    *s_out = ssign < 0 ? -s : s;
    *c_out = csign < 0 ? -c : c;
}

RLGPU_HD float rs_sinf(float x) {
    float s, c;
    rs_sincosf(x, &s, &c);
    return s;
}

RLGPU_HD float rs_cosf(float x) {
    float s, c;
    rs_sincosf(x, &s, &c);
    return c;
}

/* atan(x) (Cephes atanf). */
RLGPU_HD float rs_atanf(float xin) {
#if RLGPU_LIBM_SWAP
    return atanf(xin);
#endif
    float x = xin, y;
    int neg = 0;
    if (x < 0.0f) {
        neg = 1;
        x = -x;
    }
    if (x > 2.414213562373095f) {
        y = RLGPU_PI_F * 0.5f;
        x = -(1.0f / x);
    } else if (x > 0.4142135623730950f) {
        y = RLGPU_PI_F * 0.25f;
        x = (x - 1.0f) / (x + 1.0f);
    } else {
        y = 0.0f;
    }
    float z = x * x;
    y += (((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z - 3.33329491539e-1f) * z * x + x;
    return neg ? -y : y;
}

/* atan2(y, x) with the usual quadrant conventions. */
RLGPU_HD float rs_atan2f(float y, float x) {
#if RLGPU_LIBM_SWAP
    return atan2f(y, x);
#endif
    if (x == 0.0f) {
        if (y > 0.0f) return RLGPU_PI_F * 0.5f;
        if (y < 0.0f) return -RLGPU_PI_F * 0.5f;
        return 0.0f;
    }
    float z = rs_atanf(y / x);
    if (x < 0.0f) {
        if (y < 0.0f) z -= RLGPU_PI_F;
        else z += RLGPU_PI_F;
    }
    return z;
}

/* asin(x) = atan2(x, sqrt(1 - x^2)) (sqrt is correctly rounded on both sides). */
RLGPU_HD float rs_asinf(float x, float sqrt_one_minus_x2) {
#if RLGPU_LIBM_SWAP
    (void)sqrt_one_minus_x2;
    return asinf(x);
#endif
    return rs_atan2f(x, sqrt_one_minus_x2);
}

/* The action sampler's exp / log (the reference's torch::softmax and .log(), PPOLearner.cpp:97-113,
 * 131-141): the same Cephes-style kernels on both sides so the sampled action indices and log probs
 * of the GPU and the CPU oracle agree bit for bit.  The device sampler compiles them under
 * "#pragma clang fp contract(off)" (no FMA contraction), the oracle with -ffp-contract=off. */
RLGPU_HD float rs_bits_float(unsigned int u) {
    union {
        unsigned int u;
        float f;
    } c;
    c.u = u;
    return c.f;
}
RLGPU_HD unsigned int rs_float_bits(float f) {
    union {
        unsigned int u;
        float f;
    } c;
    c.f = f;
    return c.u;
}

/* e^x (Cephes expf: x = n ln2 + r with a 2-part ln2, degree-6 polynomial, exact scaling by 2^n).
 * Results below FLT_MIN are flushed to +0 (x < -87.33: a softmax term that small is clamped to the
 * 1e-11 floor anyway); x > 88.72 gives +inf; NaN stays NaN. */
RLGPU_HD float rs_expf(float x) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    if (x != x) return x;
    if (x > 88.72283905206835f) return rs_bits_float(0x7f800000u);
    if (x < -87.33654475055310898657f) return 0.0f;
    float fx = 1.44269504088896341f * x + 0.5f;
    int n = (int)fx;
    if ((float)n > fx) n -= 1; /* floor */
    const float z0 = (float)n;
    float r = x - z0 * 0.693359375f;
    r = r - z0 * -2.12194440e-4f;
    const float z = r * r;
    float y = ((((1.9875691500E-4f * r + 1.3981999507E-3f) * r + 8.3334519073E-3f) * r + 4.1665795894E-2f) * r +
               1.6666665459E-1f) * r + 5.0000001201E-1f;
    y = y * z + r + 1.0f;
    /* n is in [-126, 128] over the accepted x range; 2^n is built exactly from its bits (n = 128 as
     * 2 * 2^127), so the result is one correctly rounded IEEE product on both sides */
    if (n > 127) {
        y = y * 2.0f;
        n -= 1;
    }
    return y * rs_bits_float((unsigned int)(n + 127) << 23);
}

/* natural log (Cephes logf: x = m 2^e, m in [sqrt(1/2), sqrt(2)), degree-9 polynomial in m - 1,
 * 2-part ln2).  x <= 0 gives -inf (0) or NaN. */
RLGPU_HD float rs_logf(float xin) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    if (xin != xin) return xin;
    if (xin <= 0.0f) return xin == 0.0f ? rs_bits_float(0xff800000u) : rs_bits_float(0x7fc00000u);
    if (xin == rs_bits_float(0x7f800000u)) return xin;
    float x = xin;
    int ebias = 0;
    if (x < 1.17549435e-38f) { /* subnormal: scale into the normal range (exact) */
        x = x * 33554432.0f;   /* 2^25 */
        ebias = -25;
    }
    const unsigned int b = rs_float_bits(x);
    int e = (int)((b >> 23) & 0xffu) - 126 + ebias;
    x = rs_bits_float((b & 0x807fffffu) | 0x3f000000u); /* mantissa in [0.5, 1) */
    if (x < 0.707106781186547524f) {
        e -= 1;
        x = (x + x) - 1.0f;
    } else {
        x = x - 1.0f;
    }
    const float z = x * x;
    float y = ((((((((7.0376836292E-2f * x - 1.1514610310E-1f) * x + 1.1676998740E-1f) * x - 1.2420140846E-1f) * x +
                   1.4249322787E-1f) * x - 1.6668057665E-1f) * x + 2.0000714765E-1f) * x - 2.4999993993E-1f) * x +
               3.3333331174E-1f) * x * z;
    const float fe = (float)e;
    y += -2.12194440e-4f * fe;
    y += -0.5f * z;
    float r = x + y;
    r += 0.693359375f * fe;
    return r;
}

#endif
