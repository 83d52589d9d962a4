/*
 * rlgpu_detmath.h -- deterministic float transcendentals shared by the HIP kernels and the
 * CPU oracle.
 *
 * The reference calls libm sinf/cosf/atan2f/asinf (btSin/btCos in btTransformUtil.h:71-73,
 * atan2f in Car.cpp:722, btAtan2/btAsin in btMatrix3x3.h:530-532).  libm and the device
 * math library differ in the last bits, and rigid-body simulation amplifies 1-ulp
 * differences over ticks.  Both sides of the parity test therefore use these kernels, compiled with
 * -ffp-contract=off on both sides, so the GPU and the oracle agree bit for bit.  The trig kernels are
 * correctly rounded (double evaluation, one rounding): against the float64 truth over the simulator's
 * domains they are 0 ulp (glibc: <= 1 ulp, 1-13 % of its results misrounded), so against any CRT the
 * only difference is that CRT's misroundings; swapping glibc in moves one env step's rewards and GAE
 * advantages by <= 7.5e-6 relative (tests/test_detmath_bound.py).  This is
 * arithmetic infrastructure, not simulator logic.
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

/* Call sites of the transcendentals.  The product ignores them; the oracle's libm variant swaps the host libm
 * in at the sites whose bit is set in rlgpu_libm_sites (tests/test_detmath_bound.py attributes the libm
 * residual per site). */
#define RS_SITE_ANY 0x7fffffff
#define RS_SITE_INTEGRATE 0x01  /* btTransformUtil::integrateTransform, btTransformUtil.h:71-73 */
#define RS_SITE_AXIS_ANGLE 0x02 /* btQuaternion::setRotation (state setters, kickoff yaw) */
#define RS_SITE_FLIP 0x04       /* Car::_UpdateDoubleJumpOrFlip's forward angle, Car.cpp:722-726 */
#define RS_SITE_EULER 0x08      /* btMatrix3x3::getEulerYPR (auto flip), btMatrix3x3.h:530-532 */
#define RS_SITE_KICKOFF 0x10    /* KickoffProximityReward2v2Enhanced.h:122-123 */
#define RS_SITE_BOXBOX 0x20     /* btBoxBoxDetector cullPoints2's btAtan2 */
#define RS_SITE_EDGE 0x40       /* btInternalEdgeUtility's btGetAngle */
#define RS_SITE_POW 0x80        /* SaveBoostReward's powf (the oracle's powf_det) */

#if RLGPU_LIBM_SWAP
#ifdef __cplusplus
extern "C" int rlgpu_libm_sites;
#else
extern int rlgpu_libm_sites;
#endif
#define RS_LIBM_AT(site) (rlgpu_libm_sites & (site))
#endif

/* The float transcendentals are evaluated in double and rounded to float once, so they are correctly rounded
 * but for inputs whose true value lies within ~2^-29 ulp of a rounding midpoint (none found in 2^27 samples,
 * tests/test_detmath_bound.py).  The double kernels are fdlibm's (k_sin / k_cos / s_atan: Sun's public
 * minimax coefficients) in plain IEEE + - * / sqrt with a fixed operation order, so host (gcc, SSE2) and
 * device (v_*_f64) give the same bits.  Double keeps every float input's range (no overflow / underflow in
 * y / x or 1 - x^2). */
RLGPU_HD unsigned long long rs_dbits(double d) {
    union {
        unsigned long long u;
        double d;
    } c;
    c.d = d;
    return c.u;
}
RLGPU_HD double rs_bits_double(unsigned long long u) {
    union {
        unsigned long long u;
        double d;
    } c;
    c.u = u;
    return c.d;
}
/* sin(x), cos(x) for |x| <= pi/4 (fdlibm __kernel_sin / __kernel_cos with a zero tail) */
RLGPU_HD double rs__ksin(double x) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    const double z = x * x, v = z * x;
    const double r = 8.33333333332248946124e-03 +
                     z * (-1.98412698298579493134e-04 +
                          z * (2.75573137070700676789e-06 + z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)));
    return x + v * (-1.66666666666666324348e-01 + z * r);
}
RLGPU_HD double rs__kcos(double x) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    const double z = x * x;
    const double r =
        z * (4.16666666666666019037e-02 +
             z * (-1.38888888888741095749e-03 +
                  z * (2.48015872894767294178e-05 +
                       z * (-2.75573143513906633035e-07 + z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + z * r);
}

/* sin and cos of x: Cody-Waite reduction by pi/2 in three 33-bit parts (k * part exact for |k| < 2^20, so
 * the reduced argument carries ~2^-52 relative error for |x| < 2^20 pi/2; beyond that the result is still
 * deterministic but loses accuracy -- the simulator's arguments are atan2 results and half angles, |x| <= 4). */
RLGPU_HD void rs__sincosf_det(float xin, float* s_out, float* c_out) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    if (xin == 0.0f) { /* sin(+-0) = +-0 */
        *s_out = xin;
        *c_out = 1.0f;
        return;
    }
    const double x = (double)xin;
    if (x - x != 0.0) { /* +-inf, NaN */
        *s_out = *c_out = (float)(x - x);
        return;
    }
    const double t = x * 6.36619772367581382433e-01; /* 2 / pi */
    unsigned int q = 0;
    double kd = 0.0;
    if (t < 2251799813685248.0 && t > -2251799813685248.0) { /* |t| < 2^51: round to nearest by 1.5 * 2^52 */
        const double big = t + 6755399441055744.0;
        q = (unsigned int)(rs_dbits(big) & 3ull);
        kd = big - 6755399441055744.0;
    }
    const double r = ((x - kd * 1.57079632673412561417e+00) - kd * 6.07710050630396597660e-11) -
                     kd * 2.02226624871116645580e-21;
    const double sr = rs__ksin(r), cr = rs__kcos(r);
    double s, c;
    switch (q) {
    case 0: s = sr; c = cr; break;
    case 1: s = cr; c = -sr; break;
    case 2: s = -sr; c = -cr; break;
    default: s = -cr; c = sr; break;
    }
    *s_out = (float)s;
    *c_out = (float)c;
}

/* atan(x) in double, x >= 0 or NaN (fdlibm s_atan: breakpoints 7/16, 11/16, 19/16, 39/16 with atan(1/2),
 * atan(1), atan(3/2), atan(inf) in hi + lo parts, odd polynomial of degree 21) */
RLGPU_HD double rs__atan_pos(double x) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    int id;
    double hi = 0.0, lo = 0.0;
    if (x < 0.4375) {
        id = -1;
    } else if (x < 0.6875) {
        id = 0;
        hi = 4.63647609000806093515e-01;
        lo = 2.26987774529616870924e-17;
        x = (2.0 * x - 1.0) / (2.0 + x);
    } else if (x < 1.1875) {
        id = 1;
        hi = 7.85398163397448278999e-01;
        lo = 3.06161699786838301793e-17;
        x = (x - 1.0) / (x + 1.0);
    } else if (x < 2.4375) {
        id = 2;
        hi = 9.82793723247329054082e-01;
        lo = 1.39033110312309984516e-17;
        x = (x - 1.5) / (1.0 + 1.5 * x);
    } else {
        id = 3;
        hi = 1.57079632679489655800e+00;
        lo = 6.12323399573676603587e-17;
        x = -1.0 / x;
    }
    const double z = x * x, w = z * z;
    const double s1 =
        z * (3.33333333333329318027e-01 +
             w * (1.42857142725034663711e-01 +
                  w * (9.09088713343650656196e-02 +
                       w * (6.66107313738753120669e-02 + w * (4.97687799461593236017e-02 + w * 1.62858201153657823623e-02)))));
    const double s2 = w * (-1.99999999998764832476e-01 +
                           w * (-1.11111104054623557880e-01 +
                                w * (-7.69187620504482999495e-02 + w * (-5.83357013379057348645e-02 + w * -3.65315727442169155270e-02))));
    if (id < 0) return x - x * (s1 + s2);
    return hi - ((x * (s1 + s2) - lo) - x);
}

/* atan2 of doubles that are exact images of floats, with C99's signed-zero / infinity cases; the result's sign
 * is y's */
RLGPU_HD double rs__atan2_d(double y, double x) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    if (x != x || y != y) return x + y;
    const int xneg = (int)(rs_dbits(x) >> 63);
    const double ay = rs_bits_double(rs_dbits(y) & 0x7fffffffffffffffull);
    const double ax = rs_bits_double(rs_dbits(x) & 0x7fffffffffffffffull);
    const double inf = rs_bits_double(0x7ff0000000000000ull);
    double r;
    if (ay == 0.0) {
        r = xneg ? 3.14159265358979311600e+00 : 0.0;
    } else if (ay == inf && ax == inf) {
        r = xneg ? 2.35619449019234483700e+00 : 7.85398163397448278999e-01;
    } else {
        r = rs__atan_pos(ay / ax); /* ax == 0 -> inf -> pi/2; ax == inf -> 0 */
        if (xneg) r = (3.14159265358979311600e+00 - r) + 1.22464679914735317720e-16;
    }
    return rs_bits_double(rs_dbits(r) | (rs_dbits(y) & 0x8000000000000000ull));
}

RLGPU_HD float rs__atan2f_det(float y, float x) { return (float)rs__atan2_d((double)y, (double)x); }

/* asin(x) = atan2(x, sqrt((1 - x)(1 + x))): both factors and their product are exact in double for a float x,
 * so nothing cancels near |x| -> 1; |x| > 1 gives NaN (the reference clamps first, btAsin). */
RLGPU_HD float rs__asinf_det(float xin) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    const double x = (double)xin;
    const double t = (1.0 - x) * (1.0 + x);
    if (!(t >= 0.0)) return (float)((x - x) / (x - x));
    return (float)rs__atan2_d(x, sqrt(t));
}

RLGPU_HD void rs_sincosf_at(float x, float* s_out, float* c_out, int site) {
#if RLGPU_LIBM_SWAP
    if (RS_LIBM_AT(site)) {
        *s_out = sinf(x);
        *c_out = cosf(x);
        return;
    }
#endif
    (void)site;
    rs__sincosf_det(x, s_out, c_out);
}
RLGPU_HD void rs_sincosf(float x, float* s_out, float* c_out) { rs_sincosf_at(x, s_out, c_out, RS_SITE_ANY); }

RLGPU_HD float rs_sinf_at(float x, int site) {
    float s, c;
    rs_sincosf_at(x, &s, &c, site);
    return s;
}
RLGPU_HD float rs_cosf_at(float x, int site) {
    float s, c;
    rs_sincosf_at(x, &s, &c, site);
    return c;
}
RLGPU_HD float rs_sinf(float x) { return rs_sinf_at(x, RS_SITE_ANY); }
RLGPU_HD float rs_cosf(float x) { return rs_cosf_at(x, RS_SITE_ANY); }

/* atan(x) */
RLGPU_HD float rs_atanf(float xin) {
#if RLGPU_LIBM_SWAP
    if (RS_LIBM_AT(RS_SITE_ANY)) return atanf(xin);
#endif
    const double r = rs__atan_pos(rs_bits_double(rs_dbits((double)xin) & 0x7fffffffffffffffull));
    return (float)rs_bits_double(rs_dbits(r) | (rs_dbits((double)xin) & 0x8000000000000000ull));
}

/* atan2(y, x) with C99's quadrant, signed-zero and infinity conventions */
RLGPU_HD float rs_atan2f_at(float y, float x, int site) {
#if RLGPU_LIBM_SWAP
    if (RS_LIBM_AT(site)) return atan2f(y, x);
#endif
    (void)site;
    return rs__atan2f_det(y, x);
}
RLGPU_HD float rs_atan2f(float y, float x) { return rs_atan2f_at(y, x, RS_SITE_ANY); }

/* asin(x), x in [-1, 1] */
RLGPU_HD float rs_asinf_at(float x, int site) {
#if RLGPU_LIBM_SWAP
    if (RS_LIBM_AT(site)) return asinf(x);
#endif
    (void)site;
    return rs__asinf_det(x);
}
RLGPU_HD float rs_asinf(float x) { return rs_asinf_at(x, RS_SITE_ANY); }

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
