/*
 * rlgpu_detmath.h -- deterministic float transcendentals shared by the HIP kernels and the
 * CPU oracle.
 *
 * The reference calls libm sinf/cosf/atan2f (btSin/btCos in btTransformUtil.h:71-73,
 * atan2f in Car.cpp:713, btAtan2/btAsin in btMatrix3x3.h:530-532).  libm and the device
 * math library differ in the last bits, and rigid-body simulation amplifies 1-ulp
 * differences over ticks.  Both sides of the parity test therefore use these Cephes-style
 * single-precision kernels (<= 2 ulp from the true value over the ranges the simulator
 * uses), compiled with -ffp-contract=off on both sides, so the GPU and the oracle agree bit
 * for bit.  This is arithmetic infrastructure, not simulator logic.
 */
#ifndef RLGPU_DETMATH_H
#define RLGPU_DETMATH_H

#if defined(__HIPCC__) || defined(__HIP__)
#define RLGPU_HD __host__ __device__ __forceinline__
#else
#define RLGPU_HD static inline
#endif

#define RLGPU_PI_F 3.14159265358979323846f

/* sin and cos of x (Cephes sinf/cosf, octant reduction with 3-part pi/4). */
RLGPU_HD void rs_sincosf(float xin, float* s_out, float* c_out) {
    const float FOPI = 1.27323954473516f;
    const float DP1 = 0.78515625f, DP2 = 2.4187564849853515625e-4f, DP3 = 3.77489497744594108e-8f;
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
RLGPU_HD float rs_asinf(float x, float sqrt_one_minus_x2) { return rs_atan2f(x, sqrt_one_minus_x2); }

#endif
