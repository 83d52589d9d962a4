/*
 * rlgpu_arith.h -- which floating-point code paths of the reference's Bullet build the arena step
 * follows (rlgpu_envset_config.arith).
 *
 * Bullet's LinearMath and sequential-impulse solver compile to different arithmetic depending on the
 * compiler and target of the reference build:
 *   - x86 builds define BT_USE_SSE and BT_USE_SSE_IN_API (btScalar.h:113-137 for MSVC >= 2005 without
 *     clang, :217-223 for GCC / Clang on x86-64), so btVector3::normalize is rsqrtss plus one Newton
 *     step (btVector3.h:304-345), btQuaternion::dot / normalize / operator* and btMatrix3x3::setRotation /
 *     getRotation take their SSE branches (btQuaternion.h:337-405,619-650, btMatrix3x3.h:222-272,
 *     423-474), and btSolverBody.h:29-30 turns USE_SIMD on, which selects the _sse2 solver rows
 *     (btSequentialImpulseConstraintSolver.cpp:106-110,149-177,207-233,315-350);
 *   - MSVC >= 2012 also defines BT_ALLOW_SSE4, and on a CPU with SSE4.1 and FMA3 (every x86-64 CPU
 *     since 2013) setupSolverFunctions picks the _sse4_1_fma3 contact and friction rows
 *     (:180-205,235-260,359-382: _mm_dp_ps dots, fused multiply-adds); the split-impulse rows stay _sse2.
 * The reference builds with MSVC on Windows (build.ps1), so RLGPU_ARITH_MSVC_X64 is the
 * default (0).  RLGPU_ARITH_SCALAR is Bullet's scalar path (any build without SSE), kept as a regression
 * mode.
 *
 * rsqrtss is an approximation whose exact table is the CPU's own (Intel and AMD differ).  The library
 * reads this host's table once (rlgpu_x86_rsqrt_table) and the kernels look it up, so the device
 * computes what the reference computes on the machine it trains on; the oracle executes rsqrtss itself.
 */
#ifndef RLGPU_ARITH_H
#define RLGPU_ARITH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    RLGPU_ARITH_MSVC_X64 = 0, /* build.ps1: MSVC x64, SSE LinearMath, _sse4_1_fma3 contact / friction rows */
    RLGPU_ARITH_GCC_X64 = 1,  /* GCC / Clang x86-64: SSE LinearMath, _sse2 rows */
    RLGPU_ARITH_SCALAR = 2,   /* Bullet's scalar LinearMath and _scalar_reference rows */
    RLGPU_NUM_ARITH = 3
};

/* This host's rsqrtss table, read once per process: the instruction's result depends only on the input
 * exponent's parity and the top `*bits` mantissa bits (verified exhaustively over [1, 4) and across every
 * exponent when read), so table[(p << bits) | (mantissa >> (23 - bits))] holds the result bits for an
 * input of exponent 127 + p; other exponents scale by 2^-((E - p) / 2).  h_table may be NULL (query
 * only); else it must hold 2 << *bits entries (capacity given in `cap`).  RLGPU_ERR_UNSUPPORTED when the
 * host is not x86 or its rsqrtss does not have that structure (the x86 modes are then refused). */
int rlgpu_x86_rsqrt_table(uint32_t* h_table, int64_t cap, int32_t* bits);

/* The table-driven rsqrtss emulation the kernels use, evaluated on the host (tests compare it with the
 * instruction). */
float rlgpu_x86_rsqrtss_emulated(float x);

/* The mode-dependent LinearMath operations of the arena kernels on the device, one query per lane (tests
 * compare them with the oracle's restatement): op 0 btVector3::normalize v[3] -> v[3]; 1
 * btMatrix3x3::setRotation q[4] -> m[9]; 2 btMatrix3x3::getRotation m[9] -> q[4]; 3 btQuaternion product
 * a[4] b[4] -> q[4]; 4 btTransformUtil::integrateTransform of rot[9] pos[3] linvel[3] angvel[3] over 1/120 s
 * -> pos[3] rot[9]; 5 a wheel ray's btSubsimplexConvexCast (btCollisionWorld.cpp:277-310) of the segment
 * from[3] (at 9) to[3] (at 12) against a resting body of basis rot[9] (at 0) and origin o[3] (at 15), a box of
 * half extents h[3] (at 18, with its margin) or a sphere of radius r (at 21, > 0) -> hit, fraction, normal[3];
 * 6 the kernels' rsqrtss of the row's first 12 floats -> 12 floats; 7 the transcendentals of
 * include/rlgpu_detmath.h: sin in[0], cos in[0], atan2(in[1], in[2]), asin in[3], atan in[4] -> out[0..4].
 * d_in [n][24], d_out [n][12] floats (device).  Asynchronous on `stream`. */
int rlgpu_linear_math_queries(int32_t op, int32_t arith, const float* d_in, int32_t n, float* d_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
