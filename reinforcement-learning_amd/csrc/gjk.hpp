// gjk.hpp -- car hitbox (box) vs arena-mesh triangle narrowphase on the device, as Bullet 3.24 runs it
// for RocketSim (the reference's call chain, all in GigaLearnCPP/RLGymCPP/RocketSim/libsrc/bullet3-3.24/
// BulletCollision):
//   CollisionDispatch/btConvexConcaveCollisionAlgorithm.cpp:71-138   per triangle: normal early out on
//       both sides, then btConvexConvexAlgorithm (body 0 = box, body 1 = triangle)
//   CollisionDispatch/btConvexConvexAlgorithm.cpp:268-513           no polyhedral features, no perturbation:
//       one btGjkPairDetector query with maximum distance margin + contact breaking threshold
//   NarrowPhaseCollision/btGjkPairDetector.cpp:686-959              GJK on the margin-free shapes with the
//       Voronoi sub-distance solver (btVoronoiSimplexSolver.cpp:34-577), degenerate-case catch, the
//       penetration solver (btGjkEpaPenetrationDepthSolver.cpp:22-79 -> btGjkEpa2.cpp GJK + EPA with
//       margins, nine guesses, Distance fallback) and the AABB-centre normal-direction fix
//
// Layout: the Voronoi GJK state lives in registers (fixed-index arrays, runtime slots picked by selects);
// the penetration solver's GJK / EPA work set (support vertices, polytope faces and their lists, the
// horizon flood-fill stack) first runs in a small set in the arena's LDS (24 vertices, 28 live faces:
// every EPA run of the bench workload fits), and only when that overflows, or another lane of the arena
// holds it, in the lane's full-capacity GjkScratch in HBM (12 KB; MeshView::gjk; Bullet's 128 vertices /
// 256 faces).  EPA's face lists are index-linked, in Bullet's list order
// (the stock list's untouched tail is implicit), its recursions (EncloseOrigin, expand) are iterative.
// Every float operation is Bullet's, in its order (dmath.hpp conventions); the CPU oracle
// (oracle/gjk_ref.hpp) is an independent restatement and the two agree bit for bit.
#pragma once
#include "dmath.hpp"

#ifndef DEV
#define DEV __device__ __forceinline__
#endif
#ifdef RLGPU_GJK_TRACE
#define GJK_MARK(k) RLGPU_GJK_TRACE(k)
#else
#define GJK_MARK(k)
#endif
// the penetration solver's big, rarely-run pieces are called, not inlined, and their loops are not
// unrolled: one copy of each keeps the instruction footprint (and its cache misses) small
#define GJK_CALLED DEV

namespace rl {
namespace gjk {

constexpr float kLarge = 1e18f;          // BT_LARGE_FLOAT
constexpr float kRelError2 = 1.0e-6f;    // btGjkPairDetector.cpp:35
constexpr float kEqualVertex = 0.0001f;  // VORONOI_DEFAULT_EQUAL_VERTEX_THRESHOLD
constexpr int kGjkMaxIter = 128;         // GJK_MAX_ITERATIONS
constexpr float kGjkAccuracy = 0.0001f, kGjkMinDistance = 0.0001f, kGjkDuplicatedEps = 0.0001f;
constexpr int kEpaMaxVertices = 128, kEpaMaxFaces = 256, kEpaMaxIterations = 255;
constexpr float kEpaAccuracy = 0.0001f, kEpaPlaneEps = 0.00001f;
constexpr int kSV = 4 + kEpaMaxVertices;  // support vertices: GJK store 0..3, EPA store 4..131
constexpr uint16_t kNone = 0xffff;

struct SSV {
    v3 d, w;
};
struct SFace {
    v3 n;
    float d;
    uint8_t c[3];  // support vertices
    uint8_t f[3];  // adjacent faces
    uint8_t e[3];  // adjacent faces' edge indices
    uint8_t pass;
    uint16_t l[2];  // stock-list links (prev, next)
    uint16_t seq;   // > 0: in the hull, appended seq-th (0: not in the hull; findbest)
};
struct GjkScratch {
    SSV sv[kSV];
    SFace fc[kEpaMaxFaces];
    uint32_t stack[kEpaMaxFaces + 8];  // expand() frames: face | edge << 8 | stage << 10
};
// A penetration-solver work set: the full-capacity per-lane HBM scratch, or a small one in the arena's
// LDS (the narrowphase-time free tail of ArenaLDS::u).  A small set that would need more support
// vertices, live faces or expand() depth than it holds sets `overflow`; the query is then rerun on the
// HBM set from the start (every run is deterministic, so the rerun gives Bullet's result).
// AS: the address space the work set's pointers carry (1 global, 3 LDS), so that every access compiles
// to global_* / ds_* instructions instead of flat ones (a flat access to LDS pays the vector-memory path)
template <int AS>
struct ScrT {
    __attribute__((address_space(AS))) SSV* sv;
    __attribute__((address_space(AS))) SFace* fc;
    __attribute__((address_space(AS))) uint32_t* stack;
    int max_sv, max_fc, max_stack;
    int overflow;
};
struct Scr {  // the generic view handed around by the narrowphase
    SSV* sv;
    SFace* fc;
    uint32_t* stack;
    int max_sv, max_fc, max_stack;
    int overflow;
};
template <int AS>
DEV ScrT<AS> in_space(const Scr& s) {
    return ScrT<AS>{(__attribute__((address_space(AS))) SSV*)s.sv, (__attribute__((address_space(AS))) SFace*)s.fc,
                    (__attribute__((address_space(AS))) uint32_t*)s.stack, s.max_sv, s.max_fc, s.max_stack, 0};
}
// v3 members of work-set records are read / written component-wise (an address-space-qualified v3
// cannot bind the generic copy constructor / assignment)
template <typename R>
DEV v3 ldv(const R& r) {
    return v3{r.x, r.y, r.z};
}
template <typename R>
DEV void stv(R& r, v3 v) {
    r.x = v.x;
    r.y = v.y;
    r.z = v.z;
}
template <typename F>
DEV void copy_face(SFace& o, const F& f) {
    o.n = ldv(f.n);
    o.d = f.d;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        o.c[k] = f.c[k];
        o.f[k] = f.f[k];
        o.e[k] = f.e[k];
    }
    o.pass = f.pass;
    o.l[0] = f.l[0];
    o.l[1] = f.l[1];
}
DEV Scr hbm_view(GjkScratch* g) { return Scr{g->sv, g->fc, g->stack, kSV, kEpaMaxFaces, kEpaMaxFaces + 8, 0}; }
// wave mode's set (epa_wave): support vertices only, in the same bytes
constexpr int kWaveSV = 64;
DEV Scr wave_view(char* base) { return Scr{(SSV*)base, nullptr, nullptr, kWaveSV, 0, 0, 0}; }
// small set carved from `bytes` of LDS: 24 support vertices (20 EPA iterations), 28 live faces, depth 24
constexpr int kSmallSV = 24, kSmallFaces = 28, kSmallStack = 24;
constexpr int kSmallBytes = kSmallSV * (int)sizeof(SSV) + kSmallFaces * (int)sizeof(SFace) + kSmallStack * 4;
static_assert(kWaveSV * (int)sizeof(SSV) <= kSmallBytes, "the wave-mode set fits the small set's bytes");
DEV Scr lds_view(char* base) {
    return Scr{(SSV*)base, (SFace*)(base + kSmallSV * sizeof(SSV)),
               (uint32_t*)(base + kSmallSV * sizeof(SSV) + kSmallFaces * sizeof(SFace)), kSmallSV, kSmallFaces,
               kSmallStack, 0};
}

// ---------------------------------------------------------------- shapes
struct Shape {
    v3 impl;       // box half extents without margin
    float margin;  // box margin
    v3 t0, t1, t2;  // triangle (mesh space = world: identity transform)
    int ar;         // the set's arithmetic mode (include/rlgpu_arith.h): btVector3::normalize is bt_normalize
};
DEV v3 box_nm(const Shape& s, v3 d) {
    return v3{d.x >= 0 ? s.impl.x : -s.impl.x, d.y >= 0 ? s.impl.y : -s.impl.y, d.z >= 0 ? s.impl.z : -s.impl.z};
}
DEV v3 tri_nm(const Shape& s, v3 d) {  // dot3 + btVector3::maxAxis
    const float a = dot(d, s.t0), b = dot(d, s.t1), c = dot(d, s.t2);
    const int k = a < b ? (b < c ? 2 : 1) : (a < c ? 2 : 0);
    return sel3(s.t0, s.t1, s.t2, k);
}
DEV v3 unit_dir(v3 d, int ar) {  // localGetSupportVertexNonVirtual's localDirNorm.normalize() (btConvexShape.cpp:186-193)
    if (len2(d) < kEps * kEps) d = v3{-1.f, -1.f, -1.f};
    return bt_normalize(d, ar);
}
DEV v3 xf(const m3& b, v3 o, v3 x) { return b * x + o; }
DEV m3 transpose_times(const m3& a, const m3& m) {  // btMatrix3x3::transposeTimes
    m3 r;
    r.r0 = v3{a.r0.x * m.r0.x + a.r1.x * m.r1.x + a.r2.x * m.r2.x, a.r0.x * m.r0.y + a.r1.x * m.r1.y + a.r2.x * m.r2.y,
              a.r0.x * m.r0.z + a.r1.x * m.r1.z + a.r2.x * m.r2.z};
    r.r1 = v3{a.r0.y * m.r0.x + a.r1.y * m.r1.x + a.r2.y * m.r2.x, a.r0.y * m.r0.y + a.r1.y * m.r1.y + a.r2.y * m.r2.y,
              a.r0.y * m.r0.z + a.r1.y * m.r1.z + a.r2.y * m.r2.z};
    r.r2 = v3{a.r0.z * m.r0.x + a.r1.z * m.r1.x + a.r2.z * m.r2.x, a.r0.z * m.r0.y + a.r1.z * m.r1.y + a.r2.z * m.r2.y,
              a.r0.z * m.r0.z + a.r1.z * m.r1.z + a.r2.z * m.r2.z};
    return r;
}

// runtime slot of a 4-entry register array, as selects / predicated writes
DEV float pick(bool c, float a, float b) { return c ? a : b; }
DEV v3 pick(bool c, v3 a, v3 b) { return v3{c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z}; }
template <typename T>
DEV T get4(const T (&a)[4], int i) {  // selects of values (a select of lvalues selects addresses)
    const T x0 = a[0], x1 = a[1], x2 = a[2], x3 = a[3];
    return pick(i == 0, x0, pick(i == 1, x1, pick(i == 2, x2, x3)));
}
// every slot is rewritten with a select: a conditional store would become a store through a selected
// pointer, which keeps the array in private (scratch) memory
template <typename T>
DEV void put4(T (&a)[4], int i, const T& v) {
#pragma unroll
    for (int k = 0; k < 4; k++) a[k] = pick(k == i, v, a[k]);
}

// ---------------------------------------------------------------- btVoronoiSimplexSolver (registers)
struct Voronoi {
    v3 W[4], P[4], Q[4];
    int n;
    v3 lastW, cP1, cP2, cV;
    bool u[4];
    float bc[4];
    bool degenerate, needs_update, valid;
};
DEV void bc_reset(Voronoi& s) {
    s.degenerate = false;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        s.bc[k] = 0.f;
        s.u[k] = false;
    }
}
DEV bool bc_valid(const Voronoi& s) { return s.bc[0] >= 0.f && s.bc[1] >= 0.f && s.bc[2] >= 0.f && s.bc[3] >= 0.f; }
DEV void vor_reset(Voronoi& s) {
    s.valid = false;
    s.n = 0;
    s.needs_update = true;
    s.lastW = v3{kLarge, kLarge, kLarge};
    bc_reset(s);
}
template <int I>
DEV void vor_remove(Voronoi& s) {  // removeVertex(I): the last vertex moves into slot I
    const int last = s.n - 1;
    s.W[I] = get4(s.W, last);
    s.P[I] = get4(s.P, last);
    s.Q[I] = get4(s.Q, last);
    s.n = last;
}
DEV void vor_reduce(Voronoi& s) {
    if (s.n >= 4 && !s.u[3]) vor_remove<3>(s);
    if (s.n >= 3 && !s.u[2]) vor_remove<2>(s);
    if (s.n >= 2 && !s.u[1]) vor_remove<1>(s);
    if (s.n >= 1 && !s.u[0]) vor_remove<0>(s);
}
// closestPtPointTriangle with p = origin (btVoronoiSimplexSolver.cpp:313-408)
DEV void closest_tri(v3 a, v3 b, v3 c, v3& pt, bool& u0, bool& u1, bool& u2, float& w0, float& w1, float& w2) {
    const v3 p = zero3();
    u0 = u1 = u2 = false;
    const v3 ab = b - a, ac = c - a, ap = p - a;
    const float d1 = dot(ab, ap), d2 = dot(ac, ap);
    if (d1 <= 0.f && d2 <= 0.f) {
        pt = a; u0 = true; w0 = 1; w1 = 0; w2 = 0;
        return;
    }
    const v3 bp = p - b;
    const float d3 = dot(ab, bp), d4 = dot(ac, bp);
    if (d3 >= 0.f && d4 <= d3) {
        pt = b; u1 = true; w0 = 0; w1 = 1; w2 = 0;
        return;
    }
    const float vc = d1 * d4 - d3 * d2;
    if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) {
        const float v = d1 / (d1 - d3);
        pt = a + v * ab; u0 = u1 = true; w0 = 1 - v; w1 = v; w2 = 0;
        return;
    }
    const v3 cp = p - c;
    const float d5 = dot(ab, cp), d6 = dot(ac, cp);
    if (d6 >= 0.f && d5 <= d6) {
        pt = c; u2 = true; w0 = 0; w1 = 0; w2 = 1;
        return;
    }
    const float vb = d5 * d2 - d1 * d6;
    if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) {
        const float w = d2 / (d2 - d6);
        pt = a + w * ac; u0 = u2 = true; w0 = 1 - w; w1 = 0; w2 = w;
        return;
    }
    const float va = d3 * d6 - d5 * d4;
    if (va <= 0.f && (d4 - d3) >= 0.f && (d5 - d6) >= 0.f) {
        const float w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        pt = b + w * (c - b); u1 = u2 = true; w0 = 0; w1 = 1 - w; w2 = w;
        return;
    }
    const float denom = 1.f / (va + vb + vc);
    const float v = vb * denom, w = vc * denom;
    pt = a + ab * v + ac * w;
    u0 = u1 = u2 = true;
    w0 = 1 - v - w; w1 = v; w2 = w;
}
DEV int outside_plane(v3 a, v3 b, v3 c, v3 d) {  // pointOutsideOfPlane with p = origin
    const v3 p = zero3();
    const v3 nrm = cross(b - a, c - a);
    const float signp = dot(p - a, nrm), signd = dot(d - a, nrm);
    if (signd * signd < (1e-4f * 1e-4f)) return -1;
    return signp * signd < 0.f;
}
// closestPtPointTetrahedron (cpp:437-577) into the solver's bc / u / degenerate
DEV bool closest_tetra(Voronoi& s) {
    const v3 a = s.W[0], b = s.W[1], c = s.W[2], d = s.W[3];
    s.u[0] = s.u[1] = s.u[2] = s.u[3] = true;
    const int oABC = outside_plane(a, b, c, d), oACD = outside_plane(a, c, d, b), oADB = outside_plane(a, d, b, c),
              oBDC = outside_plane(b, d, c, a);
    if (oABC < 0 || oACD < 0 || oADB < 0 || oBDC < 0) {
        s.degenerate = true;
        return false;
    }
    if (!oABC && !oACD && !oADB && !oBDC) return false;
    float best = 3.40282346638528859812e+38f;  // FLT_MAX
    const v3 o = zero3();
    v3 q;
    bool t0, t1, t2;
    float w0, w1, w2;
    if (oABC) {
        closest_tri(a, b, c, q, t0, t1, t2, w0, w1, w2);
        const float sq = dot(q - o, q - o);
        if (sq < best) {
            best = sq;
            s.u[0] = t0; s.u[1] = t1; s.u[2] = t2; s.u[3] = false;
            s.bc[0] = w0; s.bc[1] = w1; s.bc[2] = w2; s.bc[3] = 0;
        }
    }
    if (oACD) {
        closest_tri(a, c, d, q, t0, t1, t2, w0, w1, w2);
        const float sq = dot(q - o, q - o);
        if (sq < best) {
            best = sq;
            s.u[0] = t0; s.u[1] = false; s.u[2] = t1; s.u[3] = t2;
            s.bc[0] = w0; s.bc[1] = 0; s.bc[2] = w1; s.bc[3] = w2;
        }
    }
    if (oADB) {
        closest_tri(a, d, b, q, t0, t1, t2, w0, w1, w2);
        const float sq = dot(q - o, q - o);
        if (sq < best) {
            best = sq;
            s.u[0] = t0; s.u[1] = t2; s.u[2] = false; s.u[3] = t1;
            s.bc[0] = w0; s.bc[1] = w2; s.bc[2] = 0; s.bc[3] = w1;
        }
    }
    if (oBDC) {
        closest_tri(b, d, c, q, t0, t1, t2, w0, w1, w2);
        const float sq = dot(q - o, q - o);
        if (sq < best) {
            best = sq;
            s.u[0] = false; s.u[1] = t0; s.u[2] = t2; s.u[3] = t1;
            s.bc[0] = 0; s.bc[1] = w0; s.bc[2] = w2; s.bc[3] = w1;
        }
    }
    return true;
}
// updateClosestVectorAndPoints (cpp:81-233)
DEV bool vor_update(Voronoi& s) {
    if (s.needs_update) {
        bc_reset(s);
        s.needs_update = false;
        if (s.n == 1) {
            s.cP1 = s.P[0];
            s.cP2 = s.Q[0];
            s.cV = s.cP1 - s.cP2;
            bc_reset(s);
            s.bc[0] = 1.f;
            s.valid = bc_valid(s);
        } else if (s.n == 2) {
            const v3 from = s.W[0], to = s.W[1];
            v3 diff = zero3() - from;
            const v3 v = to - from;
            float t = dot(v, diff);
            if (t > 0) {
                const float vv = dot(v, v);
                if (t < vv) {
                    t /= vv;
                    diff -= t * v;
                    s.u[0] = s.u[1] = true;
                } else {
                    t = 1;
                    diff -= v;
                    s.u[1] = true;
                }
            } else {
                t = 0;
                s.u[0] = true;
            }
            s.bc[0] = 1 - t; s.bc[1] = t; s.bc[2] = 0; s.bc[3] = 0;
            s.cP1 = s.P[0] + t * (s.P[1] - s.P[0]);
            s.cP2 = s.Q[0] + t * (s.Q[1] - s.Q[0]);
            s.cV = s.cP1 - s.cP2;
            vor_reduce(s);
            s.valid = bc_valid(s);
        } else if (s.n == 3) {
            v3 pt;
            closest_tri(s.W[0], s.W[1], s.W[2], pt, s.u[0], s.u[1], s.u[2], s.bc[0], s.bc[1], s.bc[2]);
            s.cP1 = s.P[0] * s.bc[0] + s.P[1] * s.bc[1] + s.P[2] * s.bc[2];
            s.cP2 = s.Q[0] * s.bc[0] + s.Q[1] * s.bc[1] + s.Q[2] * s.bc[2];
            s.cV = s.cP1 - s.cP2;
            vor_reduce(s);
            s.valid = bc_valid(s);
        } else if (s.n == 4) {
            if (closest_tetra(s)) {
                s.cP1 = s.P[0] * s.bc[0] + s.P[1] * s.bc[1] + s.P[2] * s.bc[2] + s.P[3] * s.bc[3];
                s.cP2 = s.Q[0] * s.bc[0] + s.Q[1] * s.bc[1] + s.Q[2] * s.bc[2] + s.Q[3] * s.bc[3];
                s.cV = s.cP1 - s.cP2;
                vor_reduce(s);
                s.valid = bc_valid(s);
            } else if (s.degenerate) {
                s.valid = false;
            } else {
                s.valid = true;
                s.cV = zero3();
            }
        } else {
            s.valid = false;
        }
    }
    return s.valid;
}
DEV bool vor_in_simplex(const Voronoi& s, v3 w) {
    bool found = false;
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (k < s.n && len2(w - s.W[k]) <= kEqualVertex) found = true;
    if (w.x == s.lastW.x && w.y == s.lastW.y && w.z == s.lastW.z) return true;
    return found;
}

// ---------------------------------------------------------------- btSubsimplexConvexCast (wheel rays)
// The convex branch of btCollisionWorld::rayTestSingleInternal (btCollisionWorld.cpp:277-310): the ray's point
// shape (btSphereShape(0), margin 0, identity basis) cast from `from` to `to` against a resting convex body with
// basis R and origin o by btSubsimplexConvexCast::calcTimeOfImpact (btSubSimplexConvexCast.cpp:30-153;
// btConvexCast.h:25-29: 32 iterations, epsilon 0.0001, allowed penetration 0).  sphere_r > 0: btSphereShape
// (margin = radius, btSphereShape.cpp:37-48); otherwise btBoxShape with half extents h including its margin
// (btBoxShape.h:47-56).  True when Bullet reports the cast (fraction, normal = n.normalized()).  The simplex
// state is the GJK's register Voronoi solver; the oracle (oracle/gjk_ref.hpp) restates the same.
constexpr float kSimdEps = 1.1920928955078125e-07f;  // SIMD_EPSILON = FLT_EPSILON
DEV v3 sphere_support(v3 d, float radius, int ar) {
    const v3 vn = len2(d) < kSimdEps * kSimdEps ? bt_normalize(v3{-1.f, -1.f, -1.f}, ar) : bt_normalize(d, ar);
    return radius * vn;  // getMargin() * vecnorm
}
DEV v3 box_support(v3 d, v3 h) {  // btFsels(d, h, -h)
    return v3{d.x >= 0.f ? h.x : -h.x, d.y >= 0.f ? h.y : -h.y, d.z >= 0.f ? h.z : -h.z};
}
DEV v3 interp3(v3 v0, v3 v1, float rt) {  // btVector3::setInterpolate3
    const float s = 1.f - rt;
    return v3{s * v0.x + rt * v1.x, s * v0.y + rt * v1.y, s * v0.z + rt * v1.z};
}
DEV bool ray_convex_cast(v3 from, v3 to, float sphere_r, v3 h, m3 R, v3 o, int ar, float& frac,
                                             v3& normal) {
    const m3 I = m3{v3{1.f, 0.f, 0.f}, v3{0.f, 1.f, 0.f}, v3{0.f, 0.f, 1.f}};
    auto supA = [&](v3 d, v3 org) { return I * sphere_support(vmul(d, I), 0.f, ar) + org; };
    auto supB = [&](v3 d, v3 org) {
        const v3 l = vmul(d, R);
        return R * (sphere_r > 0.f ? sphere_support(l, sphere_r, ar) : box_support(l, h)) + org;
    };
    Voronoi vs;
    vor_reset(vs);
    const v3 linA = to - from, linB = o - o;
    float lambda = 0.f;
    v3 iA = from, iB = o;
    const v3 r = linA - linB;
    v3 sa = supA(-r, iA), sb = supB(r, iB);
    v3 v = sa - sb;
    int max_iter = 32;
    v3 n = zero3();
    float dist2 = len2(v);
    while ((dist2 > 0.0001f) && max_iter--) {
        sa = supA(-v, iA);
        sb = supB(v, iB);
        v3 w = sa - sb;
        const float vdw = dot(v, w);
        if (lambda > 1.f) return false;
        if (vdw > 0.f) {
            const float vdr = dot(v, r);
            if (vdr >= -(kSimdEps * kSimdEps)) return false;
            lambda = lambda - vdw / vdr;
            iA = interp3(from, to, lambda);
            iB = interp3(o, o, lambda);
            w = sa - sb;
            n = v;
        }
        if (!vor_in_simplex(vs, w)) {  // addVertex
            vs.lastW = w;
            vs.needs_update = true;
            put4(vs.W, vs.n, w);
            put4(vs.P, vs.n, sa);
            put4(vs.Q, vs.n, sb);
            vs.n++;
        }
        const bool ok = vor_update(vs);  // closest(v)
        v = vs.cV;
        dist2 = ok ? len2(v) : 0.f;
    }
    frac = lambda;
    normal = len2(n) >= kSimdEps * kSimdEps ? bt_normalize(n, ar) : zero3();
    return !(dot(normal, r) >= -0.f);
}

// ---------------------------------------------------------------- btGjkEpa2 in the lane's scratch
struct Mink {
    Shape s;
    m3 toshape1, b0;  // b0 / o0: toshape0
    v3 o0;
    bool margins;
};
DEV Mink make_mink(const Shape& s, const m3& tb0, v3 to0, const m3& tb1, v3 to1, bool margins) {
    Mink m;
    m.s = s;
    m.toshape1 = transpose_times(tb1, tb0);
    m.b0 = transpose_times(tb0, tb1);  // btTransform::inverseTimes
    m.o0 = vmul(to1 - to0, tb0);
    m.margins = margins;
    return m;
}
DEV v3 support0(const Mink& m, v3 d) {
    if (m.margins) {
        const v3 n = unit_dir(d, m.s.ar);
        return box_nm(m.s, n) + m.s.margin * n;
    }
    return box_nm(m.s, d);
}
DEV v3 support1(const Mink& m, v3 d) {
    const v3 dd = m.toshape1 * d;
    v3 sup;
    if (m.margins) {
        const v3 n = unit_dir(dd, m.s.ar);
        sup = tri_nm(m.s, n) + 0.f * n;
    } else {
        sup = tri_nm(m.s, dd);
    }
    return xf(m.b0, m.o0, sup);
}
DEV v3 support(const Mink& m, v3 d) { return support0(m, d) - support1(m, -d); }

// the GJK of btGjkEpa2 (cpp:155-552): simplex vertex indices packed 8 bits each, store in scratch
struct Simp {
    uint32_t c;  // c[k] = (c >> 8k) & 255
    float p[4];
    int rank;
};
DEV int sc(const Simp& s, int k) { return (int)((s.c >> (8 * k)) & 255u); }
DEV void sc_set(Simp& s, int k, int v) { s.c = (s.c & ~(255u << (8 * k))) | ((uint32_t)v << (8 * k)); }
struct Gjk2 {
    Simp cs, ns;     // current / next simplex (swapped when Bullet flips m_current)
    uint32_t freev;  // free list: 4 slots of 8 bits
    int nfree;
    v3 ray;
    int status;  // Valid 0, Inside 1, Failed 2
};
template <int AS>
DEV void getsupport(ScrT<AS>& S, const Mink& m, v3 d, int idx) {
    const v3 dn = d / len(d);
    stv(S.sv[idx].d, dn);
    stv(S.sv[idx].w, support(m, dn));
}
template <int AS>
DEV void g2_append(ScrT<AS>& S, const Mink& m, Gjk2& g, Simp& s, v3 v) {
    put4(s.p, s.rank, 0.f);
    g.nfree--;
    const int idx = (int)((g.freev >> (8 * g.nfree)) & 255u);
    sc_set(s, s.rank, idx);
    s.rank++;
    getsupport(S, m, v, idx);
}
DEV void g2_remove(Gjk2& g, Simp& s) {
    s.rank--;
    const int idx = sc(s, s.rank);
    g.freev = (g.freev & ~(255u << (8 * g.nfree))) | ((uint32_t)idx << (8 * g.nfree));
    g.nfree++;
}
DEV float det3(v3 a, v3 b, v3 c) {
    return (a.y * b.z * c.x + a.z * b.x * c.y - a.x * b.z * c.y - a.y * b.x * c.z + a.x * b.y * c.z - a.z * b.y * c.x);
}
DEV float project2(v3 a, v3 b, float* w, uint32_t& m) {
    const v3 d = b - a;
    const float l = len2(d);
    if (l > 0.f) {
        const float t = l > 0 ? -dot(a, d) / l : 0;
        if (t >= 1) {
            w[0] = 0; w[1] = 1; m = 2;
            return len2(b);
        } else if (t <= 0) {
            w[0] = 1; w[1] = 0; m = 1;
            return len2(a);
        } else {
            w[1] = t;
            w[0] = 1 - t;
            m = 3;
            return len2(a + d * t);
        }
    }
    return -1;
}
DEV float project3(v3 a, v3 b, v3 c, float* w, uint32_t& m) {
    const v3 dl0 = a - b, dl1 = b - c, dl2 = c - a;
    const v3 n = cross(dl0, dl1);
    const float l = len2(n);
    if (l > 0.f) {
        float mindist = -1;
        float subw[2] = {0.f, 0.f};
        uint32_t subm = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const v3 vi = sel3(a, b, c, i), dli = sel3(dl0, dl1, dl2, i);
            if (dot(vi, cross(dli, n)) > 0) {
                const int j = i == 2 ? 0 : i + 1;
                const float subd = project2(vi, sel3(a, b, c, j), subw, subm);
                if ((mindist < 0) || (subd < mindist)) {
                    mindist = subd;
                    m = ((subm & 1) ? 1u << i : 0u) + ((subm & 2) ? 1u << j : 0u);
                    w[i] = subw[0];
                    w[j] = subw[1];
                    w[j == 2 ? 0 : j + 1] = 0;
                }
            }
        }
        if (mindist < 0) {
            const float d = dot(a, n);
            const float s = sqrtf(l);
            const v3 p = n * (d / l);
            mindist = len2(p);
            m = 7;
            w[0] = len(cross(dl1, b - p)) / s;
            w[1] = len(cross(dl2, c - p)) / s;
            w[2] = 1 - (w[0] + w[1]);
        }
        return mindist;
    }
    return -1;
}
DEV float project4(v3 a, v3 b, v3 c, v3 d, float* w, uint32_t& m) {
    const v3 dl0 = a - d, dl1 = b - d, dl2 = c - d;
    const float vl = det3(dl0, dl1, dl2);
    const bool ng = (vl * dot(a, cross(b - c, a - b))) <= 0;
    if (ng && (fabsf(vl) > 0.f)) {
        float mindist = -1;
        float subw[3] = {0.f, 0.f, 0.f};
        uint32_t subm = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int j = i == 2 ? 0 : i + 1;
            const float s = vl * dot(d, cross(sel3(dl0, dl1, dl2, i), sel3(dl0, dl1, dl2, j)));
            if (s > 0) {
                const float subd = project3(sel3(a, b, c, i), sel3(a, b, c, j), d, subw, subm);
                if ((mindist < 0) || (subd < mindist)) {
                    mindist = subd;
                    m = (subm & 1 ? 1u << i : 0u) + (subm & 2 ? 1u << j : 0u) + (subm & 4 ? 8u : 0u);
                    w[i] = subw[0];
                    w[j] = subw[1];
                    w[j == 2 ? 0 : j + 1] = 0;
                    w[3] = subw[2];
                }
            }
        }
        if (mindist < 0) {
            mindist = 0;
            m = 15;
            w[0] = det3(c, b, d) / vl;
            w[1] = det3(a, c, d) / vl;
            w[2] = det3(b, a, d) / vl;
            w[3] = 1 - (w[0] + w[1] + w[2]);
        }
        return mindist;
    }
    return -1;
}
template <int AS>
DEV v3 svw(const ScrT<AS>& S, int i) { return ldv(S.sv[i].w); }
// GJK::Evaluate (cpp:201-337); on return g.cs is m_simplex
template <int AS>
GJK_CALLED int g2_evaluate(ScrT<AS>& S, const Mink& m, Gjk2& g, v3 guess) {
    unsigned iterations = 0;
    float sqdist = 0, alpha = 0;
    v3 lastw[4];
    int clastw = 0;
    g.freev = 0u | (1u << 8) | (2u << 16) | (3u << 24);
    g.nfree = 4;
    g.status = 0;
    g.cs.rank = 0;
    g.cs.c = 0;
    g.ns.c = 0;
    g.ns.rank = 0;
    g.ray = guess;
    const float sqrl = len2(g.ray);
    g2_append(S, m, g, g.cs, sqrl > 0 ? -g.ray : v3{1, 0, 0});
    g.cs.p[0] = 1;
    g.ray = svw(S, sc(g.cs, 0));
    sqdist = sqrl;
    lastw[0] = lastw[1] = lastw[2] = lastw[3] = g.ray;
    do {
        const float rl = len(g.ray);
        if (rl < kGjkMinDistance) {
            g.status = 1;
            break;
        }
        g2_append(S, m, g, g.cs, -g.ray);
        const v3 w = svw(S, sc(g.cs, g.cs.rank - 1));
        bool found = false;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (len2(w - lastw[i]) < kGjkDuplicatedEps) found = true;
        if (found) {
            g2_remove(g, g.cs);
            break;
        }
        clastw = (clastw + 1) & 3;
        put4(lastw, clastw, w);
        const float omega = dot(g.ray, w) / rl;
        alpha = omega > alpha ? omega : alpha;
        if (((rl - alpha) - (kGjkAccuracy * rl)) <= 0) {
            g2_remove(g, g.cs);
            break;
        }
        float weights[4];
        uint32_t mask = 0;
        const v3 w0 = svw(S, sc(g.cs, 0)), w1 = svw(S, sc(g.cs, 1));
        if (g.cs.rank == 2) {
            sqdist = project2(w0, w1, weights, mask);
        } else if (g.cs.rank == 3) {
            sqdist = project3(w0, w1, svw(S, sc(g.cs, 2)), weights, mask);
        } else if (g.cs.rank == 4) {
            sqdist = project4(w0, w1, svw(S, sc(g.cs, 2)), svw(S, sc(g.cs, 3)), weights, mask);
        }
        if (sqdist >= 0) {
            g.ns.rank = 0;
            g.ns.c = 0;
            g.ray = zero3();
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (i < g.cs.rank) {
                    const int ci = sc(g.cs, i);
                    if (mask & (1u << i)) {
                        sc_set(g.ns, g.ns.rank, ci);
                        put4(g.ns.p, g.ns.rank, weights[i]);
                        g.ns.rank++;
                        g.ray += svw(S, ci) * weights[i];
                    } else {
                        g.freev = (g.freev & ~(255u << (8 * g.nfree))) | ((uint32_t)ci << (8 * g.nfree));
                        g.nfree++;
                    }
                }
            }
            const Simp t = g.cs;  // m_current = next
            g.cs = g.ns;
            g.ns = t;
            if (mask == 15) g.status = 1;
        } else {
            g2_remove(g, g.cs);
            break;
        }
        g.status = ((++iterations) < (unsigned)kGjkMaxIter) ? g.status : 2;
    } while (g.status == 0);
    return g.status;
}
// GJK::EncloseOrigin (cpp:338-402), its recursion unrolled by rank
template <int AS>
DEV bool enclose4(const ScrT<AS>& S, const Simp& s) {
    const v3 w3 = svw(S, sc(s, 3));
    return fabsf(det3(svw(S, sc(s, 0)) - w3, svw(S, sc(s, 1)) - w3, svw(S, sc(s, 2)) - w3)) > 0;
}
template <int AS>
GJK_CALLED bool enclose3(ScrT<AS>& S, const Mink& m, Gjk2& g, Simp& s) {
    const v3 w0 = svw(S, sc(s, 0));
    const v3 n = cross(svw(S, sc(s, 1)) - w0, svw(S, sc(s, 2)) - w0);
    if (len2(n) > 0) {
        g2_append(S, m, g, s, n);
        if (enclose4(S, s)) return true;
        g2_remove(g, s);
        g2_append(S, m, g, s, -n);
        if (enclose4(S, s)) return true;
        g2_remove(g, s);
    }
    return false;
}
template <int AS>
GJK_CALLED bool enclose2(ScrT<AS>& S, const Mink& m, Gjk2& g, Simp& s) {
    const v3 d = svw(S, sc(s, 1)) - svw(S, sc(s, 0));
#pragma unroll 1
    for (int i = 0; i < 3; ++i) {
        v3 axis = zero3();
        set_comp(axis, i, 1.f);
        const v3 p = cross(d, axis);
        if (len2(p) > 0) {
            g2_append(S, m, g, s, p);
            if (enclose3(S, m, g, s)) return true;
            g2_remove(g, s);
            g2_append(S, m, g, s, -p);
            if (enclose3(S, m, g, s)) return true;
            g2_remove(g, s);
        }
    }
    return false;
}
template <int AS>
DEV bool enclose_origin(ScrT<AS>& S, const Mink& m, Gjk2& g, Simp& s) {
    if (s.rank == 1) {
#pragma unroll 1
        for (int i = 0; i < 3; ++i) {
            v3 axis = zero3();
            set_comp(axis, i, 1.f);
            g2_append(S, m, g, s, axis);
            if (enclose2(S, m, g, s)) return true;
            g2_remove(g, s);
            g2_append(S, m, g, s, -axis);
            if (enclose2(S, m, g, s)) return true;
            g2_remove(g, s);
        }
        return false;
    }
    if (s.rank == 2) return enclose2(S, m, g, s);
    if (s.rank == 3) return enclose3(S, m, g, s);
    if (s.rank == 4) return enclose4(S, s);
    return false;
}

// ---- EPA (cpp:555-901) over scratch faces
struct Epa {
    uint16_t hull;    // hull list root (unused: the hull is the faces with seq > 0)
    int hull_count;
    int seq;          // hull appends so far (the newest face is the hull list's root in Bullet)
    uint16_t stock;   // recycled faces (pushed at the stock's front)
    int fresh;        // stock tail: faces fresh..255 never taken, in index order (EPA::Initialize)
    int status;       // Valid 0 .. Failed 9 (EPA::eStatus order)
    int nextsv;
};
template <int AS>
DEV void list_append(ScrT<AS>& S, uint16_t& root, int face) {
    auto& f = S.fc[face];
    f.l[0] = kNone;
    f.l[1] = root;
    if (root != kNone) S.fc[root].l[0] = (uint16_t)face;
    root = (uint16_t)face;
}
template <int AS>
DEV void list_remove(ScrT<AS>& S, uint16_t& root, int face) {
    auto& f = S.fc[face];
    if (f.l[1] != kNone) S.fc[f.l[1]].l[0] = f.l[0];
    if (f.l[0] != kNone) S.fc[f.l[0]].l[1] = f.l[1];
    if (face == root) root = f.l[1];
}
template <int AS>
DEV void stock_push(ScrT<AS>& S, Epa& E, int face) { list_append(S, E.stock, face); }
// The hull as Bullet keeps it, a list appended at its root, is only ever walked by findbest from the root;
// the walk's order is newest first, so each face's append number stands in for the links (no list updates,
// and findbest reads independent slots instead of chasing links)
template <int AS>
DEV void hull_append(ScrT<AS>& S, Epa& E, int face) {
    S.fc[face].seq = (uint16_t)(++E.seq);
    E.hull_count++;
}
template <int AS>
DEV void hull_remove(ScrT<AS>& S, Epa& E, int face) {
    S.fc[face].seq = 0;
    E.hull_count--;
}
template <int AS>
DEV void bind(ScrT<AS>& S, int fa, int ea, int fb, int eb) {
    S.fc[fa].e[ea] = (uint8_t)eb;
    S.fc[fa].f[ea] = (uint8_t)fb;
    S.fc[fb].e[eb] = (uint8_t)ea;
    S.fc[fb].f[eb] = (uint8_t)fa;
}
// EPA::newface's plane of (a, b, c): false when degenerate (|n| <= EPA_ACCURACY); else n normalised and d
// the distance of the nearest edge (EPA::getedgedist, btGjkEpa2.cpp) or of the plane
// Straight-line form (no divergent branches for the wave-mode EPA's lanes): the first edge of (ab, bc, ca)
// whose getedgedist test holds is selected, and its distance -- |a|, |b| or sqrt(max(q, 0)) -- or the
// plane's dot(a, n) / l is one select of operands for one division and one square root: the same
// operations on the same values as the short-circuit calls.
DEV bool face_plane(v3 aw, v3 bw, v3 cw, v3& n, float& d) {
    n = cross(bw - aw, cw - aw);
    const float l = len(n);
    if (!(l > kEpaAccuracy)) return false;
    const bool t0 = dot(aw, cross(bw - aw, n)) < 0, t1 = dot(bw, cross(cw - bw, n)) < 0, t2 = dot(cw, cross(aw - cw, n)) < 0;
    const bool edge = t0 || t1 || t2;
    const v3 ea = t0 ? aw : (t1 ? bw : cw), eb = t0 ? bw : (t1 ? cw : aw);
    const v3 ba = eb - ea;
    const float a_dot_ba = dot(ea, ba), b_dot_ba = dot(eb, ba);
    const float a_dot_b = dot(ea, eb);
    const bool use_a = a_dot_ba > 0, use_b = !use_a && b_dot_ba < 0;
    const float q = (edge ? (len2(ea) * len2(eb) - a_dot_b * a_dot_b) : dot(aw, n)) / (edge ? len2(ba) : l);
    const float root = sqrtf(use_a ? len2(ea) : (use_b ? len2(eb) : (q > 0.f ? q : 0.f)));
    d = edge ? root : q;
    n = n / l;
    return true;
}
// EPA::newface; returns the face or -1
template <int AS>
DEV int newface(ScrT<AS>& S, Epa& E, int a, int b, int c, bool forced) {
    int face;
    if (E.stock != kNone) {
        face = E.stock;
        list_remove(S, E.stock, face);
    } else if (E.fresh < S.max_fc) {
        face = E.fresh++;
    } else if (E.hull_count >= kEpaMaxFaces) {
        E.status = 5;  // OutOfFaces (Bullet's stock is empty: all 256 faces are in the hull)
        return -1;
    } else {
        S.overflow = 1;  // Bullet still has stock faces: too small a work set
        return -1;
    }
    hull_append(S, E, face);
    auto& F = S.fc[face];
    F.pass = 0;
    F.c[0] = (uint8_t)a;
    F.c[1] = (uint8_t)b;
    F.c[2] = (uint8_t)c;
    v3 n;
    float d;
    if (face_plane(svw(S, a), svw(S, b), svw(S, c), n, d)) {
        stv(F.n, n);
        F.d = d;
        if (forced || (d >= -kEpaPlaneEps)) return face;
        E.status = 3;  // NonConvex
    } else {
        stv(F.n, n);
        E.status = 2;  // Degenerated
    }
    hull_remove(S, E, face);
    stock_push(S, E, face);
    return -1;
}
// EPA::findbest (cpp:840-862): the first face of least d^2 on the walk from the hull's root, i.e. of the
// faces of least d^2 the one appended last.  Every allocated slot is read (independent loads, several in
// flight) instead of following the links one dependent load at a time.
template <int AS>
DEV int findbest(const ScrT<AS>& S, const Epa& E) {
    int minf = -1, bestseq = 0;
    float mind = 0.f;
#pragma unroll 4
    for (int f = 0; f < E.fresh; f++) {
        const int sq = S.fc[f].seq;
        const float d = S.fc[f].d;
        const float sqd = d * d;
        if (sq > 0 && (minf < 0 || sqd < mind || (sqd == mind && sq > bestseq))) {
            minf = f;
            mind = sqd;
            bestseq = sq;
        }
    }
    return minf;
}
// EPA::expand (cpp:864-900) as an explicit-stack walk: frame = face | edge << 8 | stage << 10.  The top
// frame lives in a register (the stack holds the frames below it), and a frame's face fields are loaded
// together before they are tested: the walk is a chain of dependent scratch round trips otherwise.  Same
// visits, same tests, same new faces and the same overflow decisions as the recursion.
template <int AS>
GJK_CALLED bool expand(ScrT<AS>& S, Epa& E, unsigned pass, int w, int f0, int e0, int& hcf, int& hff, int& hnf) {
    const v3 wv = svw(S, w);
    int sp = 1;
    uint32_t top = (uint32_t)f0 | ((uint32_t)e0 << 8);  // frame sp - 1
    bool ret = false;
    while (sp > 0) {
        const uint32_t fr = top;
        const int f = (int)(fr & 255u), e = (int)((fr >> 8) & 3u), stage = (int)(fr >> 10);
        const int e1 = e == 2 ? 0 : e + 1, e2 = e == 0 ? 2 : e - 1;
        bool pop = false;
        if (stage == 0) {
            auto& F = S.fc[f];
            const uint8_t fpass = F.pass;
            const v3 fn = ldv(F.n);
            const float fd = F.d;
            const int ce1 = F.c[e1], ce = F.c[e], nb = F.f[e1], nbe = F.e[e1];
            if (fpass != (uint8_t)pass) {
                if ((dot(fn, wv) - fd) < -kEpaPlaneEps) {
                    const int nf = newface(S, E, ce1, ce, w, false);
                    if (S.overflow) return false;
                    ret = false;
                    if (nf >= 0) {
                        bind(S, nf, 0, f, e);
                        if (hcf >= 0)
                            bind(S, hcf, 1, nf, 2);
                        else
                            hff = nf;
                        hcf = nf;
                        ++hnf;
                        ret = true;
                    }
                    pop = true;
                } else {
                    F.pass = (uint8_t)pass;
                    if (sp >= S.max_stack) {
                        S.overflow = 1;
                        return false;
                    }
                    S.stack[sp - 1] = fr | (1u << 10);
                    sp++;
                    top = (uint32_t)nb | ((uint32_t)nbe << 8);
                }
            } else {
                ret = false;
                pop = true;
            }
        } else if (stage == 1) {
            if (!ret) {
                pop = true;
            } else {
                const auto& F = S.fc[f];
                if (sp >= S.max_stack) {
                    S.overflow = 1;
                    return false;
                }
                S.stack[sp - 1] = (fr & 1023u) | (2u << 10);
                sp++;
                top = (uint32_t)F.f[e2] | ((uint32_t)F.e[e2] << 8);
            }
        } else {
            if (ret) {
                hull_remove(S, E, f);
                stock_push(S, E, f);
            }
            pop = true;
        }
        if (pop && --sp > 0) top = S.stack[sp - 1];
    }
    return ret;
}
// EPA::Evaluate (cpp:648-768) on the GJK's simplex s; out: normal, depth, result (rank, c, p)
template <int AS>
GJK_CALLED int epa_evaluate(ScrT<AS>& S, const Mink& m, Gjk2& g, Simp& s, v3 guess, v3& normal, float& depth, Simp& res) {
    Epa E;
    E.hull = kNone;
    E.hull_count = 0;
    E.seq = 0;
    E.stock = kNone;
    E.fresh = 0;
    E.status = 9;
    E.nextsv = 0;
    if ((s.rank > 1) && enclose_origin(S, m, g, s)) {
        E.status = 0;
        E.nextsv = 0;
        {
            const v3 w3 = svw(S, sc(s, 3));
            if (det3(svw(S, sc(s, 0)) - w3, svw(S, sc(s, 1)) - w3, svw(S, sc(s, 2)) - w3) < 0) {
                const int c0 = sc(s, 0), c1 = sc(s, 1);
                sc_set(s, 0, c1);
                sc_set(s, 1, c0);
                const float p0 = s.p[0];
                s.p[0] = s.p[1];
                s.p[1] = p0;
            }
        }
        const int s0 = sc(s, 0), s1 = sc(s, 1), s2 = sc(s, 2), s3 = sc(s, 3);
        const int t0 = newface(S, E, s0, s1, s2, true);
        const int t1 = newface(S, E, s1, s0, s3, true);
        const int t2 = newface(S, E, s2, s1, s3, true);
        const int t3 = newface(S, E, s0, s2, s3, true);
        if (S.overflow) return 9;
        if (E.hull_count == 4) {
            int best = findbest(S, E);
            SFace outer;
            copy_face(outer, S.fc[best]);
            unsigned pass = 0;
            bind(S, t0, 0, t1, 0);
            bind(S, t0, 1, t2, 0);
            bind(S, t0, 2, t3, 0);
            bind(S, t1, 1, t3, 2);
            bind(S, t1, 2, t2, 1);
            bind(S, t2, 2, t3, 1);
            E.status = 0;
            for (int iterations = 0; iterations < kEpaMaxIterations; ++iterations) {
                GJK_MARK(4);
                if (E.nextsv < kEpaMaxVertices) {
                    if (4 + E.nextsv >= S.max_sv) {
                        S.overflow = 1;
                        return 9;
                    }
                    int hcf = -1, hff = -1, hnf = 0;
                    const int w = 4 + E.nextsv++;
                    bool valid = true;
                    S.fc[best].pass = (uint8_t)(++pass);
                    const v3 bn = ldv(S.fc[best].n);
                    const float bd = S.fc[best].d;
                    getsupport(S, m, bn, w);
                    const float wdist = dot(bn, svw(S, w)) - bd;
                    GJK_MARK(6);
                    if (wdist > kEpaAccuracy) {
                        for (int j = 0; (j < 3) && valid; ++j) {
                            valid &= expand(S, E, pass, w, S.fc[best].f[j], S.fc[best].e[j], hcf, hff, hnf);
                            if (S.overflow) return 9;
                        }
                        GJK_MARK(7);
                        if (valid && (hnf >= 3)) {
                            bind(S, hcf, 1, hff, 2);
                            hull_remove(S, E, best);
                            stock_push(S, E, best);
                            best = findbest(S, E);
                            copy_face(outer, S.fc[best]);
                            GJK_MARK(8);
                        } else {
                            E.status = 4;  // InvalidHull
                            break;
                        }
                    } else {
                        E.status = 7;  // AccuraryReached
                        break;
                    }
                } else {
                    E.status = 6;  // OutOfVertices
                    break;
                }
            }
            const v3 projection = outer.n * outer.d;
            normal = outer.n;
            depth = outer.d;
            res.rank = 3;
            res.c = 0;
            sc_set(res, 0, outer.c[0]);
            sc_set(res, 1, outer.c[1]);
            sc_set(res, 2, outer.c[2]);
            const v3 o0 = svw(S, outer.c[0]), o1 = svw(S, outer.c[1]), o2 = svw(S, outer.c[2]);
            res.p[0] = len(cross(o1 - projection, o2 - projection));
            res.p[1] = len(cross(o2 - projection, o0 - projection));
            res.p[2] = len(cross(o0 - projection, o1 - projection));
            const float sum = res.p[0] + res.p[1] + res.p[2];
            res.p[0] /= sum;
            res.p[1] /= sum;
            res.p[2] /= sum;
            return E.status;
        }
    }
    E.status = 8;  // FallBack
    normal = -guess;
    const float nl = len(normal);
    if (nl > 0)
        normal = normal / nl;
    else
        normal = v3{1, 0, 0};
    depth = 0;
    res.rank = 1;
    res.c = 0;
    sc_set(res, 0, sc(s, 0));
    res.p[0] = 1;
    return E.status;
}

// ---- EPA on the whole wave (wave mode: every lane of the wavefront runs the same query, in lockstep)
// The polytope lives in registers: face slot k is lane k's WFace, so the hull holds at most one face per
// lane.  Per iteration the lanes test every face against the new support point at once (one ballot), the
// walk of Bullet's expand recursion runs on those bits and the faces' adjacency words read across lanes
// (uniform, scalar), the horizon's new faces are built in parallel (one lane each, in the free slots),
// and findbest is a wave reduction.  Same faces, same order (append numbers), same tests, same failures:
//   * expand's first `false` (a face met twice) ends Bullet's iteration with InvalidHull and nothing after
//     it has any effect, so the walk stops there;
//   * a newface that fails (Degenerated / NonConvex) also ends the iteration with InvalidHull, and the
//     walk that Bullet would have cut short changes nothing else: the new faces are computed after the
//     walk and any failure among them ends the iteration the same way;
//   * the walk reads adjacency that expand's own binds never touch (binds change only new faces and the
//     horizon's non-visible faces, which expand never walks through).
// More support vertices than the set holds, more faces than lanes, a deeper walk than 64 frames: overflow,
// and the caller reruns the query on the full-capacity HBM set (scalar epa_evaluate).
struct WFace {
    v3 n;
    float d;
    uint32_t c;    // support vertices c0 | c1 << 8 | c2 << 16
    uint32_t adj;  // adjacent faces f0 | f1 << 8 | f2 << 16, their edges e0 << 24 | e1 << 26 | e2 << 28
    uint32_t seq;  // > 0: in the hull, appended seq-th
};
DEV uint32_t rdl(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
DEV float rdl(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
DEV v3 rdl(v3 v, int l) { return v3{rdl(v.x, l), rdl(v.y, l), rdl(v.z, l)}; }
DEV uint32_t wrl(uint32_t v, int l, uint32_t x) { return __lane_id() == l ? x : v; }  // lane l of v = x
DEV uint32_t rdfirst(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
DEV uint32_t lane_perm(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_ds_bpermute(l << 2, (int)v); }
// wave min / max without the LDS crossbar: xor-32 / xor-16 by v_permlane32_swap / v_permlane16_swap,
// then DPP row_ror 8 / 4 / 2 / 1 (mlp_kernels.hpp wave_max_x); every lane ends with the wave's result
template <int CTRL>
DEV uint32_t dpp_u(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false); }
template <bool MX>
DEV uint32_t wred(uint32_t v) {
    auto pick2 = [](uint32_t a, uint32_t b) { return MX ? (a > b ? a : b) : (a < b ? a : b); };
    auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = pick2(r[0], r[1]);
    r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = pick2(r[0], r[1]);
    v = pick2(v, dpp_u<0x128>(v));
    v = pick2(v, dpp_u<0x124>(v));
    v = pick2(v, dpp_u<0x122>(v));
    v = pick2(v, dpp_u<0x121>(v));
    return rdfirst(v);
}
DEV uint32_t wmin(uint32_t v) { return wred<false>(v); }
DEV uint32_t wmax(uint32_t v) { return wred<true>(v); }
DEV int lowbit(uint64_t m) { return __ffsll((unsigned long long)m) - 1; }
DEV int highbit(uint64_t m) { return 63 - __clzll((long long)m); }
// findbest over the lanes: least d^2, ties to the newest face
DEV int wfindbest(const WFace& F) {
    const int L = __lane_id();
    const bool alive = F.seq != 0;
    const uint32_t key = alive ? __float_as_uint(F.d * F.d) : 0xffffffffu;
    const uint32_t mk = wmin(key);
    const uint64_t tie = __ballot(alive && key == mk);
    if (__popcll(tie) == 1) return lowbit(tie);
    const bool in = (tie >> L) & 1;
    const uint32_t ms = wmax(in ? F.seq : 0u);
    return lowbit(__ballot(in && F.seq == ms));
}
DEV int adj_f(uint32_t adj, int e) { return (int)((adj >> (8 * e)) & 255u); }
DEV int adj_e(uint32_t adj, int e) { return (int)((adj >> (24 + 2 * e)) & 3u); }
// Bullet's expand from best's three edges over the visible-face bits `vis`.  Returns 1 when every call
// returned true, 0 at the first false, -1 on overflow.  Out: the horizon edges in creation order (lane j of
// H = face | edge << 8 | c[e1] << 16 | c[e] << 24 of the j-th: the face and its new face's first two
// vertices), their count, and the visible faces the walk removes.
DEV int wexpand(const WFace& F, int best, uint64_t vis, uint64_t lanes, uint32_t& H, int& nh, uint64_t& removed) {
    uint64_t visited = 1ull << best;
    removed = 0;
    nh = 0;
    uint32_t stk = 0;  // walk frames below the top, frame k in lane k: face | edge << 8 | stage << 10
    const uint32_t badj = rdl(F.adj, best);
    for (int j = 0; j < 3; j++) {
        uint32_t top = (uint32_t)adj_f(badj, j) | ((uint32_t)adj_e(badj, j) << 8);
        int sp = 0;
        while (true) {
            const int f = (int)(top & 255u), e = (int)((top >> 8) & 3u), stage = (int)(top >> 10);
            bool pop = false;
            if (stage == 0) {
                if ((visited >> f) & 1) return 0;  // f->pass == pass: expand returns false
                if (!((vis >> f) & 1)) {           // the face sees w below it: a horizon edge, newface(c[e1], c[e], w)
                    if (nh >= 64 || ((lanes >> nh) & 1) == 0) return -1;
                    const uint32_t fc = rdl(F.c, f);
                    const int e1 = e == 2 ? 0 : e + 1;
                    H = wrl(H, nh, top | (((fc >> (8 * e1)) & 255u) << 16) | (((fc >> (8 * e)) & 255u) << 24));
                    nh++;
                    pop = true;
                } else {  // visible: mark it, walk its edge e1, then e2, then remove it
                    visited |= 1ull << f;
                    if (sp >= 64 || ((lanes >> sp) & 1) == 0) return -1;
                    stk = wrl(stk, sp, top | (1u << 10));
                    sp++;
                    const int e1 = e == 2 ? 0 : e + 1;
                    const uint32_t adj = rdl(F.adj, f);
                    top = (uint32_t)adj_f(adj, e1) | ((uint32_t)adj_e(adj, e1) << 8);
                }
            } else if (stage == 1) {
                stk = wrl(stk, sp, (top & 1023u) | (2u << 10));
                sp++;
                const int e2 = e == 0 ? 2 : e - 1;
                const uint32_t adj = rdl(F.adj, f);
                top = (uint32_t)adj_f(adj, e2) | ((uint32_t)adj_e(adj, e2) << 8);
            } else {
                removed |= 1ull << f;
                pop = true;
            }
            if (pop) {
                if (sp == 0) break;
                top = rdl(stk, --sp);
            }
        }
    }
    return 1;
}
// EPA::Evaluate (cpp:648-768) in wave mode; same contract as epa_evaluate (S: support vertices only)
template <int AS>
GJK_CALLED int epa_wave(ScrT<AS>& S, const Mink& m, Gjk2& g, Simp& s, v3 guess, v3& normal, float& depth, Simp& res) {
    const int L = __lane_id();
    const uint64_t lanes = __ballot(1);
    if ((s.rank > 1) && enclose_origin(S, m, g, s)) {
        {
            const v3 w3 = svw(S, sc(s, 3));
            if (det3(svw(S, sc(s, 0)) - w3, svw(S, sc(s, 1)) - w3, svw(S, sc(s, 2)) - w3) < 0) {
                const int c0 = sc(s, 0), c1 = sc(s, 1);
                sc_set(s, 0, c1);
                sc_set(s, 1, c0);
                const float p0 = s.p[0];
                s.p[0] = s.p[1];
                s.p[1] = p0;
            }
        }
        const int s0 = sc(s, 0), s1 = sc(s, 1), s2 = sc(s, 2), s3 = sc(s, 3);
        // the tetrahedron: lane k builds t_k = newface(..., forced) and its binds
        const int ta = L == 1 ? s1 : (L == 2 ? s2 : s0);
        const int tb = L == 0 ? s1 : (L == 1 ? s0 : (L == 2 ? s1 : s2));
        const int tc = L == 0 ? s2 : s3;
        // adjacency after bind(t0,0,t1,0) bind(t0,1,t2,0) bind(t0,2,t3,0) bind(t1,1,t3,2) bind(t1,2,t2,1) bind(t2,2,t3,1)
        const uint32_t tadj = L == 0 ? (1u | 2u << 8 | 3u << 16)
                              : L == 1 ? (0u | 3u << 8 | 2u << 16 | 0u << 24 | 2u << 26 | 1u << 28)
                              : L == 2 ? (0u | 1u << 8 | 3u << 16 | 1u << 24 | 2u << 26 | 1u << 28)
                                       : (0u | 2u << 8 | 1u << 16 | 2u << 24 | 2u << 26 | 1u << 28);
        WFace F;
        F.n = zero3();
        F.d = 0.f;
        F.c = 0;
        F.adj = 0;
        F.seq = 0;
        bool ok = true;
        if (L < 4) {
            v3 n;
            float d;
            ok = face_plane(svw(S, ta), svw(S, tb), svw(S, tc), n, d);
            F.n = n;
            F.d = d;
            F.c = (uint32_t)ta | ((uint32_t)tb << 8) | ((uint32_t)tc << 16);
            F.adj = tadj;
            F.seq = (uint32_t)(L + 1);
        }
        if (__ballot(L < 4 && !ok) == 0) {  // all four made: m_hull.count == 4
            int best = wfindbest(F);
            v3 on = rdl(F.n, best);
            float od = rdl(F.d, best);
            uint32_t oc = rdl(F.c, best);
            uint32_t seq = 4;
            int nextsv = 0, status = 0;
            for (int iterations = 0; iterations < kEpaMaxIterations; ++iterations) {
                if (nextsv >= kEpaMaxVertices) {
                    status = 6;  // OutOfVertices
                    break;
                }
                if (4 + nextsv >= S.max_sv) {
                    S.overflow = 1;
                    return 9;
                }
                GJK_MARK(4);
                const int w = 4 + nextsv++;
                const v3 bn = rdl(F.n, best);
                const float bd = rdl(F.d, best);
                getsupport(S, m, bn, w);
                const v3 wv = svw(S, w);
                const float wdist = dot(bn, wv) - bd;
                GJK_MARK(6);
                if (!(wdist > kEpaAccuracy)) {
                    status = 7;  // AccuraryReached
                    break;
                }
                const uint64_t vis = __ballot(F.seq != 0 && !((dot(F.n, wv) - F.d) < -kEpaPlaneEps));
                uint32_t H = 0;
                int nh;
                uint64_t removed;
                const int walk = wexpand(F, best, vis, lanes, H, nh, removed);
                GJK_MARK(7);
                if (walk < 0) {
                    S.overflow = 1;
                    return 9;
                }
                if (walk == 0 || nh < 3) {
                    status = 4;  // InvalidHull
                    break;
                }
                // the new faces, in horizon order, take the free slots in ascending order
                const uint64_t keep = __ballot(F.seq != 0) & ~removed & ~(1ull << best);
                const uint64_t freem = lanes & ~keep;
                if (__popcll(freem) < nh) {
                    S.overflow = 1;
                    return 9;
                }
                const uint64_t below = (1ull << L) - 1ull;
                const bool in_free = (freem >> L) & 1;
                const int r = __popcll(freem & below);
                const bool host = in_free && r < nh;
                const uint32_t h = lane_perm(H, host ? r : 0);
                const int hf = (int)(h & 255u), he = (int)((h >> 8) & 3u);
                const int na = (int)((h >> 16) & 255u), nb = (int)(h >> 24);
                v3 nn = zero3();
                float nd = 0.f;
                bool nok = true;
                if (host) nok = face_plane(svw(S, na), svw(S, nb), wv, nn, nd) && (nd >= -kEpaPlaneEps);
                if (__ballot(host && !nok) != 0) {
                    status = 4;  // a newface failed (Degenerated / NonConvex): expand false, InvalidHull
                    break;
                }
                const int first = lowbit(freem);
                const int last = lowbit(__ballot(host && r == nh - 1));
                const uint64_t above = freem & ~below & ~(1ull << L);
                const int nxt = r + 1 < nh ? lowbit(above) : first;
                const int prv = r > 0 ? highbit(freem & below) : last;
                if (host) {  // bind(nf, 0, f, e); bind(prev, 1, nf, 2); bind(nf, 1, next, 2)
                    F.n = nn;
                    F.d = nd;
                    F.c = (uint32_t)na | ((uint32_t)nb << 8) | ((uint32_t)w << 16);
                    F.seq = seq + 1u + (uint32_t)r;
                    F.adj = (uint32_t)hf | ((uint32_t)nxt << 8) | ((uint32_t)prv << 16) | ((uint32_t)he << 24) |
                            (2u << 26) | (1u << 28);
                } else if (!((keep >> L) & 1)) {
                    F.seq = 0;  // removed (the best face and the walk's visible faces)
                }
                uint64_t fm = freem;
                for (int j = 0; j < nh; j++) {  // the horizon's faces: edge e now borders the new face
                    const int sj = lowbit(fm);
                    fm &= fm - 1ull;
                    const uint32_t hj = rdl(H, j);
                    const int fj = (int)(hj & 255u), ej = (int)((hj >> 8) & 3u);
                    if (L == fj)
                        F.adj = (F.adj & ~(255u << (8 * ej)) & ~(3u << (24 + 2 * ej))) | ((uint32_t)sj << (8 * ej));
                }
                seq += (uint32_t)nh;
                GJK_MARK(9);
                best = wfindbest(F);
                on = rdl(F.n, best);
                od = rdl(F.d, best);
                oc = rdl(F.c, best);
                GJK_MARK(8);
            }
            const v3 projection = on * od;
            normal = on;
            depth = od;
            res.rank = 3;
            res.c = oc & 0xffffffu;
            const v3 o0 = svw(S, (int)(oc & 255u)), o1 = svw(S, (int)((oc >> 8) & 255u)),
                     o2 = svw(S, (int)((oc >> 16) & 255u));
            res.p[0] = len(cross(o1 - projection, o2 - projection));
            res.p[1] = len(cross(o2 - projection, o0 - projection));
            res.p[2] = len(cross(o0 - projection, o1 - projection));
            const float sum = res.p[0] + res.p[1] + res.p[2];
            res.p[0] /= sum;
            res.p[1] /= sum;
            res.p[2] /= sum;
            return status;
        }
    }
    normal = -guess;  // FallBack
    const float nl = len(normal);
    if (nl > 0)
        normal = normal / nl;
    else
        normal = v3{1, 0, 0};
    depth = 0;
    res.rank = 1;
    res.c = 0;
    sc_set(res, 0, sc(s, 0));
    res.p[0] = 1;
    return 8;
}

// btGjkEpaSolver2::Penetration (cpp:973-1017) with margins; t0 / t1 = (basis, origin); W: wave-mode EPA
template <int AS, bool W>
DEV bool penetration(ScrT<AS>& S, const Shape& sh, const m3& b0, v3 o0, const m3& b1, v3 o1, v3 guess, v3& wA, v3& wB,
                     v3& nrm) {
    const Mink m = make_mink(sh, b0, o0, b1, o1, true);
    Gjk2 g;
    GJK_MARK(2);
    if (g2_evaluate(S, m, g, -guess) != 1) return false;
    GJK_MARK(3);
    v3 en;
    float ed;
    Simp res;
    const int es = W ? epa_wave(S, m, g, g.cs, -guess, en, ed, res) : epa_evaluate(S, m, g, g.cs, -guess, en, ed, res);
    GJK_MARK(5);
    if (es == 9 || S.overflow) return false;
    v3 w0 = zero3();
    for (int i = 0; i < res.rank; ++i) w0 += support0(m, ldv(S.sv[sc(res, i)].d)) * get4(res.p, i);
    wA = xf(b0, o0, w0);
    wB = xf(b0, o0, w0 - en * ed);
    nrm = -en;
    return true;
}
// btGjkEpaSolver2::Distance (cpp:937-970), margins off
template <int AS>
DEV bool distance(ScrT<AS>& S, const Shape& sh, const m3& b0, v3 o0, const m3& b1, v3 o1, v3 guess, v3& wA, v3& wB,
                  v3& nrm) {
    const Mink m = make_mink(sh, b0, o0, b1, o1, false);
    Gjk2 g;
    if (g2_evaluate(S, m, g, guess) != 0) return false;
    v3 w0 = zero3(), w1 = zero3();
    for (int i = 0; i < g.cs.rank; ++i) {
        const float p = get4(g.cs.p, i);
        const v3 d = ldv(S.sv[sc(g.cs, i)].d);
        w0 += support0(m, d) * p;
        w1 += support1(m, -d) * p;
    }
    wA = xf(b0, o0, w0);
    wB = xf(b0, o0, w1);
    nrm = w0 - w1;
    const float dist = len(nrm);
    nrm = nrm / (dist > kGjkMinDistance ? dist : 1);
    return true;
}
// btGjkEpaPenetrationDepthSolver::calcPenDepth (cpp:22-79); called, not inlined: the rare path stays out
// of the narrowphase's hot code
template <int AS, bool W = false>
__device__ __noinline__ bool calc_pen_depth(ScrT<AS>& S, const Shape& sh, const m3& bA, v3 oA, const m3& bB, v3 oB, v3& v, v3& wA, v3& wB) {
#pragma unroll 1
    for (int i = 0; i < 9; i++) {
        v3 g;
        if (i == 0) g = safe_normalized(oB - oA);
        else if (i == 1) g = safe_normalized(oA - oB);
        else if (i == 2) g = v3{0, 0, 1};
        else if (i == 3) g = v3{0, 1, 0};
        else if (i == 4) g = v3{1, 0, 0};
        else if (i == 5) g = v3{1, 1, 0};
        else if (i == 6) g = v3{1, 1, 1};
        else if (i == 7) g = v3{0, 1, 1};
        else g = v3{1, 0, 1};
        if (penetration<AS, W>(S, sh, bA, oA, bB, oB, g, wA, wB, v)) return true;
        if (S.overflow) return false;
        if (distance(S, sh, bA, oA, bB, oB, g, wA, wB, v)) return false;
    }
    wA = wB = v = zero3();
    return false;
}

// One box-triangle query (the caller did the AABB test).  R / c: the hitbox child's world basis and
// origin; cbt: the pair manifold's contact breaking threshold.  True when Bullet would call
// btManifoldResult::addContactPoint(normal, point, depth).  S: this lane's penetration-solver scratch.
// fast / lock: a small LDS work set and the lock that serialises it among the arena's lanes (null: HBM
// only); slow: this lane's HBM set.
constexpr int kPenInline = 0, kPenDefer = 1, kPenWave = 2;
// btGjkPairDetector's state where it may hand over to the penetration solver (what the rest of the query
// reads): a deferred query (kPenDefer) keeps it, the wave-mode rerun resumes from it
struct PenState {
    v3 pA, pB, nB;
    float dist;
    int valid;
};
// the query up to the penetration solver: 0 no contact (early out), 1 GJK's result stands, 2 the
// penetration solver runs (btGjkPairDetector.cpp:847-851: no valid result, or a degenerate one with the
// core distance below 0.01)
DEV int box_triangle_gjk(const m3& R, v3 c, const Shape& s, float cbt, PenState& st) {
    // normal early out, both sides (btConvexConcaveCollisionAlgorithm.cpp:101-136)
    {
        const v3 half = s.impl + v3{s.margin, s.margin, s.margin};
        const m3 inv = inverse(R);
        v3 tn = cross(s.t1 - s.t0, s.t2 - s.t0);
        tn = bt_normalize(tn, s.ar);  // triangle_normal_world.normalize() (btConvexConcaveCollisionAlgorithm.cpp:111)
#pragma unroll
        for (int side = 0; side < 2; side++) {
            const v3 ld = inv * tn;
            const v3 lp = v3{ld.x >= 0 ? half.x : -half.x, ld.y >= 0 ? half.y : -half.y, ld.z >= 0 ? half.z : -half.z};
            const v3 wp = R * lp + c;
            const float dist = dot(tn, s.t0) - dot(tn, wp);
            if (dist > cbt) return 0;
            tn = tn * -1.f;
        }
    }
    const float maxd = s.margin + 0.f + cbt;
    const float max2 = maxd * maxd;
    const m3 I = ident3();
    const v3 po = (c + zero3()) * 0.5f;
    const v3 oA = c - po, oB = zero3() - po;
    const float mA = s.margin, mB = 0.f;
    float distance_ = 0.f;
    v3 nB = zero3(), pA = zero3(), pB = zero3();
    v3 v = v3{0.f, 1.f, 0.f};
    bool valid = false, check = false;
    int degen = 0, iter = 0;
    float sqd = kLarge, delta = 0.f;
    const float margin = mA + mB;
    Voronoi vs;
    vor_reset(vs);
    while (true) {
        const v3 sa = vmul(-v, R), sb = vmul(v, I);
        const v3 pw = xf(R, oA, box_nm(s, sa)), qw = xf(I, oB, tri_nm(s, sb));
        const v3 w = pw - qw;
        delta = dot(v, w);
        if ((delta > 0.f) && (delta * delta > sqd * max2)) {
            degen = 10;
            check = true;
            break;
        }
        if (vor_in_simplex(vs, w)) {
            degen = 1;
            check = true;
            break;
        }
        const float f0 = sqd - delta, f1 = sqd * kRelError2;
        if (f0 <= f1) {
            degen = f0 <= 0.f ? 2 : 11;
            check = true;
            break;
        }
        vs.lastW = w;  // addVertex
        vs.needs_update = true;
        put4(vs.W, vs.n, w);
        put4(vs.P, vs.n, pw);
        put4(vs.Q, vs.n, qw);
        vs.n++;
        const bool ok = vor_update(vs);
        const v3 nv = vs.cV;
        if (!ok) {
            degen = 3;
            check = true;
            break;
        }
        if (len2(nv) < kRelError2) {
            v = nv;
            degen = 6;
            check = true;
            break;
        }
        const float prev = sqd;
        sqd = len2(nv);
        if (prev - sqd <= kEps * prev) {
            check = true;
            degen = 12;
            break;
        }
        v = nv;
        if (iter++ > 1000) break;
        GJK_MARK(1);
        if (vs.n == 4) {
            degen = 13;
            break;
        }
    }
    if (check) {
        vor_update(vs);  // compute_points
        pA = vs.cP1;
        pB = vs.cP2;
        nB = v;
        const float l2 = len2(v);
        if ((double)l2 < 0.0001) degen = 5;
        if (l2 > kEps * kEps) {
            const float rlen = 1.f / sqrtf(l2);
            nB *= rlen;
            const float sq = sqrtf(sqd);
            pA -= v * (mA / sq);
            pB += v * (mB / sq);
            distance_ = (1.f / rlen) - margin;
            valid = true;
        }
    }
    const bool catch_degen = degen && ((double)(distance_ + margin) < 0.01);
    st.pA = pA;
    st.pB = pB;
    st.nB = nB;
    st.dist = distance_;
    st.valid = valid ? 1 : 0;
    return (!valid || catch_degen) ? 2 : 1;
}
// mode: kPenInline runs the penetration solver where the query needs it; kPenDefer stops there instead
// (returns false, sets *deferred and *save: the caller reruns the query in wave mode); kPenWave, called by
// every lane of the wavefront with the same query, runs it with the wave-mode EPA on `fast` (support vertices
// only, kWaveSV of them), from `resume` (a deferred query's saved state) when given.
DEV bool box_triangle(const m3& R, v3 c, const Shape& s, float cbt, Scr* fast, int* lock, Scr& slow, v3& normal,
                      v3& point, float& depth, int* pen_count = nullptr, int mode = kPenInline, bool* deferred = nullptr,
                      PenState* save = nullptr, const PenState* resume = nullptr) {
    PenState st;
    int stage;
    if (resume) {
        st = *resume;
        stage = 2;
    } else {
        stage = box_triangle_gjk(R, c, s, cbt, st);
        if (stage == 0) return false;
    }
    const float maxd = s.margin + 0.f + cbt;
    const float max2 = maxd * maxd;
    const m3 I = ident3();
    const v3 po = (c + zero3()) * 0.5f;
    const v3 oA = c - po, oB = zero3() - po;
    const float mA = s.margin, mB = 0.f;
    const float margin = mA + mB;
    float distance_ = st.dist;
    v3 nB = st.nB, pA = st.pA, pB = st.pB, v;
    bool valid = st.valid != 0;
    if (stage == 2) {
        v3 tA, tB;
        v = zero3();
        bool ok2;
        if (mode == kPenDefer) {
            if (save) *save = st;
            *deferred = true;
            return false;
        }
        if (pen_count && (mode != kPenWave || __lane_id() == 0)) atomicAdd(pen_count, 1);
        ScrT<1> slow1 = in_space<1>(slow);
        if (mode == kPenWave) {
            ScrT<3> wave3 = in_space<3>(*fast);
            ok2 = calc_pen_depth<3, true>(wave3, s, R, oA, I, oB, v, tA, tB);
            if (wave3.overflow != 0) {
                v = zero3();
                ok2 = calc_pen_depth(slow1, s, R, oA, I, oB, v, tA, tB);
            }
        } else if (fast && atomicCAS(lock, 0, 1) == 0) {
            ScrT<3> fast3 = in_space<3>(*fast);
            ok2 = calc_pen_depth(fast3, s, R, oA, I, oB, v, tA, tB);
            const bool redo = fast3.overflow != 0;
            atomicExch(lock, 0);
            if (redo) {
                v = zero3();
                ok2 = calc_pen_depth(slow1, s, R, oA, I, oB, v, tA, tB);
            }
        } else {
            ok2 = calc_pen_depth(slow1, s, R, oA, I, oB, v, tA, tB);
        }
        if (ok2) {
            v3 tn = tB - tA;
            float l2 = len2(tn);
            if (l2 <= kEps * kEps) {
                tn = v;
                l2 = len2(v);
            }
            if (l2 > kEps * kEps) {
                tn = tn / sqrtf(l2);
                const float d2 = -len(tA - tB);
                if (!valid || d2 < distance_) {
                    distance_ = d2;
                    pA = tA;
                    pB = tB;
                    nB = tn;
                    valid = true;
                }
            }
        } else if (len2(v) > 0.f) {
            const float d2 = len(tA - tB) - margin;
            if (!valid || d2 < distance_) {
                distance_ = d2;
                pA = tA;
                pB = tB;
                pA -= v * mA;
                pB += v * mB;
                nB = bt_normalize(v, s.ar);  // normalInB.normalize() (btGjkPairDetector.cpp:914)
                valid = true;
            }
        }
    }
    if (!(valid && ((distance_ < 0) || (distance_ * distance_ < max2)))) return false;
    // normal-direction fix from the two AABB centres (btGjkPairDetector.cpp:930-949)
    v3 posA, posB;
    {
        const v3 hwm = s.impl + v3{s.margin, s.margin, s.margin};
        const v3 ext = v3{dot(hwm, v3{fabsf(R.r0.x), fabsf(R.r0.y), fabsf(R.r0.z)}),
                          dot(hwm, v3{fabsf(R.r1.x), fabsf(R.r1.y), fabsf(R.r1.z)}),
                          dot(hwm, v3{fabsf(R.r2.x), fabsf(R.r2.y), fabsf(R.r2.z)})};
        const v3 mn = oA - ext, mx = oA + ext;
        posA = (mx + mn) * 0.5f;
        v3 tmn, tmx;
#pragma unroll
        for (int i = 0; i < 3; i++) {
            v3 vec = zero3();
            set_comp(vec, i, 1.f);
            v3 t = xf(I, oB, tri_nm(s, vmul(vec, I)));
            set_comp(tmx, i, comp(t, i) + 0.f);
            set_comp(vec, i, -1.f);
            t = xf(I, oB, tri_nm(s, vmul(vec, I)));
            set_comp(tmn, i, comp(t, i) - 0.f);
        }
        posB = (tmn + tmx) * 0.5f;
    }
    if (dot(posA - posB, nB) < 0.f) nB *= -1.f;
    normal = nB;
    point = pB + po;
    depth = distance_;
    return true;
}

}  // namespace gjk
}  // namespace rl
