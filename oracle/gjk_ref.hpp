// gjk_ref.hpp -- ORACLE (test infrastructure only; never linked into the product).
//
// Scalar restatement of the narrowphase Bullet 3.24 runs for a car hitbox (btBoxShape, the compound's
// one child) against one arena-mesh triangle, as RocketSim configures it:
//   btConvexConcaveCollisionAlgorithm.cpp:71-138   processTriangle: exact triangle-vs-AABB test, the
//                                                  triangle-normal early out (both sides), then the
//                                                  convex-convex algorithm with body 0 = box, 1 = triangle
//   btConvexConvexAlgorithm.cpp:268-513           box and triangle are polyhedral but carry no polyhedral
//                                                  features (RocketSim never calls initializePolyhedralFeatures)
//                                                  and no perturbation iterations: one GJK query
//   btGjkPairDetector.cpp:686-959                  getClosestPointsNonVirtual (margins, degenerate catch,
//                                                  penetration fallback, normal-direction fix)
//   btVoronoiSimplexSolver.cpp:34-577 (+ .h:24-154) the simplex sub-distance solver
//   btGjkEpaPenetrationDepthSolver.cpp:22-79       nine guess directions
//   btGjkEpa2.cpp:37-1017                          GJK / EPA / Penetration / Distance (float constants)
//   btConvexShape.cpp:126-193, btBoxShape.h/.cpp, btTriangleShape.h:60-70, btConvexInternalShape.cpp:23-66
//                                                  support mappings and AABBs
// Shapes: the box's implicit half extents (btBoxShape: half extents - 0.04, then setSafeMargin) and its
// margin; the triangle's margin is the concave mesh's, 0 (btConcaveShape.cpp:21); the mesh transform is
// the identity (Arena.cpp:1052, _AddStaticCollisionShape at the origin).
// Every operation keeps Bullet's scalar order (rsim_math.hpp conventions; vector / s = v * (1 / s)).
// The product's restatement is reinforcement-learning_amd/csrc/gjk.hpp (independent code, index-based
// EPA lists in per-lane scratch); the two agree bit for bit.
#pragma once
#include <cfloat>
#include <cstdint>

#include "rsim_math.hpp"

namespace orc {
namespace gjk {

constexpr float LARGE = 1e18f;       // BT_LARGE_FLOAT (btScalar.h:317)
constexpr float REL_ERROR2 = 1.0e-6f;  // btGjkPairDetector.cpp:35
constexpr float EQUAL_VERTEX_THRESHOLD = 0.0001f;  // VORONOI_DEFAULT_EQUAL_VERTEX_THRESHOLD
// diagnostics (this thread): EPA runs, EPA iterations, max iterations of one run, max faces taken
inline thread_local uint64_t epa_stats[4] = {0, 0, 0, 0};
// diagnostics (this thread): btGjkEpa2 GJK evaluations, their iterations, most iterations of one
inline thread_local uint64_t gjk2_stats[3] = {0, 0, 0};

struct Tr {  // btTransform: basis rows + origin
    M b;
    V o;
};
inline V xf(const Tr& t, V x) { return t.b * x + t.o; }
inline M ident() { return M::ident(); }
// btMatrix3x3::transposeTimes (btMatrix3x3.h:1147-1157): this^T * m
inline M transpose_times(const M& a, const M& m) {
    M r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r.r[i][j] = a.r[0][i] * m.r[0][j] + a.r[1][i] * m.r[1][j] + a.r[2][i] * m.r[2][j];
    return r;
}
inline int max_axis(V d) { return d.x < d.y ? (d.y < d.z ? 2 : 1) : (d.x < d.z ? 2 : 0); }  // btVector3::maxAxis
inline V normalize(V a) { return bt_normalize(a); }  // btVector3::normalize (rsim_math.hpp: rsqrtss + Newton in the x86 builds)

struct Shapes {
    V impl;       // box half extents without margin (m_implicitShapeDimensions)
    float margin;  // box margin
    V tri[3];     // triangle (mesh space = world)
};
// localGetSupportVertexWithoutMarginNonVirtual (btConvexShape.cpp:126-162)
inline V box_nm(const Shapes& s, V d) {
    return V(d.x >= 0 ? s.impl.x : -s.impl.x, d.y >= 0 ? s.impl.y : -s.impl.y, d.z >= 0 ? s.impl.z : -s.impl.z);
}
inline V tri_nm(const Shapes& s, V d) {
    V dots(dot(d, s.tri[0]), dot(d, s.tri[1]), dot(d, s.tri[2]));
    return s.tri[max_axis(dots)];
}
// localGetSupportVertexNonVirtual (btConvexShape.cpp:186-193): normalized direction + margin
inline V unit_dir(V d) {
    if (len2(d) < SIMD_EPSILON * SIMD_EPSILON) d = V(-1.f, -1.f, -1.f);
    return normalize(d);
}
inline V box_m(const Shapes& s, V d) {
    V n = unit_dir(d);
    return box_nm(s, n) + s.margin * n;
}
inline V tri_m(const Shapes& s, V d) {
    V n = unit_dir(d);
    return tri_nm(s, n) + 0.f * n;
}

// ------------------------------------------------------------------ btVoronoiSimplexSolver
struct Voronoi {
    V W[4], P[4], Q[4];
    int n = 0;
    V lastW, cP1, cP2, cV;
    bool used[4];
    float bc[4];
    bool degenerate;
    bool needs_update = true, valid_closest = false;

    void bc_reset() {
        degenerate = false;
        bc[0] = bc[1] = bc[2] = bc[3] = 0.f;
        used[0] = used[1] = used[2] = used[3] = false;
    }
    bool bc_valid() const { return bc[0] >= 0.f && bc[1] >= 0.f && bc[2] >= 0.f && bc[3] >= 0.f; }
    void reset() {
        valid_closest = false;
        n = 0;
        needs_update = true;
        lastW = V(LARGE, LARGE, LARGE);
        bc_reset();
    }
    void remove(int i) {
        n--;
        W[i] = W[n];
        P[i] = P[n];
        Q[i] = Q[n];
    }
    void reduce() {
        if (n >= 4 && !used[3]) remove(3);
        if (n >= 3 && !used[2]) remove(2);
        if (n >= 2 && !used[1]) remove(1);
        if (n >= 1 && !used[0]) remove(0);
    }
    void add(V w, V p, V q) {
        lastW = w;
        needs_update = true;
        W[n] = w;
        P[n] = p;
        Q[n] = q;
        n++;
    }
    // closestPtPointTriangle (btVoronoiSimplexSolver.cpp:313-408) with p = origin; out: point, used, bary
    static void closest_tri(V a, V b, V c, V& pt, bool u[3], float w[3]) {
        const V p(0.f, 0.f, 0.f);
        u[0] = u[1] = u[2] = false;
        V ab = b - a, ac = c - a, ap = p - a;
        float d1 = dot(ab, ap), d2 = dot(ac, ap);
        if (d1 <= 0.f && d2 <= 0.f) {
            pt = a; u[0] = true; w[0] = 1; w[1] = 0; w[2] = 0;
            return;
        }
        V bp = p - b;
        float d3 = dot(ab, bp), d4 = dot(ac, bp);
        if (d3 >= 0.f && d4 <= d3) {
            pt = b; u[1] = true; w[0] = 0; w[1] = 1; w[2] = 0;
            return;
        }
        float vc = d1 * d4 - d3 * d2;
        if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) {
            float v = d1 / (d1 - d3);
            pt = a + v * ab; u[0] = u[1] = true; w[0] = 1 - v; w[1] = v; w[2] = 0;
            return;
        }
        V cp = p - c;
        float d5 = dot(ab, cp), d6 = dot(ac, cp);
        if (d6 >= 0.f && d5 <= d6) {
            pt = c; u[2] = true; w[0] = 0; w[1] = 0; w[2] = 1;
            return;
        }
        float vb = d5 * d2 - d1 * d6;
        if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) {
            float ww = d2 / (d2 - d6);
            pt = a + ww * ac; u[0] = u[2] = true; w[0] = 1 - ww; w[1] = 0; w[2] = ww;
            return;
        }
        float va = d3 * d6 - d5 * d4;
        if (va <= 0.f && (d4 - d3) >= 0.f && (d5 - d6) >= 0.f) {
            float ww = (d4 - d3) / ((d4 - d3) + (d5 - d6));
            pt = b + ww * (c - b); u[1] = u[2] = true; w[0] = 0; w[1] = 1 - ww; w[2] = ww;
            return;
        }
        float denom = 1.f / (va + vb + vc);
        float v = vb * denom, ww = vc * denom;
        pt = a + ab * v + ac * ww;
        u[0] = u[1] = u[2] = true;
        w[0] = 1 - v - ww; w[1] = v; w[2] = ww;
    }
    // pointOutsideOfPlane (cpp:411-435), p = origin
    static int outside(V a, V b, V c, V d) {
        const V p(0.f, 0.f, 0.f);
        V nrm = cross(b - a, c - a);
        float signp = dot(p - a, nrm), signd = dot(d - a, nrm);
        if (signd * signd < (1e-4f * 1e-4f)) return -1;
        return signp * signd < 0.f;
    }
    // closestPtPointTetrahedron (cpp:437-577): writes bc / used / degenerate; returns "has separation"
    bool closest_tetra(V a, V b, V c, V d, V& best_pt) {
        best_pt = V(0.f, 0.f, 0.f);
        used[0] = used[1] = used[2] = used[3] = true;
        int oABC = outside(a, b, c, d), oACD = outside(a, c, d, b), oADB = outside(a, d, b, c), oBDC = outside(b, d, c, a);
        if (oABC < 0 || oACD < 0 || oADB < 0 || oBDC < 0) {
            degenerate = true;
            return false;
        }
        if (!oABC && !oACD && !oADB && !oBDC) return false;
        float best = FLT_MAX;
        V q;
        bool u[3];
        float w[3];
        const V origin(0.f, 0.f, 0.f);
        if (oABC) {
            closest_tri(a, b, c, q, u, w);
            float sq = dot(q - origin, q - origin);
            if (sq < best) {
                best = sq; best_pt = q;
                used[0] = u[0]; used[1] = u[1]; used[2] = u[2]; used[3] = false;
                bc[0] = w[0]; bc[1] = w[1]; bc[2] = w[2]; bc[3] = 0;
            }
        }
        if (oACD) {
            closest_tri(a, c, d, q, u, w);
            float sq = dot(q - origin, q - origin);
            if (sq < best) {
                best = sq; best_pt = q;
                used[0] = u[0]; used[1] = false; used[2] = u[1]; used[3] = u[2];
                bc[0] = w[0]; bc[1] = 0; bc[2] = w[1]; bc[3] = w[2];
            }
        }
        if (oADB) {
            closest_tri(a, d, b, q, u, w);
            float sq = dot(q - origin, q - origin);
            if (sq < best) {
                best = sq; best_pt = q;
                used[0] = u[0]; used[1] = u[2]; used[2] = false; used[3] = u[1];
                bc[0] = w[0]; bc[1] = w[2]; bc[2] = 0; bc[3] = w[1];
            }
        }
        if (oBDC) {
            closest_tri(b, d, c, q, u, w);
            float sq = dot(q - origin, q - origin);
            if (sq < best) {
                best = sq; best_pt = q;
                used[0] = false; used[1] = u[0]; used[2] = u[2]; used[3] = u[1];
                bc[0] = 0; bc[1] = w[0]; bc[2] = w[2]; bc[3] = w[1];
            }
        }
        return true;
    }
    // updateClosestVectorAndPoints (cpp:81-233)
    bool update() {
        if (needs_update) {
            bc_reset();
            needs_update = false;
            switch (n) {
                case 0: valid_closest = false; break;
                case 1:
                    cP1 = P[0];
                    cP2 = Q[0];
                    cV = cP1 - cP2;
                    bc_reset();
                    bc[0] = 1.f;
                    valid_closest = bc_valid();
                    break;
                case 2: {
                    const V from = W[0], to = W[1];
                    V diff = V(0.f, 0.f, 0.f) - from;
                    V v = to - from;
                    float t = dot(v, diff);
                    if (t > 0) {
                        float dotVV = dot(v, v);
                        if (t < dotVV) {
                            t /= dotVV;
                            diff -= t * v;
                            used[0] = used[1] = true;
                        } else {
                            t = 1;
                            diff -= v;
                            used[1] = true;
                        }
                    } else {
                        t = 0;
                        used[0] = true;
                    }
                    bc[0] = 1 - t; bc[1] = t; bc[2] = 0; bc[3] = 0;
                    cP1 = P[0] + t * (P[1] - P[0]);
                    cP2 = Q[0] + t * (Q[1] - Q[0]);
                    cV = cP1 - cP2;
                    reduce();
                    valid_closest = bc_valid();
                    break;
                }
                case 3: {
                    V pt;
                    bool u[3];
                    float w[3];
                    closest_tri(W[0], W[1], W[2], pt, u, w);
                    used[0] = u[0]; used[1] = u[1]; used[2] = u[2];
                    bc[0] = w[0]; bc[1] = w[1]; bc[2] = w[2]; bc[3] = 0;
                    cP1 = P[0] * bc[0] + P[1] * bc[1] + P[2] * bc[2];
                    cP2 = Q[0] * bc[0] + Q[1] * bc[1] + Q[2] * bc[2];
                    cV = cP1 - cP2;
                    reduce();
                    valid_closest = bc_valid();
                    break;
                }
                case 4: {
                    V pt;
                    bool sep = closest_tetra(W[0], W[1], W[2], W[3], pt);
                    if (sep) {
                        cP1 = P[0] * bc[0] + P[1] * bc[1] + P[2] * bc[2] + P[3] * bc[3];
                        cP2 = Q[0] * bc[0] + Q[1] * bc[1] + Q[2] * bc[2] + Q[3] * bc[3];
                        cV = cP1 - cP2;
                        reduce();
                    } else {
                        if (degenerate) {
                            valid_closest = false;
                        } else {
                            valid_closest = true;
                            cV = V(0.f, 0.f, 0.f);
                        }
                        break;
                    }
                    valid_closest = bc_valid();
                    break;
                }
                default: valid_closest = false;
            }
        }
        return valid_closest;
    }
    bool closest(V& v) {
        bool ok = update();
        v = cV;
        return ok;
    }
    bool in_simplex(V w) const {
        bool found = false;
        for (int i = 0; i < n; i++)
            if (len2(w - W[i]) <= EQUAL_VERTEX_THRESHOLD) {  // W[i].distance2(w) = (w - W[i]).length2()
                found = true;
                break;
            }
        if (w.x == lastW.x && w.y == lastW.y && w.z == lastW.z) return true;
        return found;
    }
    void compute_points(V& p1, V& p2) {
        update();
        p1 = cP1;
        p2 = cP2;
    }
};

// ------------------------------------------------------------------ btGjkEpa2 (gjkepa2_impl)
constexpr int GJK_MAX_ITERATIONS = 128;
constexpr float GJK_ACCURACY = 0.0001f, GJK_MIN_DISTANCE = 0.0001f, GJK_DUPLICATED_EPS = 0.0001f;
constexpr int EPA_MAX_VERTICES = 128, EPA_MAX_FACES = 256, EPA_MAX_ITERATIONS = 255;
constexpr float EPA_ACCURACY = 0.0001f, EPA_PLANE_EPS = 0.00001f;

struct Mink {  // MinkowskiDiff (cpp:80-150)
    const Shapes* s;
    M toshape1;
    Tr toshape0;
    bool margins;
    V support0(V d) const { return margins ? box_m(*s, d) : box_nm(*s, d); }
    V support1(V d) const {
        V dd = toshape1 * d;
        return xf(toshape0, margins ? tri_m(*s, dd) : tri_nm(*s, dd));
    }
    V support(V d) const { return support0(d) - support1(-d); }
    V support(V d, int index) const { return index ? support1(d) : support0(d); }
};

struct SV {
    V d, w;
};
struct Simplex {
    SV* c[4];
    float p[4];
    unsigned rank;
};

struct GJK {
    Mink shape;
    V ray;
    float distance = 0;
    Simplex simplices[2];
    SV store[4];
    SV* freev[4];
    unsigned nfree = 0, current = 0;
    Simplex* simplex = nullptr;
    int status = 2;  // Valid 0, Inside 1, Failed 2

    void getsupport(V d, SV& sv) const {
        sv.d = d / len(d);
        sv.w = shape.support(sv.d);
    }
    void removevertice(Simplex& s) { freev[nfree++] = s.c[--s.rank]; }
    void appendvertice(Simplex& s, V v) {
        s.p[s.rank] = 0;
        s.c[s.rank] = freev[--nfree];
        getsupport(v, *s.c[s.rank++]);
    }
    static float det(V a, V b, V c) {
        return (a.y * b.z * c.x + a.z * b.x * c.y - a.x * b.z * c.y - a.y * b.x * c.z + a.x * b.y * c.z - a.z * b.y * c.x);
    }
    static float project2(V a, V b, float* w, unsigned& m) {
        const V d = b - a;
        const float l = len2(d);
        if (l > 0.f) {
            const float t(l > 0 ? -dot(a, d) / l : 0);
            if (t >= 1) {
                w[0] = 0; w[1] = 1; m = 2;
                return len2(b);
            } else if (t <= 0) {
                w[0] = 1; w[1] = 0; m = 1;
                return len2(a);
            } else {
                w[0] = 1 - (w[1] = t);
                m = 3;
                return len2(a + d * t);
            }
        }
        return -1;
    }
    static float project3(V a, V b, V c, float* w, unsigned& m) {
        static const unsigned imd3[] = {1, 2, 0};
        const V* vt[] = {&a, &b, &c};
        const V dl[] = {a - b, b - c, c - a};
        const V n = cross(dl[0], dl[1]);
        const float l = len2(n);
        if (l > 0.f) {
            float mindist = -1;
            float subw[2] = {0.f, 0.f};
            unsigned subm = 0;
            for (unsigned i = 0; i < 3; ++i) {
                if (dot(*vt[i], cross(dl[i], n)) > 0) {
                    const unsigned j = imd3[i];
                    const float subd = project2(*vt[i], *vt[j], subw, subm);
                    if ((mindist < 0) || (subd < mindist)) {
                        mindist = subd;
                        m = ((subm & 1) ? 1u << i : 0) + ((subm & 2) ? 1u << j : 0);
                        w[i] = subw[0];
                        w[j] = subw[1];
                        w[imd3[j]] = 0;
                    }
                }
            }
            if (mindist < 0) {
                const float d = dot(a, n);
                const float s = std::sqrt(l);
                const V p = n * (d / l);
                mindist = len2(p);
                m = 7;
                w[0] = len(cross(dl[1], b - p)) / s;
                w[1] = len(cross(dl[2], c - p)) / s;
                w[2] = 1 - (w[0] + w[1]);
            }
            return mindist;
        }
        return -1;
    }
    static float project4(V a, V b, V c, V d, float* w, unsigned& m) {
        static const unsigned imd3[] = {1, 2, 0};
        const V* vt[] = {&a, &b, &c, &d};
        const V dl[] = {a - d, b - d, c - d};
        const float vl = det(dl[0], dl[1], dl[2]);
        const bool ng = (vl * dot(a, cross(b - c, a - b))) <= 0;
        if (ng && (std::fabs(vl) > 0.f)) {
            float mindist = -1;
            float subw[3] = {0.f, 0.f, 0.f};
            unsigned subm = 0;
            for (unsigned i = 0; i < 3; ++i) {
                const unsigned j = imd3[i];
                const float s = vl * dot(d, cross(dl[i], dl[j]));
                if (s > 0) {
                    const float subd = project3(*vt[i], *vt[j], d, subw, subm);
                    if ((mindist < 0) || (subd < mindist)) {
                        mindist = subd;
                        m = (subm & 1 ? 1u << i : 0) + (subm & 2 ? 1u << j : 0) + (subm & 4 ? 8 : 0);
                        w[i] = subw[0];
                        w[j] = subw[1];
                        w[imd3[j]] = 0;
                        w[3] = subw[2];
                    }
                }
            }
            if (mindist < 0) {
                mindist = 0;
                m = 15;
                w[0] = det(c, b, d) / vl;
                w[1] = det(a, c, d) / vl;
                w[2] = det(b, a, d) / vl;
                w[3] = 1 - (w[0] + w[1] + w[2]);
            }
            return mindist;
        }
        return -1;
    }
    // GJK::Evaluate (cpp:201-337)
    int evaluate(const Mink& sh, V guess) {
        unsigned iterations = 0;
        float sqdist = 0, alpha = 0;
        V lastw[4];
        unsigned clastw = 0;
        freev[0] = &store[0]; freev[1] = &store[1]; freev[2] = &store[2]; freev[3] = &store[3];
        nfree = 4;
        current = 0;
        status = 0;
        shape = sh;
        distance = 0;
        simplices[0].rank = 0;
        ray = guess;
        const float sqrl = len2(ray);
        appendvertice(simplices[0], sqrl > 0 ? -ray : V(1, 0, 0));
        simplices[0].p[0] = 1;
        ray = simplices[0].c[0]->w;
        sqdist = sqrl;
        lastw[0] = lastw[1] = lastw[2] = lastw[3] = ray;
        do {
            const unsigned next = 1 - current;
            Simplex& cs = simplices[current];
            Simplex& ns = simplices[next];
            const float rl = len(ray);
            if (rl < GJK_MIN_DISTANCE) {
                status = 1;
                break;
            }
            appendvertice(cs, -ray);
            const V w = cs.c[cs.rank - 1]->w;
            bool found = false;
            for (unsigned i = 0; i < 4; ++i)
                if (len2(w - lastw[i]) < GJK_DUPLICATED_EPS) {
                    found = true;
                    break;
                }
            if (found) {
                removevertice(simplices[current]);
                break;
            } else {
                lastw[clastw = (clastw + 1) & 3] = w;
            }
            const float omega = dot(ray, w) / rl;
            alpha = omega > alpha ? omega : alpha;  // btMax(omega, alpha)
            if (((rl - alpha) - (GJK_ACCURACY * rl)) <= 0) {
                removevertice(simplices[current]);
                break;
            }
            float weights[4];
            unsigned mask = 0;
            switch (cs.rank) {
                case 2: sqdist = project2(cs.c[0]->w, cs.c[1]->w, weights, mask); break;
                case 3: sqdist = project3(cs.c[0]->w, cs.c[1]->w, cs.c[2]->w, weights, mask); break;
                case 4: sqdist = project4(cs.c[0]->w, cs.c[1]->w, cs.c[2]->w, cs.c[3]->w, weights, mask); break;
            }
            if (sqdist >= 0) {
                ns.rank = 0;
                ray = V(0, 0, 0);
                current = next;
                for (unsigned i = 0, ni = cs.rank; i < ni; ++i) {
                    if (mask & (1u << i)) {
                        ns.c[ns.rank] = cs.c[i];
                        ns.p[ns.rank++] = weights[i];
                        ray += cs.c[i]->w * weights[i];
                    } else {
                        freev[nfree++] = cs.c[i];
                    }
                }
                if (mask == 15) status = 1;
            } else {
                removevertice(simplices[current]);
                break;
            }
            status = ((++iterations) < (unsigned)GJK_MAX_ITERATIONS) ? status : 2;
        } while (status == 0);
        simplex = &simplices[current];
        gjk2_stats[0]++;
        gjk2_stats[1] += iterations;
        if (iterations > gjk2_stats[2]) gjk2_stats[2] = iterations;
        if (status == 0) distance = len(ray);
        else if (status == 1) distance = 0;
        return status;
    }
    // GJK::EncloseOrigin (cpp:338-402)
    bool enclose_origin() {
        switch (simplex->rank) {
            case 1:
                for (unsigned i = 0; i < 3; ++i) {
                    V axis(0, 0, 0);
                    axis[i] = 1;
                    appendvertice(*simplex, axis);
                    if (enclose_origin()) return true;
                    removevertice(*simplex);
                    appendvertice(*simplex, -axis);
                    if (enclose_origin()) return true;
                    removevertice(*simplex);
                }
                break;
            case 2: {
                const V d = simplex->c[1]->w - simplex->c[0]->w;
                for (unsigned i = 0; i < 3; ++i) {
                    V axis(0, 0, 0);
                    axis[i] = 1;
                    const V p = cross(d, axis);
                    if (len2(p) > 0) {
                        appendvertice(*simplex, p);
                        if (enclose_origin()) return true;
                        removevertice(*simplex);
                        appendvertice(*simplex, -p);
                        if (enclose_origin()) return true;
                        removevertice(*simplex);
                    }
                }
            } break;
            case 3: {
                const V n = cross(simplex->c[1]->w - simplex->c[0]->w, simplex->c[2]->w - simplex->c[0]->w);
                if (len2(n) > 0) {
                    appendvertice(*simplex, n);
                    if (enclose_origin()) return true;
                    removevertice(*simplex);
                    appendvertice(*simplex, -n);
                    if (enclose_origin()) return true;
                    removevertice(*simplex);
                }
            } break;
            case 4:
                if (std::fabs(det(simplex->c[0]->w - simplex->c[3]->w, simplex->c[1]->w - simplex->c[3]->w,
                                  simplex->c[2]->w - simplex->c[3]->w)) > 0)
                    return true;
                break;
        }
        return false;
    }
};

struct EPA {
    struct Face {
        V n;
        float d;
        SV* c[3];
        Face* f[3];
        Face* l[2];
        uint8_t e[3];
        uint8_t pass;
    };
    struct List {
        Face* root = nullptr;
        unsigned count = 0;
    };
    struct Horizon {
        Face* cf = nullptr;
        Face* ff = nullptr;
        unsigned nf = 0;
    };
    // Valid 0, Touching 1, Degenerated 2, NonConvex 3, InvalidHull 4, OutOfFaces 5, OutOfVertices 6,
    // AccuraryReached 7, FallBack 8, Failed 9
    int status = 9;
    Simplex result;
    V normal;
    float depth = 0;
    SV sv_store[EPA_MAX_VERTICES];
    Face fc_store[EPA_MAX_FACES];
    unsigned nextsv = 0;
    List hull, stock;

    static void bind(Face* fa, unsigned ea, Face* fb, unsigned eb) {
        fa->e[ea] = (uint8_t)eb;
        fa->f[ea] = fb;
        fb->e[eb] = (uint8_t)ea;
        fb->f[eb] = fa;
    }
    static void append(List& list, Face* face) {
        face->l[0] = nullptr;
        face->l[1] = list.root;
        if (list.root) list.root->l[0] = face;
        list.root = face;
        ++list.count;
    }
    static void remove(List& list, Face* face) {
        if (face->l[1]) face->l[1]->l[0] = face->l[0];
        if (face->l[0]) face->l[0]->l[1] = face->l[1];
        if (face == list.root) list.root = face->l[1];
        --list.count;
    }
    EPA() {
        status = 9;
        normal = V(0, 0, 0);
        depth = 0;
        nextsv = 0;
        for (unsigned i = 0; i < (unsigned)EPA_MAX_FACES; ++i) append(stock, &fc_store[EPA_MAX_FACES - i - 1]);
    }
    bool getedgedist(Face* face, SV* a, SV* b, float& dist) {
        const V ba = b->w - a->w;
        const V n_ab = cross(ba, face->n);
        const float a_dot_nab = dot(a->w, n_ab);
        if (a_dot_nab < 0) {
            const float ba_l2 = len2(ba);
            const float a_dot_ba = dot(a->w, ba);
            const float b_dot_ba = dot(b->w, ba);
            if (a_dot_ba > 0) {
                dist = len(a->w);
            } else if (b_dot_ba < 0) {
                dist = len(b->w);
            } else {
                const float a_dot_b = dot(a->w, b->w);
                const float q = (len2(a->w) * len2(b->w) - a_dot_b * a_dot_b) / ba_l2;
                dist = std::sqrt(q > 0.f ? q : 0.f);  // btMax(q, 0)
            }
            return true;
        }
        return false;
    }
    Face* newface(SV* a, SV* b, SV* c, bool forced) {
        if (stock.root) {
            Face* face = stock.root;
            remove(stock, face);
            append(hull, face);
            face->pass = 0;
            face->c[0] = a;
            face->c[1] = b;
            face->c[2] = c;
            face->n = cross(b->w - a->w, c->w - a->w);
            const float l = len(face->n);
            const bool v = l > EPA_ACCURACY;
            if (v) {
                if (!(getedgedist(face, a, b, face->d) || getedgedist(face, b, c, face->d) || getedgedist(face, c, a, face->d)))
                    face->d = dot(a->w, face->n) / l;
                face->n = face->n / l;
                if (forced || (face->d >= -EPA_PLANE_EPS)) return face;
                status = 3;
            } else {
                status = 2;
            }
            remove(hull, face);
            append(stock, face);
            return nullptr;
        }
        status = stock.root ? 6 : 5;
        return nullptr;
    }
    Face* findbest() {
        Face* minf = hull.root;
        float mind = minf->d * minf->d;
        for (Face* f = minf->l[1]; f; f = f->l[1]) {
            const float sqd = f->d * f->d;
            if (sqd < mind) {
                minf = f;
                mind = sqd;
            }
        }
        return minf;
    }
    bool expand(unsigned pass, SV* w, Face* f, unsigned e, Horizon& horizon) {
        static const unsigned i1m3[] = {1, 2, 0};
        static const unsigned i2m3[] = {2, 0, 1};
        if (f->pass != pass) {
            const unsigned e1 = i1m3[e];
            if ((dot(f->n, w->w) - f->d) < -EPA_PLANE_EPS) {
                Face* nf = newface(f->c[e1], f->c[e], w, false);
                if (nf) {
                    bind(nf, 0, f, e);
                    if (horizon.cf)
                        bind(horizon.cf, 1, nf, 2);
                    else
                        horizon.ff = nf;
                    horizon.cf = nf;
                    ++horizon.nf;
                    return true;
                }
            } else {
                const unsigned e2 = i2m3[e];
                f->pass = (uint8_t)pass;
                if (expand(pass, w, f->f[e1], f->e[e1], horizon) && expand(pass, w, f->f[e2], f->e[e2], horizon)) {
                    remove(hull, f);
                    append(stock, f);
                    return true;
                }
            }
        }
        return false;
    }
    // EPA::Evaluate (cpp:648-768)
    int evaluate(GJK& gjk, V guess) {
        Simplex& simplex = *gjk.simplex;
        if ((simplex.rank > 1) && gjk.enclose_origin()) {
            while (hull.root) {
                Face* f = hull.root;
                remove(hull, f);
                append(stock, f);
            }
            status = 0;
            nextsv = 0;
            if (GJK::det(simplex.c[0]->w - simplex.c[3]->w, simplex.c[1]->w - simplex.c[3]->w,
                         simplex.c[2]->w - simplex.c[3]->w) < 0) {
                std::swap(simplex.c[0], simplex.c[1]);
                std::swap(simplex.p[0], simplex.p[1]);
            }
            Face* tetra[] = {newface(simplex.c[0], simplex.c[1], simplex.c[2], true),
                             newface(simplex.c[1], simplex.c[0], simplex.c[3], true),
                             newface(simplex.c[2], simplex.c[1], simplex.c[3], true),
                             newface(simplex.c[0], simplex.c[2], simplex.c[3], true)};
            if (hull.count == 4) {
                Face* best = findbest();
                Face outer = *best;
                unsigned pass = 0;
                unsigned iterations = 0;
                bind(tetra[0], 0, tetra[1], 0);
                bind(tetra[0], 1, tetra[2], 0);
                bind(tetra[0], 2, tetra[3], 0);
                bind(tetra[1], 1, tetra[3], 2);
                bind(tetra[1], 2, tetra[2], 1);
                bind(tetra[2], 2, tetra[3], 1);
                status = 0;
                for (; iterations < (unsigned)EPA_MAX_ITERATIONS; ++iterations) {
                    if (nextsv < (unsigned)EPA_MAX_VERTICES) {
                        Horizon horizon;
                        SV* w = &sv_store[nextsv++];
                        bool valid = true;
                        best->pass = (uint8_t)(++pass);
                        gjk.getsupport(best->n, *w);
                        const float wdist = dot(best->n, w->w) - best->d;
                        if (wdist > EPA_ACCURACY) {
                            for (unsigned j = 0; (j < 3) && valid; ++j)
                                valid &= expand(pass, w, best->f[j], best->e[j], horizon);
                            if (valid && (horizon.nf >= 3)) {
                                bind(horizon.cf, 1, horizon.ff, 2);
                                remove(hull, best);
                                append(stock, best);
                                best = findbest();
                                outer = *best;
                            } else {
                                status = 4;
                                break;
                            }
                        } else {
                            status = 7;
                            break;
                        }
                    } else {
                        status = 6;
                        break;
                    }
                }
                epa_stats[0]++;
                epa_stats[1] += iterations;
                if (iterations > epa_stats[2]) epa_stats[2] = iterations;
                {
                    uint64_t taken = 0;
                    for (Face* f = stock.root; f; f = f->l[1]) taken++;
                    taken = EPA_MAX_FACES - taken;
                    if (taken > epa_stats[3]) epa_stats[3] = taken;
                }
                const V projection = outer.n * outer.d;
                normal = outer.n;
                depth = outer.d;
                result.rank = 3;
                result.c[0] = outer.c[0];
                result.c[1] = outer.c[1];
                result.c[2] = outer.c[2];
                result.p[0] = len(cross(outer.c[1]->w - projection, outer.c[2]->w - projection));
                result.p[1] = len(cross(outer.c[2]->w - projection, outer.c[0]->w - projection));
                result.p[2] = len(cross(outer.c[0]->w - projection, outer.c[1]->w - projection));
                const float sum = result.p[0] + result.p[1] + result.p[2];
                result.p[0] /= sum;
                result.p[1] /= sum;
                result.p[2] /= sum;
                return status;
            }
        }
        status = 8;
        normal = -guess;
        const float nl = len(normal);
        if (nl > 0)
            normal = normal / nl;
        else
            normal = V(1, 0, 0);
        depth = 0;
        result.rank = 1;
        result.c[0] = simplex.c[0];
        result.p[0] = 1;
        return status;
    }
};

// Initialize (cpp:904-920)
inline Mink make_shape(const Shapes& s, const Tr& t0, const Tr& t1, bool margins) {
    Mink m;
    m.s = &s;
    m.toshape1 = transpose_times(t1.b, t0.b);
    // btTransform::inverseTimes (btTransform.h:218-223)
    m.toshape0 = Tr{transpose_times(t0.b, t1.b), vmul(t1.o - t0.o, t0.b)};
    m.margins = margins;
    return m;
}
struct Results {
    V w0, w1, normal;
    float distance;
};
// btGjkEpaSolver2::Penetration (cpp:973-1017), usemargins = true
inline bool penetration(const Shapes& s, const Tr& t0, const Tr& t1, V guess, Results& r) {
    Mink shape = make_shape(s, t0, t1, true);
    r.w0 = r.w1 = V(0, 0, 0);
    GJK* gjk = new GJK();
    bool ok = false;
    int gs = gjk->evaluate(shape, -guess);
    if (gs == 1) {
        EPA* epa = new EPA();
        int es = epa->evaluate(*gjk, -guess);
        if (es != 9) {
            V w0(0, 0, 0);
            for (unsigned i = 0; i < epa->result.rank; ++i) w0 += shape.support(epa->result.c[i]->d, 0) * epa->result.p[i];
            r.w0 = xf(t0, w0);
            r.w1 = xf(t0, w0 - epa->normal * epa->depth);
            r.normal = -epa->normal;
            r.distance = -epa->depth;
            ok = true;
        }
        delete epa;
    }
    delete gjk;
    return ok;
}
// btGjkEpaSolver2::Distance (cpp:937-970)
inline bool distance(const Shapes& s, const Tr& t0, const Tr& t1, V guess, Results& r) {
    Mink shape = make_shape(s, t0, t1, false);
    r.w0 = r.w1 = V(0, 0, 0);
    GJK gjk;
    int gs = gjk.evaluate(shape, guess);
    if (gs == 0) {
        V w0(0, 0, 0), w1(0, 0, 0);
        for (unsigned i = 0; i < gjk.simplex->rank; ++i) {
            const float p = gjk.simplex->p[i];
            w0 += shape.support(gjk.simplex->c[i]->d, 0) * p;
            w1 += shape.support(-gjk.simplex->c[i]->d, 1) * p;
        }
        r.w0 = xf(t0, w0);
        r.w1 = xf(t0, w1);
        r.normal = w0 - w1;
        r.distance = len(r.normal);
        r.normal = r.normal / (r.distance > GJK_MIN_DISTANCE ? r.distance : 1);
        return true;
    }
    return false;
}
// btGjkEpaPenetrationDepthSolver::calcPenDepth (cpp:22-79)
inline bool calc_pen_depth(const Shapes& s, const Tr& tA, const Tr& tB, V& v, V& wA, V& wB) {
    const V guesses[] = {safe_normalized(tB.o - tA.o), safe_normalized(tA.o - tB.o), V(0, 0, 1), V(0, 1, 0), V(1, 0, 0),
                         V(1, 1, 0), V(1, 1, 1), V(0, 1, 1), V(1, 0, 1)};
    for (const V& g : guesses) {
        Results r;
        if (penetration(s, tA, tB, g, r)) {
            wA = r.w0; wB = r.w1; v = r.normal;
            return true;
        } else if (distance(s, tA, tB, g, r)) {
            wA = r.w0; wB = r.w1; v = r.normal;
            return false;
        }
    }
    wA = wB = v = V(0, 0, 0);
    return false;
}

// One box-triangle query as btConvexTriangleCallback::processTriangle + btConvexConvexAlgorithm run it,
// minus the AABB test (the caller's).  Box world transform: basis R, origin c (the hitbox child's);
// cbt = the pair manifold's contact breaking threshold.  Returns true when Bullet calls
// btManifoldResult::addContactPoint(normal, point, depth) (before that function's own depth test).
// Counters: evals[0] += GJK queries, evals[1] += penetration-solver calls (diagnostics only).
inline bool box_triangle(const M& R, V c, const Shapes& s, float cbt, V& normal, V& point, float& depth,
                         uint64_t* evals = nullptr) {
    // early out along the triangle normal, both sides (btConvexConcaveCollisionAlgorithm.cpp:101-136)
    {
        const V half = s.impl + V(s.margin, s.margin, s.margin);  // btBoxShape::localGetSupportingVertex
        const M inv = inverse(R);  // btMatrix3x3::inverse (rsim_math.hpp)
        V tn = normalize(cross(s.tri[1] - s.tri[0], s.tri[2] - s.tri[0]));
        for (int side = 0; side < 2; side++) {
            V ld = inv * tn;
            V lp(ld.x >= 0 ? half.x : -half.x, ld.y >= 0 ? half.y : -half.y, ld.z >= 0 ? half.z : -half.z);
            V wp = R * lp + c;
            float dist = dot(tn, s.tri[0]) - dot(tn, wp);
            if (dist > cbt) return false;
            tn = tn * -1.f;
        }
    }
    if (evals) evals[0]++;
    // btConvexConvexAlgorithm: maximum distance (cpp:316)
    float maxd = s.margin + 0.f + cbt;
    const float max2 = maxd * maxd;
    // getClosestPointsNonVirtual (btGjkPairDetector.cpp:686-959); transform B = identity
    const M I = ident();
    const V po = (c + V(0.f, 0.f, 0.f)) * 0.5f;
    const Tr lA{R, c - po}, lB{I, V(0.f, 0.f, 0.f) - po};
    const float mA = s.margin, mB = 0.f;
    float distance = 0.f;
    V nB(0.f, 0.f, 0.f), pA, pB;
    V v(0.f, 1.f, 0.f);
    bool valid = false, check = false;
    int degen = 0, iter = 0;
    float sqd = LARGE, delta = 0.f;
    const float margin = mA + mB;
    Voronoi vs;
    vs.reset();
    while (true) {
        V sa = vmul(-v, R), sb = vmul(v, I);
        V pin = box_nm(s, sa), qin = tri_nm(s, sb);
        V pw = xf(lA, pin), qw = xf(lB, qin);
        V w = pw - qw;
        delta = dot(v, w);
        if ((delta > 0.f) && (delta * delta > sqd * max2)) {
            degen = 10; check = true;
            break;
        }
        if (vs.in_simplex(w)) {
            degen = 1; check = true;
            break;
        }
        float f0 = sqd - delta, f1 = sqd * REL_ERROR2;
        if (f0 <= f1) {
            degen = f0 <= 0.f ? 2 : 11;
            check = true;
            break;
        }
        vs.add(w, pw, qw);
        V nv;
        if (!vs.closest(nv)) {
            degen = 3; check = true;
            break;
        }
        if (len2(nv) < REL_ERROR2) {
            v = nv; degen = 6; check = true;
            break;
        }
        float prev = sqd;
        sqd = len2(nv);
        if (prev - sqd <= SIMD_EPSILON * prev) {
            check = true; degen = 12;
            break;
        }
        v = nv;
        if (iter++ > 1000) break;
        if (vs.n == 4) {
            degen = 13;
            break;
        }
    }
    if (check) {
        vs.compute_points(pA, pB);
        nB = v;
        float l2 = len2(v);
        if ((double)l2 < 0.0001) degen = 5;  // double literals in the reference
        if (l2 > SIMD_EPSILON * SIMD_EPSILON) {
            float rlen = 1.f / std::sqrt(l2);
            nB *= rlen;
            float sq = std::sqrt(sqd);
            pA -= v * (mA / sq);
            pB += v * (mB / sq);
            distance = (1.f / rlen) - margin;
            valid = true;
        }
    }
    bool catch_degen = degen && ((double)(distance + margin) < 0.01);
    if (!valid || catch_degen) {
        if (evals) evals[1]++;
        V tA, tB;
        v = V(0.f, 0.f, 0.f);
        bool ok2 = calc_pen_depth(s, lA, lB, v, tA, tB);
        if (ok2) {
            V tn = tB - tA;
            float l2 = len2(tn);
            if (l2 <= SIMD_EPSILON * SIMD_EPSILON) {
                tn = v;
                l2 = len2(v);
            }
            if (l2 > SIMD_EPSILON * SIMD_EPSILON) {
                tn = tn / std::sqrt(l2);
                float d2 = -len(tA - tB);
                if (!valid || d2 < distance) {
                    distance = d2; pA = tA; pB = tB; nB = tn; valid = true;
                }
            }
        } else if (len2(v) > 0.f) {
            float d2 = len(tA - tB) - margin;
            if (!valid || d2 < distance) {
                distance = d2; pA = tA; pB = tB;
                pA -= v * mA;
                pB += v * mB;
                nB = normalize(v);
                valid = true;
            }
        }
    }
    if (!(valid && ((distance < 0) || (distance * distance < max2)))) return false;
    // m_fixContactNormalDirection: AABB centres of both shapes in the local transforms (cpp:930-949)
    V posA, posB;
    {
        const V hwm = s.impl + V(s.margin, s.margin, s.margin);  // btTransformAabb (btAabbUtil2.h:172-180)
        V ext(dot(hwm, V(std::fabs(R.r[0].x), std::fabs(R.r[0].y), std::fabs(R.r[0].z))),
              dot(hwm, V(std::fabs(R.r[1].x), std::fabs(R.r[1].y), std::fabs(R.r[1].z))),
              dot(hwm, V(std::fabs(R.r[2].x), std::fabs(R.r[2].y), std::fabs(R.r[2].z))));
        V mn = lA.o - ext, mx = lA.o + ext;
        posA = (mx + mn) * 0.5f;
        V tmn, tmx;  // btConvexInternalShape::getAabbSlow, margin 0 (btConvexInternalShape.cpp:23-42)
        for (int i = 0; i < 3; i++) {
            V vec(0.f, 0.f, 0.f);
            vec[i] = 1.f;
            V t = xf(lB, tri_nm(s, vmul(vec, lB.b)));
            tmx[i] = t[i] + 0.f;
            vec[i] = -1.f;
            t = xf(lB, tri_nm(s, vmul(vec, lB.b)));
            tmn[i] = t[i] - 0.f;
        }
        posB = (tmn + tmx) * 0.5f;
    }
    if (dot(posA - posB, nB) < 0.f) nB *= -1.f;
    normal = nB;
    point = pB + po;
    depth = distance;
    return true;
}


// ------------------------------------------------------------------ btSubsimplexConvexCast (wheel rays)
// The convex branch of btCollisionWorld::rayTestSingleInternal (btCollisionWorld.cpp:277-310): the ray's point
// shape (btSphereShape(0), margin 0, identity basis) cast from `from` to `to` against a resting convex body with
// basis R and origin o by btSubsimplexConvexCast::calcTimeOfImpact (btSubSimplexConvexCast.cpp:30-153;
// btConvexCast.h:25-29: 32 iterations, epsilon 0.0001, allowed penetration 0).  sphere_r > 0: btSphereShape
// (margin = radius, btSphereShape.cpp:37-48); otherwise btBoxShape with half extents h including its margin
// (btBoxShape.h:47-56).  True when Bullet reports the cast (fraction, normal = n.normalized()).
inline V sphere_support(V d, float radius) {
    V vn;
    if (len2(d) < FLT_EPSILON * FLT_EPSILON)
        vn = bt_normalize(V(-1.f, -1.f, -1.f));  // the static invalidVecNorm
    else
        vn = bt_normalize(d);
    return vn * radius;  // getMargin() * vecnorm
}
inline V box_support(V d, V h) {  // btFsels(d, h, -h)
    return V(d.x >= 0.f ? h.x : -h.x, d.y >= 0.f ? h.y : -h.y, d.z >= 0.f ? h.z : -h.z);
}
inline V interp3(V v0, V v1, float rt) {  // btVector3::setInterpolate3
    const float s = 1.f - rt;
    return V(s * v0.x + rt * v1.x, s * v0.y + rt * v1.y, s * v0.z + rt * v1.z);
}
inline bool ray_convex_cast(V from, V to, float sphere_r, V h, const M& R, V o, float& frac, V& normal) {
    const M I = M::ident();
    auto supA = [&](V d, V org) { return I * sphere_support(vmul(d, I), 0.f) + org; };
    auto supB = [&](V d, V org) {
        const V l = vmul(d, R);
        return R * (sphere_r > 0.f ? sphere_support(l, sphere_r) : box_support(l, h)) + org;
    };
    Voronoi vs;
    vs.reset();
    const V linA = to - from, linB = o - o;
    float lambda = 0.f;
    V iA = from, iB = o;
    const V r = linA - linB;
    V sa = supA(-r, iA), sb = supB(r, iB);
    V v = sa - sb;
    int max_iter = 32;
    V n(0.f, 0.f, 0.f);
    float dist2 = len2(v);
    while ((dist2 > 0.0001f) && max_iter--) {
        sa = supA(-v, iA);
        sb = supB(v, iB);
        V w = sa - sb;
        const float vdw = dot(v, w);
        if (lambda > 1.f) return false;
        if (vdw > 0.f) {
            const float vdr = dot(v, r);
            if (vdr >= -(FLT_EPSILON * FLT_EPSILON)) return false;
            lambda = lambda - vdw / vdr;
            iA = interp3(from, to, lambda);
            iB = interp3(o, o, lambda);
            w = sa - sb;
            n = v;
        }
        if (!vs.in_simplex(w)) vs.add(w, sa, sb);
        if (vs.closest(v))
            dist2 = len2(v);
        else
            dist2 = 0.f;
    }
    frac = lambda;
    normal = len2(n) >= FLT_EPSILON * FLT_EPSILON ? bt_normalize(n) : V(0.f, 0.f, 0.f);
    if (dot(normal, r) >= -0.f) return false;
    return true;
}
}  // namespace gjk
}  // namespace orc
