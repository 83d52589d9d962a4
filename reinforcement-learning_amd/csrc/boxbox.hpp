// boxbox.hpp -- car hitbox vs car hitbox on the device, as Bullet 3.24 runs it for RocketSim:
// btBoxBoxCollisionAlgorithm (BulletCollision/CollisionDispatch/btBoxBoxCollisionAlgorithm.cpp:44-71) ->
// btBoxBoxDetector::getClosestPoints (btBoxBoxDetector.cpp:730-767) -> ODE's dBoxBox2 (:267-728):
// separating-axis test over the 15 axes (face axes strict, edge axes scaled with the 1.05 fudge factor),
// then one edge-edge point (dLineClosestApproach :84-108) or the incident face clipped to the reference
// face (intersectRectQuad2 :116-175), penetrating points kept and culled to four by their angle about
// the polygon centroid (cullPoints2 :187-265).  Each point reaches btManifoldResult::addContactPoint
// (-normal, point, -depth).  Boxes are given as (centre, basis rows, half extents with margin); the
// matrices are read in ODE's element order (R(i, j) = row i, column j).  btAtan2 = rs_atan2f.
// The CPU oracle's independent restatement is oracle/boxbox_ref.hpp; the two agree bit for bit.
#pragma once
#include "dmath.hpp"

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

namespace rl {
namespace boxbox {

constexpr float kPi = 3.14159265f;  // M__PI of btBoxBoxDetector.cpp

DEV float el(const m3& m, int i, int j) { return comp(row(m, i), j); }
// column dot column (dDOT44 of two dMatrix3 columns), column . vector (dDOT14 / dDOT41)
DEV float colcol(const m3& a, int i, const m3& b, int j) {
    return el(a, 0, i) * el(b, 0, j) + el(a, 1, i) * el(b, 1, j) + el(a, 2, i) * el(b, 2, j);
}
DEV float vcol(v3 v, const m3& a, int j) { return v.x * el(a, 0, j) + v.y * el(a, 1, j) + v.z * el(a, 2, j); }
DEV float colv(const m3& a, int j, v3 v) { return el(a, 0, j) * v.x + el(a, 1, j) * v.y + el(a, 2, j) * v.z; }
DEV v3 colvec(const m3& a, int j) { return v3{el(a, 0, j), el(a, 1, j), el(a, 2, j)}; }

// intersectRectQuad2: the quad p (4 points) clipped against |x| < h0, |y| < h1; ret holds <= 8 points
DEV int clip_rect_quad(float h0, float h1, const float p[8], float ret[16]) {
    float bufA[16], bufB[16];
    for (int k = 0; k < 8; k++) bufA[k] = p[k];
    float* q = bufA;
    float* r = bufB;
    int nq = 4, nr = 0;
    bool stop = false;
    for (int dir = 0; dir <= 1 && !stop; dir++) {
        const float h = dir ? h1 : h0;
        for (int sign = -1; sign <= 1 && !stop; sign += 2) {
            nr = 0;
            for (int i = 0; i < nq && !stop; i++) {
                const float* pq = q + 2 * i;
                const float* nx = (i + 1 < nq) ? pq + 2 : q;
                const bool in = sign * pq[dir] < h;
                if (in) {
                    r[2 * nr] = pq[0];
                    r[2 * nr + 1] = pq[1];
                    nr++;
                    if (nr & 8) stop = true;
                }
                if (!stop && (in ^ (sign * nx[dir] < h))) {
                    r[2 * nr + 1 - dir] = pq[1 - dir] + (nx[1 - dir] - pq[1 - dir]) / (nx[dir] - pq[dir]) * (sign * h - pq[dir]);
                    r[2 * nr + dir] = sign * h;
                    nr++;
                    if (nr & 8) stop = true;
                }
            }
            float* t = q;  // the chopped polygon becomes the input of the next chop
            q = r;
            r = t;
            nq = nr;
        }
    }
    for (int k = 0; k < 2 * nr; k++) ret[k] = q[k];
    return nr;
}

// cullPoints2 with m = 4 out of n (5..8) points; i0 = the deepest point
DEV void cull_points(int n, const float p[16], int i0, int iret[4]) {
    float a = 0, cx = 0, cy = 0, q;
    for (int i = 0; i < n - 1; i++) {
        q = p[i * 2] * p[i * 2 + 3] - p[i * 2 + 2] * p[i * 2 + 1];
        a += q;
        cx += q * (p[i * 2] + p[i * 2 + 2]);
        cy += q * (p[i * 2 + 1] + p[i * 2 + 3]);
    }
    q = p[n * 2 - 2] * p[1] - p[0] * p[n * 2 - 1];
    a = fabsf(a + q) > kEps ? 1.f / (3.0f * (a + q)) : 1e18f;
    cx = a * (cx + q * (p[n * 2 - 2] + p[0]));
    cy = a * (cy + q * (p[n * 2 - 1] + p[1]));
    float ang[8];
    unsigned avail = 0;
    for (int i = 0; i < n; i++) {
        ang[i] = rs_atan2f(p[i * 2 + 1] - cy, p[i * 2] - cx);
        avail |= 1u << i;
    }
    avail &= ~(1u << i0);
    iret[0] = i0;
    for (int j = 1; j < 4; j++) {
        float t = float(j) * (2 * kPi / 4) + ang[i0];
        if (t > kPi) t -= 2 * kPi;
        float best = 1e9f;
        int pick = i0;
        for (int i = 0; i < n; i++) {
            if (avail & (1u << i)) {
                float d = fabsf(ang[i] - t);
                if (d > kPi) d = 2 * kPi - d;
                if (d < best) {
                    best = d;
                    pick = i;
                }
            }
        }
        avail &= ~(1u << pick);
        iret[j] = pick;
    }
}

// dBoxBox2 (maxc = 4) of box 1 (c1, R1, half h1) and box 2; emit(normal on B, point, depth) per point
template <typename Emit>
DEV int box_box(v3 c1, const m3& R1, v3 h1, v3 c2, const m3& R2, v3 h2, Emit&& emit) {
    const v3 A = (h1 * 2.f) * 0.5f, B = (h2 * 2.f) * 0.5f;  // side = 2 h (getClosestPoints), side * 0.5
    const v3 p = c2 - c1;
    const v3 pp = v3{colv(R1, 0, p), colv(R1, 1, p), colv(R1, 2, p)};
    const float R11 = colcol(R1, 0, R2, 0), R12 = colcol(R1, 0, R2, 1), R13 = colcol(R1, 0, R2, 2);
    const float R21 = colcol(R1, 1, R2, 0), R22 = colcol(R1, 1, R2, 1), R23 = colcol(R1, 1, R2, 2);
    const float R31 = colcol(R1, 2, R2, 0), R32 = colcol(R1, 2, R2, 1), R33 = colcol(R1, 2, R2, 2);
    float Q11 = fabsf(R11), Q12 = fabsf(R12), Q13 = fabsf(R13), Q21 = fabsf(R21), Q22 = fabsf(R22), Q23 = fabsf(R23),
          Q31 = fabsf(R31), Q32 = fabsf(R32), Q33 = fabsf(R33);
    float s = -3.40282346638528859812e+38f;
    int code = 0, nbox = 0, ncol = 0;  // face normal = column ncol of box nbox (1 / 2); 0 = normalC
    bool inv = false;
    v3 normalC = zero3();
    // face axes: separated when |e1| - e2 > 0
#define RL_FACE(e1v, e2v, box, col_, cc)   \
    {                                      \
        const float e1 = (e1v);            \
        const float s2 = fabsf(e1) - (e2v); \
        if (s2 > 0) return 0;              \
        if (s2 > s) {                      \
            s = s2;                        \
            nbox = box;                    \
            ncol = col_;                   \
            inv = e1 < 0;                  \
            code = cc;                     \
        }                                  \
    }
    RL_FACE(pp.x, (A.x + B.x * Q11 + B.y * Q12 + B.z * Q13), 1, 0, 1)
    RL_FACE(pp.y, (A.y + B.x * Q21 + B.y * Q22 + B.z * Q23), 1, 1, 2)
    RL_FACE(pp.z, (A.z + B.x * Q31 + B.y * Q32 + B.z * Q33), 1, 2, 3)
    RL_FACE(colv(R2, 0, p), (A.x * Q11 + A.y * Q21 + A.z * Q31 + B.x), 2, 0, 4)
    RL_FACE(colv(R2, 1, p), (A.x * Q12 + A.y * Q22 + A.z * Q32 + B.y), 2, 1, 5)
    RL_FACE(colv(R2, 2, p), (A.x * Q13 + A.y * Q23 + A.z * Q33 + B.z), 2, 2, 6)
#undef RL_FACE
    const float f2 = 1.0e-5f;
    Q11 += f2; Q12 += f2; Q13 += f2; Q21 += f2; Q22 += f2; Q23 += f2; Q31 += f2; Q32 += f2; Q33 += f2;
    // edge axes u_i x v_j, normal (n1, n2, n3) in box-1 coordinates
#define RL_EDGE(e1v, e2v, n1, n2, n3, cc)                           \
    {                                                               \
        const float e1 = (e1v);                                     \
        float s2 = fabsf(e1) - (e2v);                               \
        if (s2 > kEps) return 0;                                    \
        const float l = sqrtf((n1) * (n1) + (n2) * (n2) + (n3) * (n3)); \
        if (l > kEps) {                                             \
            s2 /= l;                                                \
            if (s2 * 1.05f > s) {                                   \
                s = s2;                                             \
                nbox = 0;                                           \
                normalC = v3{(n1) / l, (n2) / l, (n3) / l};         \
                inv = e1 < 0;                                       \
                code = cc;                                          \
            }                                                       \
        }                                                           \
    }
    const float z = 0.f;
    RL_EDGE(pp.z * R21 - pp.y * R31, (A.y * Q31 + A.z * Q21 + B.y * Q13 + B.z * Q12), z, -R31, R21, 7)
    RL_EDGE(pp.z * R22 - pp.y * R32, (A.y * Q32 + A.z * Q22 + B.x * Q13 + B.z * Q11), z, -R32, R22, 8)
    RL_EDGE(pp.z * R23 - pp.y * R33, (A.y * Q33 + A.z * Q23 + B.x * Q12 + B.y * Q11), z, -R33, R23, 9)
    RL_EDGE(pp.x * R31 - pp.z * R11, (A.x * Q31 + A.z * Q11 + B.y * Q23 + B.z * Q22), R31, z, -R11, 10)
    RL_EDGE(pp.x * R32 - pp.z * R12, (A.x * Q32 + A.z * Q12 + B.x * Q23 + B.z * Q21), R32, z, -R12, 11)
    RL_EDGE(pp.x * R33 - pp.z * R13, (A.x * Q33 + A.z * Q13 + B.x * Q22 + B.y * Q21), R33, z, -R13, 12)
    RL_EDGE(pp.y * R11 - pp.x * R21, (A.x * Q21 + A.y * Q11 + B.y * Q33 + B.z * Q32), -R21, R11, z, 13)
    RL_EDGE(pp.y * R12 - pp.x * R22, (A.x * Q22 + A.y * Q12 + B.x * Q33 + B.z * Q31), -R22, R12, z, 14)
    RL_EDGE(pp.y * R13 - pp.x * R23, (A.x * Q23 + A.y * Q13 + B.x * Q32 + B.y * Q31), -R23, R13, z, 15)
#undef RL_EDGE
    if (!code) return 0;
    v3 normal = nbox == 1 ? colvec(R1, ncol) : (nbox == 2 ? colvec(R2, ncol) : R1 * normalC);
    if (inv) normal = -normal;
    const float depth = -s;
    const v3 nout = -normal;
    if (code > 6) {  // edge-edge: one point on box 2's edge
        v3 pa = c1, pb = c2;
        for (int j = 0; j < 3; j++) {
            const float sg = vcol(normal, R1, j) > 0 ? 1.0f : -1.0f;
            const float aj = comp(A, j);
            pa = v3{pa.x + sg * aj * el(R1, 0, j), pa.y + sg * aj * el(R1, 1, j), pa.z + sg * aj * el(R1, 2, j)};
        }
        for (int j = 0; j < 3; j++) {
            const float sg = vcol(normal, R2, j) > 0 ? -1.0f : 1.0f;
            const float bj = comp(B, j);
            pb = v3{pb.x + sg * bj * el(R2, 0, j), pb.y + sg * bj * el(R2, 1, j), pb.z + sg * bj * el(R2, 2, j)};
        }
        const v3 ua = colvec(R1, (code - 7) / 3), ub = colvec(R2, (code - 7) % 3);
        // dLineClosestApproach
        const v3 d = pb - pa;
        const float uaub = dot(ua, ub), q1 = dot(ua, d), q2 = -dot(ub, d);
        float den = 1 - uaub * uaub, beta = 0.f;
        if (!(den <= 0.0001f)) {
            den = 1.f / den;
            beta = (uaub * q1 + q2) * den;
        }
        pb = v3{pb.x + ub.x * beta, pb.y + ub.y * beta, pb.z + ub.z * beta};
        emit(nout, pb, -depth);
        return 1;
    }
    // face - something: reference face on box a, incident face on box b
    const bool one = code <= 3;
    const m3 Ra = one ? R1 : R2, Rb = one ? R2 : R1;
    const v3 pa = one ? c1 : c2, pb = one ? c2 : c1, Sa = one ? A : B, Sb = one ? B : A;
    const v3 normal2 = one ? normal : -normal;
    const v3 nr = v3{colv(Rb, 0, normal2), colv(Rb, 1, normal2), colv(Rb, 2, normal2)};
    const float an0 = fabsf(nr.x), an1 = fabsf(nr.y), an2 = fabsf(nr.z);
    int lanr, a1, a2;
    if (an1 > an0) {
        if (an1 > an2) { a1 = 0; lanr = 1; a2 = 2; }
        else { a1 = 0; a2 = 1; lanr = 2; }
    } else {
        if (an0 > an2) { lanr = 0; a1 = 1; a2 = 2; }
        else { a1 = 0; a2 = 1; lanr = 2; }
    }
    const float sbl = comp(Sb, lanr);
    v3 center;
    if (comp(nr, lanr) < 0)
        center = v3{pb.x - pa.x + sbl * el(Rb, 0, lanr), pb.y - pa.y + sbl * el(Rb, 1, lanr), pb.z - pa.z + sbl * el(Rb, 2, lanr)};
    else
        center = v3{pb.x - pa.x - sbl * el(Rb, 0, lanr), pb.y - pa.y - sbl * el(Rb, 1, lanr), pb.z - pa.z - sbl * el(Rb, 2, lanr)};
    const int codeN = one ? code - 1 : code - 4;
    const int code1 = codeN == 0 ? 1 : 0, code2 = codeN == 2 ? 1 : 2;
    const float c1_ = vcol(center, Ra, code1), c2_ = vcol(center, Ra, code2);
    float m11 = colcol(Ra, code1, Rb, a1), m12 = colcol(Ra, code1, Rb, a2), m21 = colcol(Ra, code2, Rb, a1),
          m22 = colcol(Ra, code2, Rb, a2);
    float quad[8];
    {
        const float k1 = m11 * comp(Sb, a1), k2 = m21 * comp(Sb, a1), k3 = m12 * comp(Sb, a2), k4 = m22 * comp(Sb, a2);
        quad[0] = c1_ - k1 - k3;
        quad[1] = c2_ - k2 - k4;
        quad[2] = c1_ - k1 + k3;
        quad[3] = c2_ - k2 + k4;
        quad[4] = c1_ + k1 + k3;
        quad[5] = c2_ + k2 + k4;
        quad[6] = c1_ + k1 - k3;
        quad[7] = c2_ + k2 - k4;
    }
    float ret[16];
    const int n = clip_rect_quad(comp(Sa, code1), comp(Sa, code2), quad, ret);
    if (n < 1) return 0;
    float pt[24], dep[8];
    const float det1 = 1.f / (m11 * m22 - m12 * m21);
    m11 *= det1;
    m12 *= det1;
    m21 *= det1;
    m22 *= det1;
    const v3 ca1 = colvec(Rb, a1), ca2 = colvec(Rb, a2);
    const float saN = comp(Sa, codeN);
    int cnum = 0;
    for (int j = 0; j < n; j++) {
        const float x = ret[j * 2] - c1_, y = ret[j * 2 + 1] - c2_;
        const float k1 = m22 * x - m12 * y;
        const float k2 = -m21 * x + m11 * y;
        const v3 q = v3{center.x + k1 * ca1.x + k2 * ca2.x, center.y + k1 * ca1.y + k2 * ca2.y, center.z + k1 * ca1.z + k2 * ca2.z};
        const float dp = saN - dot(normal2, q);
        pt[cnum * 3] = q.x;
        pt[cnum * 3 + 1] = q.y;
        pt[cnum * 3 + 2] = q.z;
        dep[cnum] = dp;
        if (dp >= 0) {
            ret[cnum * 2] = ret[j * 2];
            ret[cnum * 2 + 1] = ret[j * 2 + 1];
            cnum++;
        }
    }
    if (cnum < 1) return 0;
    int iret[4] = {0, 1, 2, 3};
    int m = cnum;
    if (cnum > 4) {
        int i1 = 0;
        float md = dep[0];
        for (int i = 1; i < cnum; i++)
            if (dep[i] > md) {
                md = dep[i];
                i1 = i;
            }
        cull_points(cnum, ret, i1, iret);
        m = 4;
    }
    for (int j = 0; j < m; j++) {
        const int k = iret[j];
        v3 w = v3{pt[k * 3] + pa.x, pt[k * 3 + 1] + pa.y, pt[k * 3 + 2] + pa.z};
        if (code >= 4) w = w - normal * dep[k];
        emit(nout, w, -dep[k]);
    }
    return m;
}

}  // namespace boxbox
}  // namespace rl
