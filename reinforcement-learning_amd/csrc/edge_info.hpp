// edge_info.hpp -- Bullet's internal-edge utility on the arena meshes (RocketSim loads every mesh with
// it: RocketSim.cpp:166-170 btGenerateInternalEdgeInfo; Arena.cpp:275-279 btAdjustInternalEdgeContacts
// at the end of the contact-added callback).
//
//   edge_info_object   btGenerateInternalEdgeInfo + btConnectivityProcessor
//                      (BT/BulletCollision/CollisionDispatch/btInternalEdgeUtility.cpp:50-358): per
//                      triangle, the angle to the neighbour across each edge and the convex / swap flags
//   adjust_edge_contact btAdjustInternalEdgeContacts (:414-798) with btClampNormal (:385-412) and
//                      btNearestPointInLineSegment (:362-383), normalAdjustFlags = 0
//
// Host (mesh.hip, at env-set create) and device (the contact commit, env_contacts.hpp) share this code;
// the CPU oracle restates it independently (oracle/rsim_ref.cpp).  The meshes are static at the
// identity transform, so the triangle-local frame is the world frame (the reference's basis products
// with the identity are skipped: they only turn a -0 component into +0).
// `ar` is the set's arithmetic mode (include/rlgpu_arith.h): every btVector3::normalize here is
// bt_normalize (rsqrtss + Newton in the x86 modes), the quaternion products and setRotation follow dmath.hpp.
// Neighbour order: a triangle's edge info is written by every neighbour that shares the edge, the last
// one winning; neighbours are visited in the quantized BVH's traversal order, as the reference does
// (mesh.hip mesh_edge_info; it matters on edges shared by three or more triangles).
#pragma once
#include "dmath.hpp"

namespace rl {

// btTriangleInfoMap defaults (btTriangleInfoMap.h:60-70)
constexpr float kEdgeConvexEps = 0.f;
constexpr float kEdgePlanarEps = 0.0001f;
constexpr float kEdgeEqualVertex = 0.0001f * 0.0001f;
constexpr float kEdgeDistance = 0.1f;
constexpr float kEdge2Pi = 2.0f * kPi;  // SIMD_2_PI: the "no neighbour" angle and the max-angle threshold

// btTriangleInfo flags (btTriangleInfoMap.h:24-29); kEdgeHasInfo marks a triangle with an info record
enum : int {
    kV0V1Convex = 1,
    kV1V2Convex = 2,
    kV2V0Convex = 4,
    kV0V1Swap = 8,
    kV1V2Swap = 16,
    kV2V0Swap = 32,
    kEdgeHasInfo = 1 << 30,
};

struct EdgeInfo {  // btTriangleInfo
    float a01, a12, a20;  // m_edgeV0V1Angle, m_edgeV1V2Angle, m_edgeV2V0Angle
    int flags;
};

// btGetAngle: atan2(swing . edgeA, swing . normalA)
HD float edge_angle(v3 edge_a, v3 normal_a, v3 normal_b) { return rs_atan2f(dot(normal_b, edge_a), dot(normal_b, normal_a)); }
// btTriangleShape::calcNormal
HD v3 tri_normal(v3 v0, v3 v1, v3 v2, int ar) { return bt_normalize(cross(v1 - v0, v2 - v0), ar); }
// quatRotate(rotation, v) = (rotation * v) *= rotation.inverse() (btQuaternion.h:916-927; the quaternion x
// vector product has the same operation order in both paths, the quaternion product is qmul's)
HD v3 quat_rotate(quat q, v3 w, int ar) {
    const quat p{q.w * w.x + q.y * w.z - q.z * w.y, q.w * w.y + q.z * w.x - q.x * w.z, q.w * w.z + q.x * w.y - q.y * w.x,
                 -q.x * w.x - q.y * w.y - q.z * w.z};
    const quat r = qmul(p, quat{-q.x, -q.y, -q.z, q.w}, ar);
    return v3{r.x, r.y, r.z};
}

// btConnectivityProcessor::processTriangle for triangle A (va) and a neighbour candidate B (vb)
HD void edge_connect(const v3 (&va)[3], const v3 (&vb)[3], EdgeInfo& info, int ar) {
    if (len2(cross(vb[1] - vb[0], vb[2] - vb[0])) < kEdgeEqualVertex) return;  // degenerate B
    if (len2(cross(va[1] - va[0], va[2] - va[0])) < kEdgeEqualVertex) return;  // degenerate A
    int numshared = 0;
    int sa[3] = {-1, -1, -1}, sb[3] = {-1, -1, -1};
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) {
            if (len2(va[i] - vb[j]) < kEdgeEqualVertex) {
                sa[numshared] = i;
                sb[numshared] = j;
                numshared++;
                if (numshared >= 3) return;  // degenerate (duplicate triangle)
            }
        }
        if (numshared >= 3) return;
    }
    if (numshared != 2) return;
    if (sa[0] == 0 && sa[1] == 2) {  // edge order V2V0, not V0V2
        sa[0] = 2;
        sa[1] = 0;
        const int tmp = sb[1];
        sb[1] = sb[0];
        sb[0] = tmp;
    }
    if (!(info.flags & kEdgeHasInfo)) info = EdgeInfo{kEdge2Pi, kEdge2Pi, kEdge2Pi, kEdgeHasInfo};
    const int sumverts = sa[0] + sa[1];
    const int other_a = 3 - sumverts;
    v3 edge = va[sa[1]] - va[sa[0]];
    const int other_b = 3 - (sb[0] + sb[1]);
    const v3 normal_a = tri_normal(va[0], va[1], va[2], ar);
    const v3 normal_b = tri_normal(vb[sb[1]], vb[sb[0]], vb[other_b], ar);
    edge = bt_normalize(edge, ar);
    v3 cross_a = bt_normalize(cross(edge, normal_a), ar);
    if (dot(cross_a, va[other_a] - va[sa[0]]) < 0.f) cross_a *= -1.f;
    v3 cross_b = bt_normalize(cross(edge, normal_b), ar);
    if (dot(cross_b, vb[other_b] - vb[sb[0]]) < 0.f) cross_b *= -1.f;
    float corrected = 0.f;
    bool convex = false;
    v3 calc_edge = cross(cross_a, cross_b);
    if (!(len2(calc_edge) < kEdgePlanarEps)) {
        calc_edge = bt_normalize(calc_edge, ar);
        const v3 calc_normal_a = bt_normalize(cross(calc_edge, cross_a), ar);
        const float angle2 = edge_angle(calc_normal_a, cross_a, cross_b);
        const float ang4 = kPi - angle2;
        convex = dot(normal_a, cross_b) < 0.f;
        corrected = convex ? ang4 : -ang4;
    }
    // the edge between the two shared vertices of A: sum 1 = V0V1, 2 = V2V0, 3 = V1V2
    const v3 e = sumverts == 1 ? va[0] - va[1] : (sumverts == 2 ? va[2] - va[0] : va[1] - va[2]);
    const v3 computed = quat_rotate(quat_axis_angle(e, -corrected), normal_a, ar);
    const bool swap = dot(computed, normal_b) < 0.f;
    if (sumverts == 1) {
        if (swap) info.flags |= kV0V1Swap;
        info.a01 = -corrected;
        if (convex) info.flags |= kV0V1Convex;
    } else if (sumverts == 2) {
        if (swap) info.flags |= kV2V0Swap;
        info.a20 = -corrected;
        if (convex) info.flags |= kV2V0Convex;
    } else if (sumverts == 3) {
        if (swap) info.flags |= kV1V2Swap;
        info.a12 = -corrected;
        if (convex) info.flags |= kV1V2Convex;
    }
}

// btNearestPointInLineSegment
HD v3 nearest_on_segment(v3 p, v3 l0, v3 l1) {
    const v3 d = l1 - l0;
    if (fuzzy_zero(d)) return l0;
    float t = dot(p - l0, d) / dot(d, d);
    if (t < 0.f) t = 0.f;
    else if (t > 1.f) t = 1.f;
    return l0 + d * t;
}

// btClampNormal: rotate the contact normal back inside the edge's angle range
HD bool clamp_normal(v3 edge, v3 tri_n, v3 n_local, float corrected, v3& clamped, int ar) {
    const v3 edge_cross = bt_normalize(cross(edge, tri_n), ar);
    const float cur = edge_angle(edge_cross, tri_n, n_local);
    if (corrected < 0.f) {
        if (cur < corrected) {
            clamped = mat_from_quat(quat_axis_angle(edge, corrected - cur), ar) * n_local;
            return true;
        }
    }
    if (corrected >= 0.f) {
        if (cur > corrected) {
            clamped = mat_from_quat(quat_axis_angle(edge, corrected - cur), ar) * n_local;
            return true;
        }
    }
    return false;
}

// one edge block of btAdjustInternalEdgeContacts (edge = v_i - v_j of the reference's block): n_unit is
// the normalized contact normal of the back-facing test, n_clamp the normal the block clamps (the
// reference clamps the normalized one in the V0V1 block and re-reads the raw contact normal in the
// other two)
HD void edge_block(v3 edge, float angle, int convex_flag, int swap_flag, int flags, v3 tri_n, v3 n_unit, v3 n_clamp,
                   v3& normal, v3& point_b, v3 point_a, float dist, int& concave_hits, int ar) {
    if (angle == 0.f) {
        concave_hits++;
        return;
    }
    const float swap_factor = (flags & convex_flag) ? 1.f : -1.f;
    const v3 n_a = tri_n * swap_factor;
    v3 computed = quat_rotate(quat_axis_angle(edge, angle), tri_n, ar);
    if (flags & swap_flag) computed *= -1.f;
    const v3 n_b = computed * swap_factor;
    const bool back_facing = dot(n_unit, n_a) < kEdgeConvexEps && dot(n_unit, n_b) < kEdgeConvexEps;
    if (back_facing) {
        concave_hits++;
        return;
    }
    v3 clamped;
    if (clamp_normal(edge, tri_n * swap_factor, n_clamp, angle, clamped, ar) && dot(clamped, tri_n) > 0.f) {
        normal = clamped;
        point_b = point_a - normal * dist;  // reproject along the new normal
    }
}

// btAdjustInternalEdgeContacts for a contact on mesh triangle (v0, v1, v2) with info `info`: the
// contact's normal on the mesh and its point on the mesh are updated in place (point_a = the point
// on the other body, dist = the contact distance, both unchanged).  At most one edge block acts,
// the one of the nearest edge that has a neighbour.
HD void adjust_edge_contact(v3 v0, v3 v1, v3 v2, const EdgeInfo& info, v3& normal, v3& point_b, v3 point_a, float dist,
                            int ar) {
    if (!(info.flags & kEdgeHasInfo)) return;
    const v3 tri_n = tri_normal(v0, v1, v2, ar);
    const v3 contact = point_b;
    const v3 n_unit = bt_normalize(normal, ar);
    int best = -1;
    float best_d = 1e18f;  // BT_LARGE_FLOAT
    if (fabsf(info.a01) < kEdge2Pi) {
        const float d = len(contact - nearest_on_segment(contact, v0, v1));
        if (d < best_d) {
            best = 0;
            best_d = d;
        }
    }
    if (fabsf(info.a12) < kEdge2Pi) {
        const float d = len(contact - nearest_on_segment(contact, v1, v2));
        if (d < best_d) {
            best = 1;
            best_d = d;
        }
    }
    if (fabsf(info.a20) < kEdge2Pi) {
        const float d = len(contact - nearest_on_segment(contact, v2, v0));
        if (d < best_d) {
            best = 2;
            best_d = d;
        }
    }
    bool near_edge = false;
    int concave_hits = 0;
    if (fabsf(info.a01) < kEdge2Pi && len(contact - nearest_on_segment(contact, v0, v1)) < kEdgeDistance && best == 0) {
        near_edge = true;
        edge_block(v0 - v1, info.a01, kV0V1Convex, kV0V1Swap, info.flags, tri_n, n_unit, n_unit, normal, point_b, point_a,
                   dist, concave_hits, ar);
    }
    if (fabsf(info.a12) < kEdge2Pi && len(contact - nearest_on_segment(contact, v1, v2)) < kEdgeDistance && best == 1) {
        near_edge = true;
        edge_block(v1 - v2, info.a12, kV1V2Convex, kV1V2Swap, info.flags, tri_n, n_unit, normal, normal, point_b, point_a,
                   dist, concave_hits, ar);
    }
    if (fabsf(info.a20) < kEdge2Pi && len(contact - nearest_on_segment(contact, v2, v0)) < kEdgeDistance && best == 2) {
        near_edge = true;
        edge_block(v2 - v0, info.a20, kV2V0Convex, kV2V0Swap, info.flags, tri_n, n_unit, normal, normal, point_b, point_a,
                   dist, concave_hits, ar);
    }
    if (near_edge && concave_hits > 0) {
        // frontFacing = 1 (no BT_TRIANGLE_CONVEX_BACKFACE_MODE), not concave double-sided
        if (dot(tri_n, n_unit) < 0.f) return;
        normal = tri_n;
        point_b = point_a - normal * dist;
    }
}

}  // namespace rl
