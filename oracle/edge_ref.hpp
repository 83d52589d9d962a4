// edge_ref.hpp -- TEST INFRASTRUCTURE (CPU oracle): Bullet's internal-edge utility restated for the
// oracle's world, independently of the kernel's csrc/edge_info.hpp.
//
//   gen_edge_info      btGenerateInternalEdgeInfo + btConnectivityProcessor::processTriangle
//                      (BT/BulletCollision/CollisionDispatch/btInternalEdgeUtility.cpp:50-358)
//   adjust_edge        btAdjustInternalEdgeContacts (:414-798), btClampNormal (:385-412),
//                      btNearestPointInLineSegment (:362-383); normalAdjustFlags = 0
//
// Called by RocketSim for every arena mesh (RocketSim.cpp:166-170) and at the end of the contact-added
// callback (Arena.cpp:275-279).  Meshes are static at the identity transform (local = world frame).
// Neighbour candidates of a triangle: the other triangles of its collision object whose AABB, grown
// by 2e-4, overlaps its own, in the order the object's quantized BVH visits them (`visit`, bvh_ref.hpp;
// the reference's processAllTriangles query, btInternalEdgeUtility.cpp:340-356) -- the last neighbour
// sharing an edge writes its record.
#pragma once
#include <cmath>
#include <map>
#include <vector>

#include "rsim_math.hpp"

namespace orc {

struct TriInfo {  // btTriangleInfo
    float e01 = 2.0f * 3.1415926535897932384626433832795029f;  // m_edgeV0V1Angle = SIMD_2_PI
    float e12 = 2.0f * 3.1415926535897932384626433832795029f;
    float e20 = 2.0f * 3.1415926535897932384626433832795029f;
    int flags = 0;
    bool present = false;
};

namespace edge {
const float PI = 3.1415926535897932384626433832795029f;  // SIMD_PI
const float TWO_PI = 2.0f * PI;                            // SIMD_2_PI
const float CONVEX_EPS = 0.00f, PLANAR_EPS = 0.0001f;      // btTriangleInfoMap()
const float EQUAL_VERTEX = 0.0001f * 0.0001f, EDGE_DIST = 0.1f, MAX_EDGE_ANGLE = TWO_PI;
enum { V0V1_CONVEX = 1, V1V2_CONVEX = 2, V2V0_CONVEX = 4, V0V1_SWAP = 8, V1V2_SWAP = 16, V2V0_SWAP = 32 };

inline float get_angle(V edgeA, V normalA, V normalB) {  // btGetAngle
    return rs_atan2f_at(dot(normalB, edgeA), dot(normalB, normalA), RS_SITE_EDGE);
}
inline V calc_normal(V a, V b, V c) {  // btTriangleShape::calcNormal
    return bt_normalize(cross(b - a, c - a));
}
inline V quat_rotate(Q r, V w) {  // quatRotate: (r * w) *= r.inverse()
    Q q{r.w * w.x + r.y * w.z - r.z * w.y, r.w * w.y + r.z * w.x - r.x * w.z, r.w * w.z + r.x * w.y - r.y * w.x,
        -r.x * w.x - r.y * w.y - r.z * w.z};
    Q inv{-r.x, -r.y, -r.z, r.w};
    Q o = qmul(q, inv);
    return V(o.x, o.y, o.z);
}

// btConnectivityProcessor::processTriangle(triangle = B), A = the triangle being processed
inline void process_triangle(const V* A, const V* B, TriInfo& info) {
    int numshared = 0;
    int sharedVertsA[3] = {-1, -1, -1};
    int sharedVertsB[3] = {-1, -1, -1};
    float crossBSqr = len2(cross(B[1] - B[0], B[2] - B[0]));
    if (crossBSqr < EQUAL_VERTEX) return;
    float crossASqr = len2(cross(A[1] - A[0], A[2] - A[0]));
    if (crossASqr < EQUAL_VERTEX) return;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) {
            if (len2(A[i] - B[j]) < EQUAL_VERTEX) {
                sharedVertsA[numshared] = i;
                sharedVertsB[numshared] = j;
                numshared++;
                if (numshared >= 3) return;
            }
        }
        if (numshared >= 3) return;
    }
    if (numshared != 2) return;  // case 0 / 1: nothing to record
    if (sharedVertsA[0] == 0 && sharedVertsA[1] == 2) {
        sharedVertsA[0] = 2;
        sharedVertsA[1] = 0;
        int tmp = sharedVertsB[1];
        sharedVertsB[1] = sharedVertsB[0];
        sharedVertsB[0] = tmp;
    }
    if (!info.present) {
        info = TriInfo();
        info.present = true;
    }
    int sumvertsA = sharedVertsA[0] + sharedVertsA[1];
    int otherIndexA = 3 - sumvertsA;
    V edgeVec = A[sharedVertsA[1]] - A[sharedVertsA[0]];
    int otherIndexB = 3 - (sharedVertsB[0] + sharedVertsB[1]);
    V normalA = calc_normal(A[0], A[1], A[2]);
    V normalB = calc_normal(B[sharedVertsB[1]], B[sharedVertsB[0]], B[otherIndexB]);
    edgeVec = bt_normalize(edgeVec);
    V edgeCrossA = bt_normalize(cross(edgeVec, normalA));
    {
        V tmp = A[otherIndexA] - A[sharedVertsA[0]];
        if (dot(edgeCrossA, tmp) < 0) edgeCrossA *= -1;
    }
    V edgeCrossB = bt_normalize(cross(edgeVec, normalB));
    {
        V tmp = B[otherIndexB] - B[sharedVertsB[0]];
        if (dot(edgeCrossB, tmp) < 0) edgeCrossB *= -1;
    }
    V calculatedEdge = cross(edgeCrossA, edgeCrossB);
    float len2e = len2(calculatedEdge);
    float correctedAngle = 0;
    bool isConvex = false;
    if (len2e < PLANAR_EPS) {
        // angle2 = ang4 = 0
    } else {
        calculatedEdge = bt_normalize(calculatedEdge);
        V calculatedNormalA = bt_normalize(cross(calculatedEdge, edgeCrossA));
        float angle2 = get_angle(calculatedNormalA, edgeCrossA, edgeCrossB);
        float ang4 = PI - angle2;
        float dotA = dot(normalA, edgeCrossB);
        isConvex = (dotA < 0.);
        correctedAngle = isConvex ? ang4 : -ang4;
    }
    switch (sumvertsA) {
        case 1: {
            V e = A[0] - A[1];
            V computedNormalB = quat_rotate(quat_axis_angle(e, -correctedAngle), normalA);
            if (dot(computedNormalB, normalB) < 0) info.flags |= V0V1_SWAP;
            info.e01 = -correctedAngle;
            if (isConvex) info.flags |= V0V1_CONVEX;
            break;
        }
        case 2: {
            V e = A[2] - A[0];
            V computedNormalB = quat_rotate(quat_axis_angle(e, -correctedAngle), normalA);
            if (dot(computedNormalB, normalB) < 0) info.flags |= V2V0_SWAP;
            info.e20 = -correctedAngle;
            if (isConvex) info.flags |= V2V0_CONVEX;
            break;
        }
        case 3: {
            V e = A[1] - A[2];
            V computedNormalB = quat_rotate(quat_axis_angle(e, -correctedAngle), normalA);
            if (dot(computedNormalB, normalB) < 0) info.flags |= V1V2_SWAP;
            info.e12 = -correctedAngle;
            if (isConvex) info.flags |= V1V2_CONVEX;
            break;
        }
    }
}

// btGenerateInternalEdgeInfo over every collision object of a mesh (tri: 3 vertices per triangle)
// visit: the mesh's triangles in BVH visit order (each object's range permuted within itself)
inline std::vector<TriInfo> gen_edge_info(const std::vector<V>& tri, const std::vector<int>& tri_obj,
                                          const std::vector<int>& visit) {
    const int n = (int)tri_obj.size();
    std::vector<TriInfo> out(n);
    std::vector<V> mn(n), mx(n);
    for (int t = 0; t < n; t++) {
        mn[t] = mx[t] = tri[3 * t];
        for (int k = 1; k < 3; k++)
            for (int a = 0; a < 3; a++) {
                mn[t][a] = std::fmin(mn[t][a], tri[3 * t + k][a]);
                mx[t][a] = std::fmax(mx[t][a], tri[3 * t + k][a]);
            }
    }
    const float g = 2e-4f;
    for (int a = 0; a < n; a++)
        for (int k = 0; k < n; k++) {
            const int b = visit[k];
            if (b == a || tri_obj[b] != tri_obj[a]) continue;
            bool apart = false;
            for (int k = 0; k < 3; k++) apart |= mn[b][k] > mx[a][k] + g || mx[b][k] < mn[a][k] - g;
            if (apart) continue;
            process_triangle(&tri[3 * a], &tri[3 * b], out[a]);
        }
    return out;
}

inline V nearest_point_in_line_segment(V point, V line0, V line1) {
    V lineDelta = line1 - line0;
    if (fuzzy_zero(lineDelta)) return line0;
    float delta = dot(point - line0, lineDelta) / dot(lineDelta, lineDelta);
    if (delta < 0) delta = 0;
    else if (delta > 1) delta = 1;
    return line0 + lineDelta * delta;
}

inline bool clamp_normal(V edgeV, V tri_normal, V localContactNormalOnB, float correctedEdgeAngle, V& clamped) {
    V edgeCross = bt_normalize(cross(edgeV, tri_normal));
    float curAngle = get_angle(edgeCross, tri_normal, localContactNormalOnB);
    if (correctedEdgeAngle < 0) {
        if (curAngle < correctedEdgeAngle) {
            float diffAngle = correctedEdgeAngle - curAngle;
            clamped = mat_from_quat(quat_axis_angle(edgeV, diffAngle)) * localContactNormalOnB;
            return true;
        }
    }
    if (correctedEdgeAngle >= 0) {
        if (curAngle > correctedEdgeAngle) {
            float diffAngle = correctedEdgeAngle - curAngle;
            clamped = mat_from_quat(quat_axis_angle(edgeV, diffAngle)) * localContactNormalOnB;
            return true;
        }
    }
    return false;
}

// btAdjustInternalEdgeContacts on one manifold point: n = m_normalWorldOnB, localB = m_localPointB
// (= m_positionWorldOnB), posA = m_positionWorldOnA, dist = m_distance1
inline void adjust_edge(const V* tv, const TriInfo& info, V& n, V& localB, V posA, float dist) {
    if (!info.present) return;
    const float frontFacing = 1.f;
    V v0 = tv[0], v1 = tv[1], v2 = tv[2];
    V tri_normal = calc_normal(v0, v1, v2);
    V nearest = nearest_point_in_line_segment(localB, v0, v1);
    V contact = localB;
    bool isNearEdge = false;
    int numConcaveEdgeHits = 0;
    V localContactNormalOnB = bt_normalize(n);
    int bestedge = -1;
    float disttobestedge = 1e18f;  // BT_LARGE_FLOAT
    if (std::fabs(info.e01) < MAX_EDGE_ANGLE) {
        V nr = nearest_point_in_line_segment(localB, v0, v1);
        float l = len(contact - nr);
        if (l < disttobestedge) {
            bestedge = 0;
            disttobestedge = l;
        }
    }
    if (std::fabs(info.e12) < MAX_EDGE_ANGLE) {
        V nr = nearest_point_in_line_segment(localB, v1, v2);
        float l = len(contact - nr);
        if (l < disttobestedge) {
            bestedge = 1;
            disttobestedge = l;
        }
    }
    if (std::fabs(info.e20) < MAX_EDGE_ANGLE) {
        V nr = nearest_point_in_line_segment(localB, v2, v0);
        float l = len(contact - nr);
        if (l < disttobestedge) {
            bestedge = 2;
            disttobestedge = l;
        }
    }
    auto reproject = [&]() { localB = posA - n * dist; };
    // edge 0 -> 1
    if (std::fabs(info.e01) < MAX_EDGE_ANGLE) {
        float l = len(contact - nearest);
        if (l < EDGE_DIST && bestedge == 0) {
            V edgeV = v0 - v1;
            isNearEdge = true;
            if (info.e01 == 0.f) {
                numConcaveEdgeHits++;
            } else {
                bool isEdgeConvex = (info.flags & V0V1_CONVEX);
                float swapFactor = isEdgeConvex ? 1.f : -1.f;
                V nA = swapFactor * tri_normal;
                V computedNormalB = quat_rotate(quat_axis_angle(edgeV, info.e01), tri_normal);
                if (info.flags & V0V1_SWAP) computedNormalB *= -1;
                V nB = swapFactor * computedNormalB;
                float NdotA = dot(localContactNormalOnB, nA), NdotB = dot(localContactNormalOnB, nB);
                bool backFacingNormal = (NdotA < CONVEX_EPS) && (NdotB < CONVEX_EPS);
                if (backFacingNormal) {
                    numConcaveEdgeHits++;
                } else {
                    V clamped;
                    if (clamp_normal(edgeV, swapFactor * tri_normal, localContactNormalOnB, info.e01, clamped) &&
                        dot(clamped, frontFacing * tri_normal) > 0) {
                        n = clamped;
                        reproject();
                    }
                }
            }
        }
    }
    // edge 1 -> 2
    nearest = nearest_point_in_line_segment(contact, v1, v2);
    if (std::fabs(info.e12) < MAX_EDGE_ANGLE) {
        float l = len(contact - nearest);
        if (l < EDGE_DIST && bestedge == 1) {
            isNearEdge = true;
            V edgeV = v1 - v2;
            if (info.e12 == 0.f) {
                numConcaveEdgeHits++;
            } else {
                bool isEdgeConvex = (info.flags & V1V2_CONVEX) != 0;
                float swapFactor = isEdgeConvex ? 1.f : -1.f;
                V nA = swapFactor * tri_normal;
                V computedNormalB = quat_rotate(quat_axis_angle(edgeV, info.e12), tri_normal);
                if (info.flags & V1V2_SWAP) computedNormalB *= -1;
                V nB = swapFactor * computedNormalB;
                float NdotA = dot(localContactNormalOnB, nA), NdotB = dot(localContactNormalOnB, nB);
                bool backFacingNormal = (NdotA < CONVEX_EPS) && (NdotB < CONVEX_EPS);
                if (backFacingNormal) {
                    numConcaveEdgeHits++;
                } else {
                    V localNormalNow = n;  // re-read from the point (identity basis), not normalized
                    V clamped;
                    if (clamp_normal(edgeV, swapFactor * tri_normal, localNormalNow, info.e12, clamped) &&
                        dot(clamped, frontFacing * tri_normal) > 0) {
                        n = clamped;
                        reproject();
                    }
                }
            }
        }
    }
    // edge 2 -> 0
    nearest = nearest_point_in_line_segment(contact, v2, v0);
    if (std::fabs(info.e20) < MAX_EDGE_ANGLE) {
        float l = len(contact - nearest);
        if (l < EDGE_DIST && bestedge == 2) {
            isNearEdge = true;
            V edgeV = v2 - v0;
            if (info.e20 == 0.f) {
                numConcaveEdgeHits++;
            } else {
                bool isEdgeConvex = (info.flags & V2V0_CONVEX) != 0;
                float swapFactor = isEdgeConvex ? 1.f : -1.f;
                V nA = swapFactor * tri_normal;
                V computedNormalB = quat_rotate(quat_axis_angle(edgeV, info.e20), tri_normal);
                if (info.flags & V2V0_SWAP) computedNormalB *= -1;
                V nB = swapFactor * computedNormalB;
                float NdotA = dot(localContactNormalOnB, nA), NdotB = dot(localContactNormalOnB, nB);
                bool backFacingNormal = (NdotA < CONVEX_EPS) && (NdotB < CONVEX_EPS);
                if (backFacingNormal) {
                    numConcaveEdgeHits++;
                } else {
                    V localNormalNow = n;
                    V clamped;
                    if (clamp_normal(edgeV, swapFactor * tri_normal, localNormalNow, info.e20, clamped) &&
                        dot(clamped, frontFacing * tri_normal) > 0) {
                        n = clamped;
                        reproject();
                    }
                }
            }
        }
    }
    if (isNearEdge && numConcaveEdgeHits > 0) {
        V newNormal = tri_normal * frontFacing;
        float d = dot(newNormal, localContactNormalOnB);
        if (d < 0) return;
        n = newNormal;
        reproject();
    }
}
}  // namespace edge
}  // namespace orc
