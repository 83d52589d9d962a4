// bvh_ref.hpp -- ORACLE (test infrastructure only; never linked into the product).
//
// The order in which Bullet visits the triangles of one arena collision mesh: RocketSim builds each mesh
// as btBvhTriangleMeshShape(mesh, useQuantizedAabbCompression = true) (RocketSim.cpp:167), whose
// quantized BVH (btOptimizedBvh::build, btOptimizedBvh.cpp:28-160; btQuantizedBvh::buildTree /
// calcSplittingAxis / sortAndCalcSplittingIndex, btQuantizedBvh.cpp:116-305) partitions the leaf array in
// place; the default stackless walk (walkStacklessQuantizedTree, :676-740) visits the nodes in array
// order, so overlapping triangles reach btConvexTriangleCallback::processTriangle in final leaf order.
// Restated here:
//   * the mesh's local AABB (btTriangleMeshShape::recalcLocalAabb over every vertex, margin 0),
//   * setQuantizationValues(min, max, margin 1) with its two re-quantization passes (:76-114),
//   * per triangle: AABB of its vertices, widened to 0.002 where thinner, quantized (min: & 0xfffe,
//     max: (v + 1) | 1) (btOptimizedBvh.cpp:118-150, btQuantizedBvh.h:331-358),
//   * buildTree's recursion: split axis = largest variance of the unquantized leaf centres, split value =
//     their mean, leaves with centre > split swapped to the front in order, the 1/3 balance fallback.
// Returns order[k] = the triangle (index within the mesh) visited k-th.
#pragma once
#include <algorithm>
#include <cstdint>
#include <utility>
#include <vector>

#include "rsim_math.hpp"

namespace orc {
namespace bvh {

struct Q {
    V mn, mx, quant;  // m_bvhAabbMin / Max, m_bvhQuantization
    void quantize(uint16_t out[3], V p, bool is_max) const {
        V v = (p - mn) * quant;
        for (int i = 0; i < 3; i++)
            out[i] = is_max ? (uint16_t)(((uint16_t)(v[i] + 1.f)) | 1) : (uint16_t)(((uint16_t)(v[i])) & 0xfffe);
    }
    V unquantize(const uint16_t in[3]) const {
        V o((float)in[0] / quant.x, (float)in[1] / quant.y, (float)in[2] / quant.z);
        return o + mn;
    }
    void set(V bmin, V bmax) {
        const V clamp(1.f, 1.f, 1.f);
        mn = bmin - clamp;
        mx = bmax + clamp;
        auto q65533 = [&]() {
            V size = mx - mn;
            quant = V(65533.f / size.x, 65533.f / size.y, 65533.f / size.z);
        };
        q65533();
        uint16_t t[3];
        quantize(t, mn, false);
        V v = unquantize(t) - clamp;
        mn = V(mn.x < v.x ? mn.x : v.x, mn.y < v.y ? mn.y : v.y, mn.z < v.z ? mn.z : v.z);  // setMin (btMin)
        q65533();
        quantize(t, mx, true);
        v = unquantize(t) + clamp;
        mx = V(mx.x > v.x ? mx.x : v.x, mx.y > v.y ? mx.y : v.y, mx.z > v.z ? mx.z : v.z);  // setMax (btMax)
        q65533();
    }
};

struct Leaf {
    uint16_t qmin[3], qmax[3];
    int tri;
};

struct Builder {
    Q q;
    std::vector<Leaf> leaves;
    V center(int i) const {
        return (q.unquantize(leaves[i].qmax) + q.unquantize(leaves[i].qmin)) * 0.5f;  // 0.5 * (max + min)
    }
    int split_axis(int s, int e) const {
        V means(0.f, 0.f, 0.f), var(0.f, 0.f, 0.f);
        const int n = e - s;
        for (int i = s; i < e; i++) means += center(i);
        means *= (1.f / (float)n);
        for (int i = s; i < e; i++) {
            V d = center(i) - means;
            var += d * d;
        }
        var *= (1.f / ((float)n - 1));
        return var.x < var.y ? (var.y < var.z ? 2 : 1) : (var.x < var.z ? 2 : 0);  // maxAxis
    }
    int split_index(int s, int e, int axis) {
        const int n = e - s;
        V means(0.f, 0.f, 0.f);
        for (int i = s; i < e; i++) means += center(i);
        means *= (1.f / (float)n);
        const float split = means[axis];
        int k = s;
        for (int i = s; i < e; i++)
            if (center(i)[axis] > split) std::swap(leaves[i], leaves[k++]);
        const int bal = n / 3;
        if (k <= s + bal || k >= e - 1 - bal) k = s + (n >> 1);
        return k;
    }
    // buildTree's nodes in the order it emits them (depth first, left first): node i covers leaf positions
    // [ns[i], ne[i]), nskip[i] = the node after its subtree (the stackless walk's escape index)
    std::vector<int> ns, ne, nskip;
    void build(int s, int e) {
        const int me = (int)ns.size();
        ns.push_back(s);
        ne.push_back(e);
        nskip.push_back(0);
        if (e - s > 1) {
            const int axis = split_axis(s, e);
            const int k = split_index(s, e, axis);
            build(s, k);
            build(k, e);
        }
        nskip[me] = (int)ns.size();
    }
};

// The walk of one mesh's BVH (walkStacklessQuantizedTree / ...AgainstRay, btQuantizedBvh.cpp:676-740,
// 479-590): nodes in array order, a subtree skipped (escape index) when its box misses the query, the
// overlapping leaves reported in leaf order.  Bullet tests quantized node boxes, which contain the exact ones,
// and processTriangle then applies the exact triangle AABB test (btConvexConcaveCollisionAlgorithm.cpp:71-138);
// testing exact boxes here drops the same triangles earlier, so the reported set and order are Bullet's.
struct Tree {
    std::vector<int> ns, ne, nskip;  // node -> leaf positions [ns, ne), escape index
    std::vector<V> mn, mx;           // node boxes: the union of their triangles' exact AABBs
    // calls f(k) for every leaf position k whose triangle box overlaps [qmn, qmx], in leaf order
    template <class F>
    void walk(V qmn, V qmx, F&& f) const {
        const int n = (int)ns.size();
        for (int i = 0; i < n;) {
            const bool hit = !(qmn.x > mx[i].x || qmx.x < mn[i].x || qmn.y > mx[i].y || qmx.y < mn[i].y ||
                               qmn.z > mx[i].z || qmx.z < mn[i].z);
            if (!hit) {
                i = nskip[i];
                continue;
            }
            if (ne[i] - ns[i] == 1) f(ns[i]);
            i++;
        }
    }
};

// tris: ntris x 9 floats (bullet units), one mesh (collision object); tree (optional): the node hierarchy
// over the leaf positions with exact triangle boxes
inline std::vector<int> leaf_order(const float* tris, int ntris, Tree* tree = nullptr) {
    std::vector<int> order;
    if (ntris <= 0) return order;
    V lo(1e18f, 1e18f, 1e18f), hi(-1e18f, -1e18f, -1e18f);
    // recalcLocalAabb: per axis the largest / smallest vertex coordinate (SupportVertexCallback keeps a
    // strictly larger dot), + / - margin 0
    float mx[3] = {-1e18f, -1e18f, -1e18f}, mn[3] = {-1e18f, -1e18f, -1e18f};
    for (int t = 0; t < ntris; t++)
        for (int k = 0; k < 3; k++)
            for (int i = 0; i < 3; i++) {
                const float c = tris[9 * t + 3 * k + i];
                if (c > mx[i]) mx[i] = c;
                if (-c > mn[i]) mn[i] = -c;
            }
    for (int i = 0; i < 3; i++) {
        hi[i] = mx[i] + 0.f;
        lo[i] = -mn[i] - 0.f;
    }
    Builder b;
    b.q.set(lo, hi);
    b.leaves.resize(ntris);
    for (int t = 0; t < ntris; t++) {
        V a(1e18f, 1e18f, 1e18f), z(-1e18f, -1e18f, -1e18f);
        for (int k = 0; k < 3; k++)
            for (int i = 0; i < 3; i++) {
                const float c = tris[9 * t + 3 * k + i];
                if (c < a[i]) a[i] = c;  // setMin / setMax
                if (z[i] < c) z[i] = c;
            }
        for (int i = 0; i < 3; i++)
            if (z[i] - a[i] < 0.002f) {  // MIN_AABB_DIMENSION / MIN_AABB_HALF_DIMENSION
                z[i] = z[i] + 0.001f;
                a[i] = a[i] - 0.001f;
            }
        b.q.quantize(b.leaves[t].qmin, a, false);
        b.q.quantize(b.leaves[t].qmax, z, true);
        b.leaves[t].tri = t;
    }
    b.build(0, ntris);
    order.resize(ntris);
    for (int k = 0; k < ntris; k++) order[k] = b.leaves[k].tri;
    if (tree) {
        tree->ns = b.ns;
        tree->ne = b.ne;
        tree->nskip = b.nskip;
        const int nn = (int)b.ns.size();
        std::vector<V> lmn(ntris), lmx(ntris);  // exact triangle boxes by leaf position
        for (int k = 0; k < ntris; k++) {
            const float* p = tris + 9 * (size_t)order[k];
            V a(p[0], p[1], p[2]), z = a;
            for (int v = 1; v < 3; v++)
                for (int i = 0; i < 3; i++) {
                    a[i] = std::min(a[i], p[3 * v + i]);
                    z[i] = std::max(z[i], p[3 * v + i]);
                }
            lmn[k] = a;
            lmx[k] = z;
        }
        tree->mn.assign(nn, V());
        tree->mx.assign(nn, V());
        for (int i = nn - 1; i >= 0; i--) {  // children follow their parent: fold leaves bottom-up per node
            V a = lmn[b.ns[i]], z = lmx[b.ns[i]];
            for (int k = b.ns[i] + 1; k < b.ne[i]; k++)
                for (int c = 0; c < 3; c++) {
                    a[c] = std::min(a[c], lmn[k][c]);
                    z[c] = std::max(z[c], lmx[k][c]);
                }
            tree->mn[i] = a;
            tree->mx[i] = z;
        }
    }
    return order;
}

}  // namespace bvh
}  // namespace orc
