// mesh.hip -- collision-mesh ingestion (include/rlgpu_mesh.h) and the host build of the env
// kernel's mesh table + uniform-grid index (mesh.hpp).  Host code only.
#include "mesh.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>

#include "../../include/rlgpu_arena_mesh.h"
#include "../../include/rlgpu_env.h"
#include "../../include/rlgpu_mesh.h"
#include "common.hpp"
#include "edge_info.hpp"

namespace rlgpu {

namespace {

// The reference converts each vertex component with `uint32_t curVal = float`
// (CollisionMeshFile.cpp:79).  Out-of-range conversions are undefined in C++; x86-64 compilers
// emit a truncating float->int64 conversion (cvttss2si) and keep the low 32 bits, which is what
// this restates (NaN and |x| >= 2^63 give the int64 "indefinite" value, low bits 0).
uint32_t hash_component(float x) {
    if (!(std::fabs(x) < 9.2233720368547758e18f)) return 0u;
    return (uint32_t)(uint64_t)(int64_t)x;
}

// CollisionMeshFile::UpdateHash (CollisionMeshFile.cpp:70-95)
uint32_t cmf_hash(const int32_t* idx, int ntris, const float* verts, int nverts) {
    uint32_t hash = (uint32_t)((uint64_t)nverts + (uint64_t)ntris * (uint64_t)nverts);
    const uint32_t kMueller = 0x45D9F3B, kShift = 0x9E3779B9;
    for (int t = 0; t < ntris; t++)
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                uint32_t v = hash_component(verts[3 * idx[3 * t + i] + j]);
                for (int k = 0; k < 2; k++) v = ((v >> 16) ^ v) * kMueller;
                v = (v >> 16) ^ v;
                hash ^= v + kShift + (hash << 6) + (hash >> 2);
            }
    return hash;
}

const uint32_t kSoccarHashes[] = {0xA160BAF9, 0x2811EEE8, 0xB81AC8B9, 0x760358D3, 0x73AE4940, 0x918F4A4E,
                                  0x1F8EE550, 0x255BA8C1, 0x14B84668, 0xEC759EBF, 0x94FB0D5C, 0xDEA07102,
                                  0xBD4FBEA8, 0x39A47F63, 0x3D79D25D, 0xD84C7A68};
const uint32_t kHoopsHashes[] = {0x72F2359E, 0x5ED14A26, 0xFD5A0D07, 0x92AFA5B5, 0x0E4133C7, 0x399E8B5F,
                                 0xBB9D4FB5, 0x8C87FB93, 0x1CFD0E16, 0xE19E1DF6, 0x9CA179DC, 0x16F3CC19};

}  // namespace

std::vector<float> builtin_mesh_bt() {
    std::vector<float> out((size_t)RLGPU_MESH_TRIS * 9);
    const float UU = 1.f / 50.f;
    for (int t = 0; t < RLGPU_MESH_TRIS; t++)
        for (int k = 0; k < 9; k++) out[(size_t)t * 9 + k] = RLGPU_MESH_UU[t][k] * UU;
    return out;
}

MeshGrid build_mesh_grid(const float* tris_in, int ntris, const int32_t* object_ntris, int nobjects, int arith) {
    RLGPU_REQUIRE(tris_in && ntris > 0, "mesh: no triangles");
    RLGPU_REQUIRE(ntris < (1 << 20), "mesh: more than 2^20 - 1 triangles");
    if (!object_ntris) nobjects = 1;
    RLGPU_REQUIRE(nobjects >= 1 && nobjects <= RLGPU_MAX_MESH_OBJECTS,
                  "mesh: object count must be in [1, RLGPU_MAX_MESH_OBJECTS]");
    MeshGrid g;
    g.ntris = ntris;
    std::vector<int> obj(ntris, 0);
    if (object_ntris) {
        int64_t sum = 0;
        for (int k = 0; k < nobjects; k++) {
            RLGPU_REQUIRE(object_ntris[k] >= 0, "mesh: negative object triangle count");
            sum += object_ntris[k];
        }
        RLGPU_REQUIRE(sum == ntris, "mesh: object triangle counts do not add up to mesh_ntris");
        int t = 0;
        for (int k = 0; k < nobjects; k++)
            for (int i = 0; i < object_ntris[k]; i++) obj[t++] = k;
    }
    for (size_t i = 0; i < (size_t)ntris * 9; i++)
        RLGPU_REQUIRE(std::isfinite(tris_in[i]), "mesh: non-finite vertex coordinate");
    // The device tables number the triangles in Bullet's BVH visit order (one btBvhTriangleMeshShape per
    // object): a triangle's index is its visit position, so every "lower index first" rule of the kernel
    // (grid cells list ascending indices, the commit sorts candidates by (pair, index), ray ties go to the
    // lower index) follows the reference's walk.  visit_tri maps a position back to the load order.
    g.visit_pos.assign(ntris, 0);
    g.visit_tri.assign(ntris, 0);
    for (int t0 = 0; t0 < ntris;) {
        int t1 = t0;
        while (t1 < ntris && obj[t1] == obj[t0]) t1++;
        const std::vector<int> order = bvh_visit_order(tris_in + (size_t)t0 * 9, t1 - t0);
        for (int k = 0; k < t1 - t0; k++) {
            g.visit_tri[t0 + k] = t0 + order[k];
            g.visit_pos[t0 + order[k]] = t0 + k;
        }
        t0 = t1;
    }
    std::vector<float> visit_tris((size_t)ntris * 9);
    for (int p = 0; p < ntris; p++)
        std::memcpy(&visit_tris[(size_t)p * 9], tris_in + (size_t)g.visit_tri[p] * 9, 9 * sizeof(float));
    const float* tris = visit_tris.data();  // obj[] is unchanged: objects keep their ranges
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int t = 0; t < ntris; t++)
        for (int v = 0; v < 3; v++)
            for (int a = 0; a < 3; a++) {
                float x = tris[(size_t)t * 9 + v * 3 + a];
                mn[a] = std::fmin(mn[a], x);
                mx[a] = std::fmax(mx[a], x);
            }
    // cells of >= 160 uu (3.2 bullet units): a wheel ray touches one or two cells per axis, a car
    // or ball two or three; a SOCCAR-density mesh (quarter pipes of 10 x 36 segments) lists ~15
    // triangles in a cell it crosses.  Measured on the procedural SOCCAR mesh (env kernel per launch):
    // 1.5 bt 1.071 ms, 2.56 bt 1.066, 3.2 bt 1.054-1.057, 4.0 bt 1.061, 5.12 bt 1.075
    // (profiles/r04ad_env_ab.txt)
    float ext = std::fmax(mx[0] - mn[0], std::fmax(mx[1] - mn[1], mx[2] - mn[2]));
    float cell = std::fmax(3.2f, ext / 128.f);
    g.inv_cell = 1.f / cell;
    g.ox = mn[0];
    g.oy = mn[1];
    g.oz = mn[2];
    int* dims[3] = {&g.nx, &g.ny, &g.nz};
    for (int a = 0; a < 3; a++) {
        int n = (int)std::floor((mx[a] - mn[a]) * g.inv_cell) + 1;
        *dims[a] = n < 1 ? 1 : (n > 128 ? 128 : n);
    }
    const float o[3] = {g.ox, g.oy, g.oz};
    const int n3[3] = {g.nx, g.ny, g.nz};
    auto cell_range = [&](int t, int lo[3], int hi[3]) {
        const float* p = tris + (size_t)t * 9;
        for (int a = 0; a < 3; a++) {
            float tmn = std::fmin(p[a], std::fmin(p[3 + a], p[6 + a]));
            float tmx = std::fmax(p[a], std::fmax(p[3 + a], p[6 + a]));
            lo[a] = grid_cell_host(tmn, o[a], g.inv_cell, n3[a]);
            hi[a] = grid_cell_host(tmx, o[a], g.inv_cell, n3[a]);
        }
    };
    const size_t ncell = (size_t)g.nx * g.ny * g.nz;
    std::vector<int> count(ncell + 1, 0);
    for (int t = 0; t < ntris; t++) {
        int lo[3], hi[3];
        cell_range(t, lo, hi);
        for (int z = lo[2]; z <= hi[2]; z++)
            for (int y = lo[1]; y <= hi[1]; y++)
                for (int x = lo[0]; x <= hi[0]; x++) count[((size_t)z * g.ny + y) * g.nx + x]++;
    }
    g.cell_start.assign(ncell + 1, 0);
    for (size_t c = 0; c < ncell; c++) g.cell_start[c + 1] = g.cell_start[c] + count[c];
    {  // the empty box: from the centre cell (if empty), grow one face at a time while the added slab is empty
        auto slab_empty = [&](int x0, int x1, int y0, int y1, int z0, int z1) {
            for (int z = z0; z <= z1; z++)
                for (int y = y0; y <= y1; y++)
                    for (int x = x0; x <= x1; x++)
                        if (count[((size_t)z * g.ny + y) * g.nx + x]) return false;
            return true;
        };
        int b[6] = {g.nx / 2, g.nx / 2, g.ny / 2, g.ny / 2, g.nz / 2, g.nz / 2};
        if (slab_empty(b[0], b[1], b[2], b[3], b[4], b[5])) {
            const int lim[6] = {0, g.nx - 1, 0, g.ny - 1, 0, g.nz - 1};
            for (bool grew = true; grew;) {
                grew = false;
                for (int f = 0; f < 6; f++) {
                    if (b[f] == lim[f]) continue;
                    int c[6] = {b[0], b[1], b[2], b[3], b[4], b[5]};
                    c[f] += (f & 1) ? 1 : -1;
                    const int ax = f >> 1;  // the new slab: the face's new layer across the box
                    int s[6] = {b[0], b[1], b[2], b[3], b[4], b[5]};
                    s[2 * ax] = s[2 * ax + 1] = c[f];
                    if (slab_empty(s[0], s[1], s[2], s[3], s[4], s[5])) {
                        b[f] = c[f];
                        grew = true;
                    }
                }
            }
            std::memcpy(g.empty, b, sizeof b);
        }
    }
    RLGPU_REQUIRE(g.cell_start[ncell] < (1 << 26), "mesh: grid index too large");
    g.cell_tri.assign((size_t)g.cell_start[ncell] * 12, 0.f);
    std::vector<int> fill(g.cell_start.begin(), g.cell_start.end() - 1);
    for (int t = 0; t < ntris; t++) {  // ascending t within every cell
        int lo[3], hi[3];
        cell_range(t, lo, hi);
        const float* p = tris + (size_t)t * 9;
        for (int z = lo[2]; z <= hi[2]; z++)
            for (int y = lo[1]; y <= hi[1]; y++)
                for (int x = lo[0]; x <= hi[0]; x++) {
                    float* d = &g.cell_tri[(size_t)fill[((size_t)z * g.ny + y) * g.nx + x]++ * 12];
                    for (int v = 0; v < 3; v++)
                        for (int a = 0; a < 3; a++) d[v * 4 + a] = p[v * 3 + a];
                    std::memcpy(&d[3], &obj[t], sizeof(int));
                    std::memcpy(&d[7], &t, sizeof(int));
                    const int cell = x | (y << 8) | (z << 16);  // the entry's cell (dims <= 128 per axis)
                    std::memcpy(&d[11], &cell, sizeof(int));
                }
    }
    g.tri.assign((size_t)ntris * 12, 0.f);
    for (int t = 0; t < ntris; t++) {
        float* d = &g.tri[(size_t)t * 12];
        const float* p = tris + (size_t)t * 9;
        for (int v = 0; v < 3; v++)
            for (int a = 0; a < 3; a++) d[v * 4 + a] = p[v * 3 + a];
        std::memcpy(&d[3], &obj[t], sizeof(int));
    }
    // internal-edge records of the mesh as loaded (neighbour order = load order), moved with their triangles
    const std::vector<float> edge = mesh_edge_info(tris_in, ntris, object_ntris, object_ntris ? nobjects : 1, arith);
    g.edge.resize(edge.size());
    for (int p = 0; p < ntris; p++) std::memcpy(&g.edge[(size_t)p * 4], &edge[(size_t)g.visit_tri[p] * 4], 4 * sizeof(float));
    return g;
}

namespace {
// btQuantizedBvh's quantizer (btQuantizedBvh.h:331-415): bounds, scale, 16-bit snapped coordinates
struct BvhQuant {
    float lo[3], hi[3], scale[3];
    void rescale() {
        for (int a = 0; a < 3; a++) scale[a] = 65533.f / (hi[a] - lo[a]);
    }
    uint16_t q(float x, int a, bool upper) const {
        const float v = (x - lo[a]) * scale[a];
        return upper ? (uint16_t)((uint16_t)(v + 1.f) | 1) : (uint16_t)((uint16_t)v & 0xfffe);
    }
    float uq(uint16_t x, int a) const { return (float)x / scale[a] + lo[a]; }
};
}  // namespace

std::vector<int> bvh_visit_order(const float* tris, int n) {
    std::vector<int> out(n);
    if (n <= 0) return out;
    // btTriangleMeshShape::recalcLocalAabb: support vertices along +-axes (a vertex replaces the best
    // only with a strictly larger dot), margin 0
    float best_hi[3], best_lo[3];
    for (int a = 0; a < 3; a++) best_hi[a] = best_lo[a] = -1e18f;
    for (int i = 0; i < 3 * n; i++)
        for (int a = 0; a < 3; a++) {
            const float c = tris[3 * i + a];
            if (c > best_hi[a]) best_hi[a] = c;
            if (-c > best_lo[a]) best_lo[a] = -c;
        }
    BvhQuant Q;
    for (int a = 0; a < 3; a++) {  // setQuantizationValues(min, max, 1.0) with its two refinements
        Q.lo[a] = (-best_lo[a] - 0.f) - 1.f;
        Q.hi[a] = (best_hi[a] + 0.f) + 1.f;
    }
    Q.rescale();
    for (int a = 0; a < 3; a++) {
        const float v = Q.uq(Q.q(Q.lo[a], a, false), a) - 1.f;
        Q.lo[a] = Q.lo[a] < v ? Q.lo[a] : v;
    }
    Q.rescale();
    for (int a = 0; a < 3; a++) {
        const float v = Q.uq(Q.q(Q.hi[a], a, true), a) + 1.f;
        Q.hi[a] = Q.hi[a] > v ? Q.hi[a] : v;
    }
    Q.rescale();
    // leaves: quantized vertex AABBs widened to 0.002 (btOptimizedBvh.cpp:118-150); the partitioning
    // only ever needs each leaf's unquantized centre, 0.5 * (max + min)
    struct L {
        float c[3];
        int t;
    };
    std::vector<L> leaf(n);
    for (int t = 0; t < n; t++) {
        for (int a = 0; a < 3; a++) {
            float mn = 1e18f, mx = -1e18f;
            for (int k = 0; k < 3; k++) {
                const float c = tris[9 * t + 3 * k + a];
                mn = c < mn ? c : mn;
                mx = mx < c ? c : mx;
            }
            if (mx - mn < 0.002f) {
                mx = mx + 0.001f;
                mn = mn - 0.001f;
            }
            const float umax = Q.uq(Q.q(mx, a, true), a), umin = Q.uq(Q.q(mn, a, false), a);
            leaf[t].c[a] = (umax + umin) * 0.5f;
        }
        leaf[t].t = t;
    }
    // buildTree (btQuantizedBvh.cpp:116-305) without the nodes: ranges split depth first, left first
    std::vector<std::pair<int, int>> todo{{0, n}};
    while (!todo.empty()) {
        const auto [s, e] = todo.back();
        todo.pop_back();
        const int m = e - s;
        if (m <= 1) continue;
        float mean[3] = {0.f, 0.f, 0.f}, var[3] = {0.f, 0.f, 0.f};
        for (int i = s; i < e; i++)
            for (int a = 0; a < 3; a++) mean[a] += leaf[i].c[a];
        const float inv = 1.f / (float)m;
        for (int a = 0; a < 3; a++) mean[a] *= inv;
        for (int i = s; i < e; i++)
            for (int a = 0; a < 3; a++) {
                const float d = leaf[i].c[a] - mean[a];
                var[a] += d * d;
            }
        const float inv1 = 1.f / ((float)m - 1);
        for (int a = 0; a < 3; a++) var[a] *= inv1;
        const int axis = var[0] < var[1] ? (var[1] < var[2] ? 2 : 1) : (var[0] < var[2] ? 2 : 0);
        // sortAndCalcSplittingIndex recomputes the means (same operations, same value)
        const float split = mean[axis];
        int k = s;
        for (int i = s; i < e; i++)
            if (leaf[i].c[axis] > split) std::swap(leaf[i], leaf[k++]);
        if (k <= s + m / 3 || k >= e - 1 - m / 3) k = s + (m >> 1);
        todo.push_back({k, e});  // right after left
        todo.push_back({s, k});
    }
    for (int i = 0; i < n; i++) out[i] = leaf[i].t;
    return out;
}

// btGenerateInternalEdgeInfo per collision object (one btBvhTriangleMeshShape per object, partId 0):
// for every triangle A, every other triangle B of the object whose AABB overlaps A's, in the order the
// object's quantized BVH visits them (the reference's overlap query, btInternalEdgeUtility.cpp:300-356:
// the last neighbour sharing an edge writes A's record)
std::vector<float> mesh_edge_info(const float* tris, int ntris, const int32_t* object_ntris, int nobjects, int arith) {
    std::vector<float> out((size_t)ntris * 4, 0.f);
    auto vert = [&](int t, int k) {
        const float* p = tris + (size_t)t * 9 + 3 * k;
        return rl::v3{p[0], p[1], p[2]};
    };
    int t0 = 0;
    for (int o = 0; o < nobjects; o++) {
        const int n = object_ntris ? object_ntris[o] : ntris;
        std::vector<rl::v3> mn(n), mx(n);
        const std::vector<int> visit = bvh_visit_order(tris + (size_t)t0 * 9, n);
        for (int i = 0; i < n; i++) {
            rl::v3 a = vert(t0 + i, 0), b = vert(t0 + i, 1), c = vert(t0 + i, 2);
            mn[i] = rl::v3{std::fmin(a.x, std::fmin(b.x, c.x)), std::fmin(a.y, std::fmin(b.y, c.y)), std::fmin(a.z, std::fmin(b.z, c.z))};
            mx[i] = rl::v3{std::fmax(a.x, std::fmax(b.x, c.x)), std::fmax(a.y, std::fmax(b.y, c.y)), std::fmax(a.z, std::fmax(b.z, c.z))};
        }
        for (int i = 0; i < n; i++) {
            const rl::v3 va[3] = {vert(t0 + i, 0), vert(t0 + i, 1), vert(t0 + i, 2)};
            rl::EdgeInfo info{rl::kEdge2Pi, rl::kEdge2Pi, rl::kEdge2Pi, 0};
            for (int k = 0; k < n; k++) {
                const int j = visit[k];
                if (j == i) continue;  // self
                // AABB overlap grown by 2e-4 (twice the shared-vertex distance): a neighbour whose shared
                // vertices differ by less than the threshold always passes, as in the BVH's
                // conservative (quantized) query
                const float g = 2e-4f;
                if (mn[j].x > mx[i].x + g || mx[j].x < mn[i].x - g || mn[j].y > mx[i].y + g || mx[j].y < mn[i].y - g ||
                    mn[j].z > mx[i].z + g || mx[j].z < mn[i].z - g)
                    continue;
                const rl::v3 vb[3] = {vert(t0 + j, 0), vert(t0 + j, 1), vert(t0 + j, 2)};
                rl::edge_connect(va, vb, info, arith);
            }
            float* d = &out[(size_t)(t0 + i) * 4];
            d[0] = info.a01;
            d[1] = info.a12;
            d[2] = info.a20;
            std::memcpy(&d[3], &info.flags, sizeof(int));
        }
        t0 += n;
    }
    return out;
}

}  // namespace rlgpu

extern "C" int rlgpu_cmf_parse(const void* data, int64_t size, float* out_tris, int32_t max_tris, int32_t* out_ntris,
                               int32_t* out_nverts, uint32_t* out_hash) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(data || size == 0, "rlgpu_cmf_parse: null data");
        RLGPU_REQUIRE(size >= 8, "Invalid collision mesh file (input data overflown)");
        const unsigned char* b = (const unsigned char*)data;
        int32_t nt, nv;
        std::memcpy(&nt, b, 4);
        std::memcpy(&nv, b + 4, 4);
        RLGPU_REQUIRE(!(std::min(nt, nv) <= 0 || std::max(nt, nv) > RLGPU_CMF_MAX_COUNT),
                      "Invalid collision mesh file (bad triangle/vertex count: [" + std::to_string(nt) + ", " +
                          std::to_string(nv) + "])");
        const int64_t need = 8 + (int64_t)nt * 12 + (int64_t)nv * 12;
        RLGPU_REQUIRE(size >= need, "Invalid collision mesh file (input data overflown by " +
                                        std::to_string(need - size) + " bytes!)");
        std::vector<int32_t> idx((size_t)nt * 3);
        std::vector<float> verts((size_t)nv * 3);
        std::memcpy(idx.data(), b + 8, idx.size() * 4);
        std::memcpy(verts.data(), b + 8 + (size_t)nt * 12, verts.size() * 4);
        for (int32_t v : idx)
            RLGPU_REQUIRE(v >= 0 && v < nv, "Invalid collision mesh file (bad triangle vertex index)");
        if (out_ntris) *out_ntris = nt;
        if (out_nverts) *out_nverts = nv;
        if (out_hash) *out_hash = rlgpu::cmf_hash(idx.data(), nt, verts.data(), nv);
        if (out_tris) {
            int32_t n = nt < max_tris ? nt : max_tris;
            for (int32_t t = 0; t < n; t++)
                for (int i = 0; i < 3; i++)
                    for (int j = 0; j < 3; j++) out_tris[(size_t)t * 9 + i * 3 + j] = verts[(size_t)idx[(size_t)t * 3 + i] * 3 + j];
        }
    });
}

extern "C" int rlgpu_mesh_edge_info(const float* tris, int32_t ntris, const int32_t* object_ntris, int32_t nobjects,
                                    int32_t arith, float* out) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(tris && out && ntris > 0, "rlgpu_mesh_edge_info: null argument or no triangles");
        RLGPU_REQUIRE(arith >= 0 && arith < RLGPU_NUM_ARITH, "rlgpu_mesh_edge_info: unknown arithmetic mode");
        if (object_ntris) {
            RLGPU_REQUIRE(nobjects >= 1, "rlgpu_mesh_edge_info: nobjects must be >= 1");
            int64_t sum = 0;
            for (int k = 0; k < nobjects; k++) {
                RLGPU_REQUIRE(object_ntris[k] >= 0, "rlgpu_mesh_edge_info: negative object triangle count");
                sum += object_ntris[k];
            }
            RLGPU_REQUIRE(sum == ntris, "rlgpu_mesh_edge_info: object triangle counts do not add up to ntris");
        }
        const std::vector<float> e = rlgpu::mesh_edge_info(tris, ntris, object_ntris, object_ntris ? nobjects : 1, arith);
        std::memcpy(out, e.data(), e.size() * sizeof(float));
    });
}

extern "C" int rlgpu_mesh_bvh_order(const float* tris, int32_t ntris, const int32_t* object_ntris, int32_t nobjects,
                                    int32_t* out) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(out, "rlgpu_mesh_bvh_order: null argument");
        const rlgpu::MeshGrid g = rlgpu::build_mesh_grid(tris, ntris, object_ntris, nobjects, RLGPU_ARITH_SCALAR);
        std::copy(g.visit_tri.begin(), g.visit_tri.end(), out);
    });
}

extern "C" int rlgpu_mesh_known_hash(int32_t game_mode, uint32_t hash) {
    const uint32_t* list = nullptr;
    int n = 0;
    if (game_mode == RLGPU_GAMEMODE_SOCCAR) {
        list = rlgpu::kSoccarHashes;
        n = (int)(sizeof(rlgpu::kSoccarHashes) / sizeof(uint32_t));
    } else if (game_mode == RLGPU_GAMEMODE_HOOPS) {
        list = rlgpu::kHoopsHashes;
        n = (int)(sizeof(rlgpu::kHoopsHashes) / sizeof(uint32_t));
    }
    for (int i = 0; i < n; i++)
        if (list[i] == hash) return i;
    return -1;
}
