// env_device.hpp -- per-arena device functions of the env kernel (see env_kernel.hpp).
// Every function cites the reference code it restates; the operation order matches the
// CPU oracle so strict-FP builds agree bit for bit.
#pragma once
#include "env_kernel.hpp"

namespace rl {

// the env set constants (make_env_const): one copy per translation unit, each uploaded by env.hip
// (ensure_const: its own for the test kernels, the specialised env kernels' through env_kN_upload)
static __constant__ EnvConst C;

#define DEV __device__ __forceinline__

// ------------------------------------------------------------------ state accessors
DEV v3 ld3(const float* p) { return v3{p[0], p[1], p[2]}; }
DEV void st3(float* p, v3 v) {
    p[0] = v.x;
    p[1] = v.y;
    p[2] = v.z;
}
DEV m3 ldm(const float* p) { return m3{v3{p[0], p[1], p[2]}, v3{p[3], p[4], p[5]}, v3{p[6], p[7], p[8]}}; }
DEV void stm(float* p, const m3& m) {
    p[0] = m.r0.x; p[1] = m.r0.y; p[2] = m.r0.z;
    p[3] = m.r1.x; p[4] = m.r1.y; p[5] = m.r1.z;
    p[6] = m.r2.x; p[7] = m.r2.y; p[8] = m.r2.z;
}
DEV rlgpu_body* body(ArenaLDS* A, int i) { return i == 0 ? &A->s.ball : &A->s.cars[i - 1].body; }
DEV v3 bpos(ArenaLDS* A, int i) { return ld3(body(A, i)->pos); }
DEV v3 bvel(ArenaLDS* A, int i) { return ld3(body(A, i)->vel); }
DEV v3 bang(ArenaLDS* A, int i) { return ld3(body(A, i)->angvel); }
DEV m3 brot(ArenaLDS* A, int i) { return ldm(body(A, i)->rot); }
// the set's RLGPU_ARITH_* mode: a constant in the specialised env kernels (env_step.hpp), else the arena's
#ifdef RLGPU_ENV_ARITH
DEV int arith(const ArenaLDS*) { return RLGPU_ENV_ARITH; }
#else
DEV int arith(const ArenaLDS* A) { return A->a.arith; }
#endif
DEV float binv_mass(int i) { return i == 0 ? C.ball_inv_mass : C.car_inv_mass; }
DEV v3 binv_iner(int i) { return i == 0 ? C.ball_inv_inertia : C.car_inv_inertia; }
DEV v3 vel_at(ArenaLDS* A, int i, v3 rel) { return bvel(A, i) + cross(bang(A, i), rel); }
DEV void update_inertia(ArenaLDS* A, int i) {
    m3 r = brot(A, i);
    A->a.iiw[i] = scaled(r, binv_iner(i)) * transpose(r);
}
DEV void apply_central_impulse(ArenaLDS* A, int i, v3 imp) {
    rlgpu_body* b = body(A, i);
    st3(b->vel, ld3(b->vel) + imp * binv_mass(i));
}
DEV void apply_impulse(ArenaLDS* A, int i, v3 imp, v3 rel) {
    if (binv_mass(i) != 0.f) {
        apply_central_impulse(A, i, imp);
        rlgpu_body* b = body(A, i);
        st3(b->angvel, ld3(b->angvel) + A->a.iiw[i] * cross(rel, imp));
    }
}
DEV float impulse_denominator(ArenaLDS* A, int i, v3 pos_w, v3 n) {
    v3 r0 = pos_w - bpos(A, i);
    v3 c0 = cross(r0, n);
    v3 vec = cross(vmul(c0, A->a.iiw[i]), r0);
    return binv_mass(i) + dot(n, vec);
}
DEV void add_force(ArenaLDS* A, int i, v3 f) { A->a.force[i] = A->a.force[i] + f; }
DEV void add_torque(ArenaLDS* A, int i, v3 t) { A->a.torque[i] = A->a.torque[i] + t; }
DEV float clampf(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }
DEV float stdclamp(float v, float lo, float hi) { return v < lo ? lo : (hi < v ? hi : v); }  // std::clamp
DEV float stdmax(float a, float b) { return a < b ? b : a; }                                  // std::max
DEV float stdmin(float a, float b) { return b < a ? b : a; }                                  // std::min
DEV int sgn(float x) { return x > 0 ? 1 : (x < 0 ? -1 : 0); }                                  // RS_SGN

// ------------------------------------------------------------------ LinearPieceCurve (Math.cpp:5-34)
// The curves are compile-time constants (template arguments) of a fully unrolled lookup, so every
// knot is an immediate: no memory loads (the lookup used to walk knots in global memory, a
// dependent load chain per call, several calls per car per tick).
struct Curve {
    int n;
    float k[6], v[6];
};
// RLConst.h:342-437
constexpr Curve kSteerAngle = {6, {0, 500, 1000, 1500, 1750, 3000}, {0.53356f, 0.31930f, 0.18203f, 0.10570f, 0.08507f, 0.03454f}};
constexpr Curve kPowerslideSteer = {2, {0, 2500}, {0.39235f, 0.12610f}};
constexpr Curve kDriveTorque = {3, {0, 1400, 1410}, {1.0f, 0.1f, 0.0f}};
constexpr Curve kNonSticky = {3, {0, 0.7075f, 1}, {0.1f, 0.5f, 1.0f}};
constexpr Curve kLatFriction = {2, {0, 1}, {1.0f, 0.2f}};
constexpr Curve kLongFriction = {0, {}, {}};
constexpr Curve kHbLat = {1, {0}, {0.1f}};
constexpr Curve kHbLong = {2, {0, 1}, {0.5f, 0.9f}};
constexpr Curve kBallCarExtra = {4, {0, 500, 2300, 4600}, {0.65f, 0.65f, 0.55f, 0.30f}};
constexpr Curve kBumpGround = {3, {0, 1400, 2200}, {5.f / 6.f, 1100.f, 1530.f}};
constexpr Curve kBumpAir = {3, {0, 1400, 2200}, {5.f / 6.f, 1390.f, 1945.f}};
constexpr Curve kBumpUp = {3, {0, 1400, 2200}, {2.f / 6.f, 278.f, 417.f}};

template <const Curve& CV>
DEV float curve_out(float input, float def = 1.f) {
    if (CV.n == 0) return def;
    if (input <= CV.k[0]) return CV.v[0];
#pragma unroll
    for (int i = 1; i < 6; i++) {
        if (i < CV.n && CV.k[i] > input) {
            float range = CV.k[i] - CV.k[i - 1];
            float diff = CV.v[i] - CV.v[i - 1];
            float f = (input - CV.k[i - 1]) / range;
            return CV.v[i - 1] + diff * f;
        }
    }
    return CV.v[CV.n > 0 ? CV.n - 1 : 0];
}

// ------------------------------------------------------------------ Philox 4x32-10 (same as oracle)
DEV uint32_t philox0(uint64_t key, uint32_t c0, uint32_t c1) {
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
    uint32_t x0 = c0, x1 = c1, x2 = 0x9E3779B9u, x3 = 0x85EBCA6Bu;
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * x0, p1 = (uint64_t)0xCD9E8D57u * x2;
        uint32_t y0 = (uint32_t)(p1 >> 32) ^ x1 ^ k0, y1 = (uint32_t)p1, y2 = (uint32_t)(p0 >> 32) ^ x3 ^ k1,
                 y3 = (uint32_t)p0;
        x0 = y0;
        x1 = y1;
        x2 = y2;
        x3 = y3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return x0;
}
DEV uint32_t rng_next(ArenaLDS* A, uint64_t seed, int arena) { return philox0(seed, (uint32_t)arena, A->s.env.rng_counter++); }
// a uniform float in [0, 1) from the next draw (24 bits): RocketSim's RandFloat fraction e() / e.max()
DEV float rng_uniform(ArenaLDS* A, uint64_t seed, int arena) {
    return (float)(rng_next(A, seed, arena) >> 8) * (1.f / 16777216.f);
}

// ------------------------------------------------------------------ shapes / AABBs
DEV v3 car_box_center(ArenaLDS* A, int bi) { return bpos(A, bi) + brot(A, bi) * C.car_offset; }
DEV void body_aabb(int bi, v3 pos, const m3& rot, v3& mn, v3& mx) {
    if (bi == 0) {
        float m = C.ball_radius + 0.08f;
        mn = pos - v3{m, m, m};
        mx = pos + v3{m, m, m};
    } else {
        v3 center = pos + rot * C.car_offset;
        v3 e;
        e.x = fabsf(rot.r0.x) * C.car_half.x + fabsf(rot.r0.y) * C.car_half.y + fabsf(rot.r0.z) * C.car_half.z;
        e.y = fabsf(rot.r1.x) * C.car_half.x + fabsf(rot.r1.y) * C.car_half.y + fabsf(rot.r1.z) * C.car_half.z;
        e.z = fabsf(rot.r2.x) * C.car_half.x + fabsf(rot.r2.y) * C.car_half.y + fabsf(rot.r2.z) * C.car_half.z;
        mn = center - e;
        mx = center + e;
    }
}
DEV void broad_aabb(ArenaLDS* A, int bi, v3& mn, v3& mx) {
    v3 a0, a1, p0, p1;
    body_aabb(bi, bpos(A, bi), brot(A, bi), a0, a1);
    body_aabb(bi, A->a.pred_pos[bi], A->a.pred_rot[bi], p0, p1);
    mn = v3{stdmin(a0.x, p0.x) - 0.02f, stdmin(a0.y, p0.y) - 0.02f, stdmin(a0.z, p0.z) - 0.02f};
    mx = v3{stdmax(a1.x, p1.x) + 0.02f, stdmax(a1.y, p1.y) + 0.02f, stdmax(a1.z, p1.z) + 0.02f};
}
DEV bool aabb_overlap(v3 a0, v3 a1, v3 b0, v3 b1) {
    return !(a0.x > b1.x || a1.x < b0.x || a0.y > b1.y || a1.y < b0.y || a0.z > b1.z || a1.z < b0.z);
}

// ------------------------------------------------------------------ mesh grid queries
// cell of a coordinate along one axis: IEEE sub / mul / floor / min / max only, so host binning
// (mesh.hip) and device queries agree exactly; NaN maps to cell 0
DEV int grid_cell(float x, float o, float inv, int n) {
    float f = floorf((x - o) * inv);
    f = fminf(fmaxf(f, 0.f), (float)(n - 1));
    return (int)f;
}
constexpr int kGridBatch = 4;  // grid entries whose loads are issued together
constexpr int kRayBatch = 8;   // the same for a wheel ray's walk (one query per lane, the phase's longest chain)
constexpr int kGridRows = 4;   // (y, z) rows of a query walked as one sequence (more: row by row)
// Calls f(t, v0, v1, v2, obj) once for every triangle whose AABB overlaps [qmn, qmx] (the exact
// test of the linear scan it replaces), in no particular order.  A triangle is listed in every
// cell its AABB touches; it is visited only from the cell max(query lo, triangle lo) per axis,
// which lies in both cell ranges whenever the boxes overlap (grid_cell is monotone); every entry
// carries its cell (x | y << 8 | z << 16) for that rule.  Entries hold their triangle inline (no index
// indirection).  The walk is latency-bound (one dependent L2 round trip per batch): the cells x0..x1 of
// one (y, z) row are one contiguous entry range, the ranges of a query's rows (up to kGridRows: a wheel
// ray, a car or a ball at the usual cell size) are read with one round of loads and walked as one
// sequence, kGridBatch entries' loads issued before the first is tested, batches running across row ends.
// Entry i of the sequence goes to caller i % parts.
template <class F>
DEV void grid_entry(const MeshView& M, const float4 (&q)[3], v3 qmn, v3 qmx, int x0, int y0, int z0, F&& f) {
    const v3 v0 = v3{q[0].x, q[0].y, q[0].z}, v1 = v3{q[1].x, q[1].y, q[1].z}, v2 = v3{q[2].x, q[2].y, q[2].z};
    const int obj = __float_as_int(q[0].w), t = __float_as_int(q[1].w), cell = __float_as_int(q[2].w);
    const v3 tmn = v3{fminf(v0.x, fminf(v1.x, v2.x)), fminf(v0.y, fminf(v1.y, v2.y)), fminf(v0.z, fminf(v1.z, v2.z))};
    const v3 tmx = v3{fmaxf(v0.x, fmaxf(v1.x, v2.x)), fmaxf(v0.y, fmaxf(v1.y, v2.y)), fmaxf(v0.z, fmaxf(v1.z, v2.z))};
    if (!aabb_overlap(qmn, qmx, tmn, tmx)) return;
    const int vx = max(x0, grid_cell(tmn.x, M.ox, M.inv_cell, M.nx)), vy = max(y0, grid_cell(tmn.y, M.oy, M.inv_cell, M.ny)),
              vz = max(z0, grid_cell(tmn.z, M.oz, M.inv_cell, M.nz));
    if (cell != (vx | (vy << 8) | (vz << 16))) return;
    f(t, v0, v1, v2, obj);
}
template <int kBatch = kGridBatch, class F>
DEV void grid_query(const MeshView& M, v3 qmn, v3 qmx, int part, int parts, F&& f) {
    const int x0 = grid_cell(qmn.x, M.ox, M.inv_cell, M.nx), x1 = grid_cell(qmx.x, M.ox, M.inv_cell, M.nx);
    const int y0 = grid_cell(qmn.y, M.oy, M.inv_cell, M.ny), y1 = grid_cell(qmx.y, M.oy, M.inv_cell, M.ny);
    const int z0 = grid_cell(qmn.z, M.oz, M.inv_cell, M.nz), z1 = grid_cell(qmx.z, M.oz, M.inv_cell, M.nz);
    // every cell of the query inside the grid's empty box: no entries to walk (the same result, no loads)
    if (x0 >= M.empty[0] && x1 <= M.empty[1] && y0 >= M.empty[2] && y1 <= M.empty[3] && z0 >= M.empty[4] && z1 <= M.empty[5])
        return;
    const int nyr = y1 - y0 + 1, nrows = nyr * (z1 - z0 + 1);
    if (nrows > kGridRows) {  // a larger query: row by row, the sequence numbering continued across rows
        int seen = 0;
        for (int cz = z0; cz <= z1; cz++)
            for (int cy = y0; cy <= y1; cy++) {
                const int row = (cz * M.ny + cy) * M.nx;
                const int b = M.cell_start[row + x0], e = M.cell_start[row + x1 + 1];
                int k = b + ((part - seen % parts) + parts) % parts;
                seen += e - b;
                for (; k < e; k += kGridBatch * parts) {
                    float4 q[kGridBatch][3];
#pragma unroll
                    for (int j = 0; j < kGridBatch; j++) {  // past the range's end: the last entry again (not visited)
                        const float4* p = M.cell_tri + 3 * (size_t)min(k + j * parts, e - 1);
                        q[j][0] = p[0];
                        q[j][1] = p[1];
                        q[j][2] = p[2];
                    }
#pragma unroll
                    for (int j = 0; j < kGridBatch; j++) {
                        if (k + j * parts >= e) break;
                        grid_entry(M, q[j], qmn, qmx, x0, y0, z0, f);
                    }
                }
            }
        return;
    }
    // the rows' entry ranges, all loads issued together; c[r] = entries before row r in the sequence
    int b[kGridRows], c[kGridRows + 1];
    c[0] = 0;
#pragma unroll
    for (int r = 0; r < kGridRows; r++) {
        const bool live = r < nrows;
        const int rr = live ? r : 0;
        const int row = ((z0 + rr / nyr) * M.ny + (y0 + rr % nyr)) * M.nx;
        const int bb = M.cell_start[row + x0], ee = M.cell_start[row + x1 + 1];
        b[r] = bb;
        c[r + 1] = c[r] + (live ? ee - bb : 0);
    }
    const int total = c[kGridRows];
    for (int i = part; i < total; i += kBatch * parts) {
        float4 q[kBatch][3];
#pragma unroll
        for (int j = 0; j < kBatch; j++) {  // past the sequence's end: its last entry again (not visited)
            const int s = min(i + j * parts, total - 1);
            int e = b[0] + s;
#pragma unroll
            for (int r = 1; r < kGridRows; r++) e = s >= c[r] ? b[r] + (s - c[r]) : e;
            const float4* p = M.cell_tri + 3 * (size_t)e;
            q[j][0] = p[0];
            q[j][1] = p[1];
            q[j][2] = p[2];
        }
#pragma unroll
        for (int j = 0; j < kBatch; j++) {
            if (i + j * parts >= total) break;
            grid_entry(M, q[j], qmn, qmx, x0, y0, z0, f);
        }
    }
}

// ------------------------------------------------------------------ ray cast (btCollisionWorld::rayTest)
// btVector3::setInterpolate3 (btVector3.h:496-520): (1 - rt) * v0 + rt * v1
DEV v3 lerp3(v3 v0, v3 v1, float rt) {
    const float s = 1.f - rt;
    return v3{s * v0.x + rt * v1.x, s * v0.y + rt * v1.y, s * v0.z + rt * v1.z};
}
// btTriangleRaycastCallback::processTriangle (btRaycastCallback.cpp:35-117, ClosestRayResultCallback flags 0):
// the hit fraction of [from, to] on the triangle when it lies inside (with the edge tolerance) and is
// closer than `best` (or equal, when `tie`), else -1; n = the unit normal facing `from`
DEV float ray_tri(v3 v0, v3 v1, v3 v2, v3 from, v3 to, float best, bool tie, v3& n, int ar) {
    const v3 tn = cross(v1 - v0, v2 - v0);
    const float dist = dot(v0, tn);
    const float da = dot(tn, from) - dist, db = dot(tn, to) - dist;
    if (da * db >= 0.f) return -1.f;
    const float f = da / (da - db);
    if (!(f < best || (tie && f == best))) return -1.f;
    const float tol = len2(tn) * -0.0001f;
    const v3 pt = lerp3(from, to, f);
    const v3 v0p = v0 - pt, v1p = v1 - pt, v2p = v2 - pt;
    if (!(dot(cross(v0p, v1p), tn) >= tol && dot(cross(v1p, v2p), tn) >= tol && dot(cross(v2p, v0p), tn) >= tol))
        return -1.f;
    const v3 u = bt_normalize(tn, ar);  // triangleNormal.normalize() (btRaycastCallback.cpp:102)
    n = da <= 0.f ? -u : u;
    return f;
}
// btPlaneSpace1 (btVector3.h:1266-1294)
DEV void plane_space1(v3 n, v3& p, v3& q) {
    if (fabsf(n.z) > 0.7071067811865475244008443621048490f) {
        const float a = n.y * n.y + n.z * n.z, k = 1.f / sqrtf(a);
        p = v3{0.f, -n.z * k, n.y * k};
        q = v3{a * k, -n.x * p.z, n.x * p.y};
    } else {
        const float a = n.x * n.x + n.y * n.y, k = 1.f / sqrtf(a);
        p = v3{-n.y * k, n.x * k, 0.f};
        q = v3{-n.z * p.y, n.z * p.x, a * k};
    }
}
// a dynamic body's position in every cell's dynamic list (ties: creation order); env_contacts.hpp keeps the ranks
DEV int bp_key(const ArenaLDS* A, int b) { return A->s.env.bp_rank[b] * 8 + b; }  // list position (ties: creation)
// btCollisionWorld::rayTest of a wheel ray, first half: the closest hit among the static objects (mesh
// triangles, planes) into W.rc_*, and a cast job per dynamic body the ray may reach (wheel_casts runs them
// on all lanes; ray_cast_finish combines them in the cell list's order)
DEV void ray_cast_static(ArenaLDS* A, const MeshView& M, v3 from, v3 to, int self, int wheel, WheelT& W) {
    float best = 1.0f;
    int obj = -1;
    v3 nrm = zero3();
    v3 d = to - from;
    // the ray cell's static proxies in creation order (btRSBroadphase::rayTest, btRSBroadphase.cpp:325-336):
    // the mesh objects, then the planes, then the dynamic bodies; each object keeps a hit only when strictly
    // closer than the best so far (btTriangleRaycastCallback, the convex casts), so the first one wins a tie.
    // Mesh: segment AABB grown by a margin well above the edge-test tolerance (a triangle whose grown AABB
    // misses it cannot be hit); ties in f go to the lower triangle index = the earlier BVH visit position
    const float kRayCull = 0.1f;
    const v3 smin = v3{fminf(from.x, to.x) - kRayCull, fminf(from.y, to.y) - kRayCull, fminf(from.z, to.z) - kRayCull};
    const v3 smax = v3{fmaxf(from.x, to.x) + kRayCull, fmaxf(from.y, to.y) + kRayCull, fmaxf(from.z, to.z) + kRayCull};
    int best_t = -1;
    const int ar = arith(A);
    grid_query<kRayBatch>(M, smin, smax, 0, 1, [&](int t, v3 v0, v3 v1, v3 v2, int) {
        v3 n;
        const float f = ray_tri(v0, v1, v2, from, to, best, best_t >= 0 && t < best_t, n, ar);
        if (f < 0.f) return;
        best = f;
        best_t = t;
        obj = 10;
        nrm = n;
    });
    // planes: btStaticPlaneShape (normal, constant 0) at plane_p with the identity basis; the ray in its frame
    // (x - plane_p) gives the AABB from which processAllTriangles (btStaticPlaneShape.cpp:56-82) builds two
    // triangles, each through processTriangle
    for (int p = 0; p < 4; p++) {
        const v3 pn = C.plane_n[p], fl = from - C.plane_p[p], tl = to - C.plane_p[p];
        // an axis plane's triangles lie exactly in the plane (the normal coordinate of every vertex is 0, the
        // normal is +-C e_k), so processTriangle's dist_a / dist_b are C * fl_k / C * tl_k: unless fl_k and
        // tl_k have strictly opposite signs, dist_a * dist_b >= 0 and neither triangle can be hit
        const int ax = C.plane_axis[p];
        if (ax >= 0) {
            const float a = comp(fl, ax), b = comp(tl, ax);
            if (!((a < 0.f && b > 0.f) || (a > 0.f && b < 0.f))) continue;
        }
        const v3 amn = v3{tl.x < fl.x ? tl.x : fl.x, tl.y < fl.y ? tl.y : fl.y, tl.z < fl.z ? tl.z : fl.z};
        const v3 amx = v3{fl.x < tl.x ? tl.x : fl.x, fl.y < tl.y ? tl.y : fl.y, fl.z < tl.z ? tl.z : fl.z};
        const v3 he = (amx - amn) * 0.5f;
        const float radius = sqrtf(he.x * he.x + he.y * he.y + he.z * he.z);
        const v3 c = (amx + amn) * 0.5f;
        v3 t0, t1;
        plane_space1(pn, t0, t1);
        const v3 pc = c - pn * ((pn.x * c.x + pn.y * c.y + pn.z * c.z) - 0.f);
        const v3 ta = t0 * radius, tb = t1 * radius;
        const v3 ppp = (pc + ta) + tb, ppm = (pc + ta) - tb, pmm = (pc - ta) - tb, pmp = (pc - ta) + tb;
        v3 n;
        float f = ray_tri(ppp, ppm, pmm, fl, tl, best, false, n, ar);
        if (f >= 0.f) {
            best = f;
            obj = 10;
            nrm = n;
        }
        f = ray_tri(pmm, pmp, ppp, fl, tl, best, false, n, ar);
        if (f >= 0.f) {
            best = f;
            obj = 10;
            nrm = n;
        }
    }
    // the dynamic bodies of the ray's cell in the cell list's order (bp_key), the wheel's own car skipped
    // (ClosestRayResultCallback's ignore object): btSubsimplexConvexCast of the ray's point against the ball's
    // sphere or the car compound's box child (btCollisionWorld.cpp:277-310,339-400), kept when strictly closer
    // and its normal long enough.  A body is in the cells around its home cell (btRSBroadphase.cpp:182-200),
    // wider than any wheel ray, so every body within reach is listed; a body whose bounding sphere the
    // segment misses by more than the cast's tolerances cannot be hit and gets no job (the oracle casts
    // against every body: the env parity tests check that this skip is exact).  Jobs go in list order;
    // none after a fraction-0 static hit (btSingleRayCallback::process stops at fraction 0).
    W.rc_best = best;
    W.rc_obj = obj;
    W.rc_nrm = nrm;
    if (best == 0.f) return;
    int done = 0;
    for (int k = 0; k < 5; k++) {
        int bi = -1, key = 1 << 30;
        for (int c = 0; c < 5; c++)
            if (!(done >> c & 1) && bp_key(A, c) < key) {
                key = bp_key(A, c);
                bi = c;
            }
        done |= 1 << bi;
        if (bi == self) continue;
        const v3 c = bi == 0 ? bpos(A, 0) : car_box_center(A, bi);
        const float reach = bi == 0 ? C.ball_radius : len(C.car_half);
        const float t = fminf(fmaxf(dot(c - from, d) / fmaxf(dot(d, d), 1e-30f), 0.f), 1.f);
        if (len2(from + d * t - c) > (reach + 0.05f) * (reach + 0.05f)) continue;
        const int slot = atomicAdd(&A->u.wc.njob, 1);
        CastJob& J = A->u.wc.job[slot];
        J.wheel = (uint8_t)wheel;
        J.body = (uint8_t)bi;
    }
}
// the cast jobs of the workgroup's arenas (base, nvalid of them), dealt over all its lanes
DEV void wheel_casts(ArenaLDS* base, int nvalid) {
    int start[kArenas + 1];
    start[0] = 0;
#pragma unroll
    for (int a = 0; a < kArenas; a++) start[a + 1] = start[a] + (a < nvalid ? base[a].u.wc.njob : 0);
    for (int k = threadIdx.x; k < start[kArenas]; k += kWG) {
        int ar = 0;
#pragma unroll
        for (int j = 1; j < kArenas; j++) ar += k >= start[j] ? 1 : 0;
        int off = start[0];
#pragma unroll
        for (int j = 1; j < kArenas; j++) off = ar == j ? start[j] : off;
        ArenaLDS* A = base + ar;
        CastJob& J = A->u.wc.job[k - off];
        const WheelT& W = A->u.wt[J.wheel];
        const int bi = J.body;
        const v3 c = bi == 0 ? bpos(A, 0) : car_box_center(A, bi);
        // one inlined cast for both shapes (the sphere radius or the box half extents select its support);
        // the ray: the wheel's hard point to its contact point as first set (the target)
        const bool ball = bi == 0;
        float f = 0.f;
        v3 n = zero3();
        const bool hit = gjk::ray_convex_cast(W.hard_point, W.contact_point, ball ? C.ball_radius : 0.f,
                                              ball ? zero3() : C.car_half, brot(A, bi), c, arith(A), f, n);
        J.f = f;
        J.nx = n.x;
        J.ny = n.y;
        J.nz = n.z;
        J.hit = hit ? 1 : 0;
    }
}
// second half: this ray's cast results in list order (kept when strictly closer and the normal is long
// enough, none after a fraction-0 hit), then ClosestRayResultCallback's point and normal
DEV int ray_cast_finish(ArenaLDS* A, v3 from, v3 to, int wheel, const WheelT& W, v3& hit_point, v3& hit_normal) {
    float best = W.rc_best;
    int obj = W.rc_obj;
    v3 nrm = W.rc_nrm;
    const int ar = arith(A);
    const int nj = A->u.wc.njob;
    for (int s = 0; s < nj; s++) {
        const CastJob& J = A->u.wc.job[s];
        if (J.wheel != wheel || best == 0.f) continue;
        const v3 n = v3{J.nx, J.ny, J.nz};
        if (!J.hit || !(len2(n) > 0.0001f) || !(J.f < best)) continue;
        best = J.f;
        obj = J.body;
        nrm = bt_normalize(n, ar);  // castResult.m_normal.normalize()
    }
    if (obj < 0) return -1;
    hit_point = lerp3(from, to, best);  // ClosestRayResultCallback::addSingleResult
    hit_normal = bt_normalize(nrm, ar);  // btDefaultVehicleRaycaster::castRay (btDefaultVehicleRaycaster.cpp:47)
    if (obj >= 1 && obj <= 4 && !A->a.active[obj]) return -1;
    return obj;
}

// ------------------------------------------------------------------ vehicle, one wheel per lane
// btVehicleRL::updateWheelTransform + rayCast (btVehicleRL.cpp:64-207).  First half of the wheel phase (btVehicleRL::updateVehicle, btVehicleRL.cpp:64-190): the wheel's
// transform and its ray against the static objects, cast jobs for the dynamic bodies
DEV void wheel_phase(ArenaLDS* A, const MeshView& M, int ci, int i) {
    rlgpu_car& cs = A->s.cars[ci];
    WheelT& W = A->u.wt[ci * 4 + i];
    int bi = ci + 1;
    m3 R = brot(A, bi);
    v3 P = bpos(A, bi);
    W.hard_point = R * C.wheel_conn[i] + P;
    W.wheel_dir = R * v3{0, 0, -1};
    v3 axle = R * v3{0, -1, 0};
    v3 up = -W.wheel_dir;
    quat q = quat_axis_angle(up, cs.wheel_steer[i]);
    m3 steer = mat_from_quat(q, arith(A));
    W.wt_col1 = steer * (-axle);
    // rayCast
    W.in_contact = 0;
    W.contact_world = 0;
    float rest = C.wheel_rest[i], radius = C.wheel_radius[i], travel = C.susp_travel;
    float ray_len = rest + travel + radius - 0.05f;
    v3 source = W.hard_point;
    v3 target = source + W.wheel_dir * ray_len;
    W.contact_point = target;
    W.ground = -1;
    ray_cast_static(A, M, source, target, bi, ci * 4 + i, W);
}
// Second half of the wheel phase (after wheel_casts): the ray's hit, suspension, friction impulses
DEV void wheel_phase_b(ArenaLDS* A, int ci, int i) {
    rlgpu_car& cs = A->s.cars[ci];
    WheelT& W = A->u.wt[ci * 4 + i];
    int bi = ci + 1;
    m3 R = brot(A, bi);
    v3 P = bpos(A, bi);
    float rest = C.wheel_rest[i], radius = C.wheel_radius[i], travel = C.susp_travel;
    v3 hp, hn;
    int obj = ray_cast_finish(A, W.hard_point, W.contact_point, ci * 4 + i, W, hp, hn);
    v3 upv = col(R, 2);
    if (obj >= 0) {
        W.contact_point = hp;
        W.contact_normal = hn;
        W.in_contact = 1;
        W.contact_world = (obj == 10);
        W.ground = obj;
        float trace = dot(W.hard_point - W.contact_point, upv);
        W.susp_len = trace - radius;
        W.susp_len = stdclamp(W.susp_len, rest - travel, rest + travel);
        float denom = dot(W.contact_normal, upv);
        v3 relpos = W.contact_point - P;
        v3 va = vel_at(A, bi, relpos);
        float proj = dot(W.contact_normal, va);
        if (denom > 0.1f) {
            float inv = 1.f / denom;
            W.susp_rel_vel = proj * inv;
            W.clipped_inv = inv;
        } else {
            W.susp_rel_vel = 0.f;
            W.clipped_inv = 10.f;
        }
        if (obj == 10) {
            float thresh = (rest + radius) - 0.05f;
            if (trace < thresh) {
                float dist = trace - thresh;
                v3 rel1 = hp - P;
                v3 v1 = vel_at(A, bi, rel1);
                float rel_vel = dot(hn, v1);
                float pos_err = 0.2f * -dist / kTick;
                float vel_err = -(1.0f + 0.f) * rel_vel;
                float denom0 = impulse_denominator(A, bi, hp, hn);
                float jinv = 1.f / (denom0 + 0.f);
                float imp = pos_err * jinv + vel_err * jinv;
                imp = 0.f > imp ? 0.f : imp;
                cs.wheel_extra_pushback[i] = imp / 4;
            }
        }
    } else {
        W.susp_len = rest + travel;
        W.susp_rel_vel = 0.f;
        W.contact_normal = -W.wheel_dir;
        W.clipped_inv = 1.f;
        cs.wheel_extra_pushback[i] = 0.f;
    }
    // calcFrictionImpulses (btVehicleRL.cpp:308-369), tick-start velocities of a dynamic ground
    if (W.ground < 0) {
        W.impulse = zero3();
        return;
    }
    const float friction_scale = kCarMass / 3;
    v3 ax = W.wt_col1;
    v3 n = W.contact_normal;
    float pj = dot(ax, n);
    ax -= n * pj;
    ax = safe_normalized(ax);
    v3 fwd = safe_normalized(cross(n, ax));
    bool dyn = W.ground >= 0 && W.ground <= 4;
    int g = W.ground;
    float side;
    {
        v3 cp = W.contact_point;
        v3 rel1 = cp - P;
        v3 gcom = dyn ? bpos(A, g) : zero3();
        float g_inv_mass = dyn ? binv_mass(g) : 0.f;
        v3 g_iner = dyn ? binv_iner(g) : zero3();
        v3 rel2 = cp - gcom;
        v3 v1 = vel_at(A, bi, rel1);
        v3 v2 = dyn ? (A->a.snap_vel[g] + cross(A->a.snap_ang[g], rel2)) : zero3();
        v3 vel = v1 - v2;
        v3 aJ = transpose(R) * cross(rel1, ax);
        // static ground: identity rotation (bJ = cross(rel2, -ax) exactly); no select of a whole
        // matrix (a select of two 3x3 aggregates is lowered through a private-memory copy)
        v3 bJ = cross(rel2, -ax);
        if (dyn) bJ = transpose(brot(A, g)) * bJ;
        v3 m0 = C.car_inv_inertia * aJ;
        v3 m1 = g_iner * bJ;
        float adiag = C.car_inv_mass + dot(m0, aJ) + g_inv_mass + dot(m1, bJ);
        float jinv = 1.f / adiag;
        float rel_vel = dot(ax, vel);
        side = -0.2f * rel_vel * jinv;
    }
    float rolling;
    if (cs.wheel_engine_force[i] == 0.f) {
        if (cs.wheel_brake[i] != 0.f) {
            v3 car_rel = W.contact_point - P;
            v3 v1 = vel_at(A, bi, car_rel);
            v3 v2 = dyn ? (A->a.snap_vel[g] + cross(A->a.snap_ang[g], car_rel)) : zero3();
            float rel_vel = dot(v1 - v2, fwd);
            const float MAGIC = 113.73963f;
            rolling = stdclamp(-rel_vel * MAGIC, -cs.wheel_brake[i], cs.wheel_brake[i]);
        } else {
            rolling = 0.f;
        }
    } else {
        rolling = -cs.wheel_engine_force[i] / friction_scale;
    }
    v3 total = (fwd * rolling * cs.wheel_long_friction[i]) + (ax * side * cs.wheel_lat_friction[i]);
    W.impulse = total * friction_scale;
}

DEV v3 upwards_dir_from_wheels(ArenaLDS* A, int ci) {
    v3 sum = zero3();
    for (int i = 0; i < 4; i++)
        if (A->u.wt[ci * 4 + i].in_contact) sum += A->u.wt[ci * 4 + i].contact_normal;
    if (sum.x == 0 && sum.y == 0 && sum.z == 0) return col(brot(A, ci + 1), 2);
    return safe_normalized(sum);
}

// Car::_UpdateWheels (Car.cpp:330-475), in three parts so that the per-wheel friction runs one wheel per lane:
// update_wheels_pre (the car's lane: handbrake, throttle / brake, engine and brake forces, steer; the throttle
// for the friction lanes into A->a.real_throttle), wheel_friction (lane 4 car + wheel: the wheel's lateral and
// longitudinal friction, the loop body of Car.cpp's per-wheel loop, same operations) and update_wheels_post (the
// car's lane: the world-contact sticky force).  Every wheel's values depend only on the car state the pre part
// leaves and on its own wheel, so the split gives the sequential loop's bits.
DEV void update_wheels_pre(ArenaLDS* A, int ci, int nwc, float fwd_speed) {
    rlgpu_car& cs = A->s.cars[ci];
    const float* ctl = cs.controls;
    float abs_fwd = fabsf(fwd_speed);
    if (ctl[7] != 0.f)
        cs.handbrake_val += 5.f * kTick;
    else
        cs.handbrake_val -= 2.f * kTick;
    cs.handbrake_val = stdclamp(cs.handbrake_val, 0.f, 1.f);
    float real_throttle = ctl[0];
    float real_brake = 0;
    if (ctl[6] != 0.f && cs.boost > 0) real_throttle = 1;
    {
        float drive_scale = curve_out<kDriveTorque>(abs_fwd);
        float engine_throttle = real_throttle;
        if (ctl[7] != 0.f) {
        } else {
            float abs_throttle = fabsf(real_throttle);
            if (abs_throttle >= 0.001f) {
                if (abs_fwd > 25.f && sgn(real_throttle) != sgn(fwd_speed)) {
                    real_brake = 1;
                    if (abs_fwd > 0.01f) engine_throttle = 0;
                }
            } else {
                engine_throttle = 0;
                bool full_stop = abs_fwd < 25.f;
                real_brake = full_stop ? 1 : 0.15f;
            }
        }
        if (nwc < 3) drive_scale /= 4;
        float engine = engine_throttle * (kCarMass * 400.f * kUU2BT) * drive_scale;
        float brake = real_brake * (kCarMass * (14.25f + (1.f / 3.f)) * kUU2BT);
        for (int i = 0; i < 4; i++) {
            cs.wheel_engine_force[i] = engine;
            cs.wheel_brake[i] = brake;
        }
    }
    {
        float steer = curve_out<kSteerAngle>(abs_fwd);
        if (cs.handbrake_val != 0.f) steer += (curve_out<kPowerslideSteer>(abs_fwd) - steer) * cs.handbrake_val;
        steer *= ctl[1];
        cs.wheel_steer[0] = steer;
        cs.wheel_steer[1] = steer;
    }
    A->a.real_throttle[ci] = real_throttle;
}
DEV void wheel_friction(ArenaLDS* A, int ci, int i) {
    rlgpu_car& cs = A->s.cars[ci];
    const int bi = ci + 1;
    WheelT& W = A->u.wt[ci * 4 + i];
    if (W.ground < 0) return;
    const float real_throttle = A->a.real_throttle[ci];
    v3 P = bpos(A, bi), Vv = bvel(A, bi), Av = bang(A, bi);
    v3 lat_dir = W.wt_col1;
    v3 long_dir = cross(lat_dir, W.contact_normal);
    float fin = 0;
    v3 delta = W.hard_point - P;
    v3 cv = (cross(Av, delta) + Vv) * kBT2UU;
    float base = fabsf(dot(cv, lat_dir));
    if (base > 5) fin = base / (fabsf(dot(cv, long_dir)) + base);
    float lat = curve_out<kLatFriction>(fin);
    float lon = curve_out<kLongFriction>(fin);
    if (cs.handbrake_val != 0.f) {
        float hb = cs.handbrake_val;
        lat *= (curve_out<kHbLat>(fin) - 1) * hb + 1;
        lon *= (curve_out<kHbLong>(fin) - 1) * hb + 1;
    } else {
        lon = 1;
    }
    bool sticky = real_throttle != 0;
    if (!sticky) {
        float ns = curve_out<kNonSticky>(W.contact_normal.z);
        lat *= ns;
        lon *= ns;
    }
    cs.wheel_lat_friction[i] = lat;
    cs.wheel_long_friction[i] = lon;
}
DEV void update_wheels_post(ArenaLDS* A, int ci, float fwd_speed) {
    int bi = ci + 1;
    bool world_contact = false;
    for (int i = 0; i < 4; i++) world_contact |= A->u.wt[ci * 4 + i].contact_world != 0;
    if (world_contact) {
        const float real_throttle = A->a.real_throttle[ci];
        v3 up = upwards_dir_from_wheels(A, ci);
        bool full = (real_throttle != 0) || (fabsf(fwd_speed) > 25.f);
        float scale = 0.5f;
        if (full) scale += 1 - fabsf(up.z);
        add_force(A, bi, up * scale * (-650.f * kUU2BT) * kCarMass);
    }
}

// Car::_UpdateBoost (Car.cpp:477-505)
DEV void update_boost(ArenaLDS* A, int ci) {
    rlgpu_car& cs = A->s.cars[ci];
    int bi = ci + 1;
    bool boosting = cs.controls[6] != 0.f;
    if (cs.time_spent_boosting > 0) {
        if (!boosting && cs.time_spent_boosting >= 0.1f)
            cs.time_spent_boosting = 0;
        else
            cs.time_spent_boosting += kTick;
    } else {
        if (boosting) cs.time_spent_boosting = kTick;
    }
    if (cs.boost > 0 && cs.time_spent_boosting > 0) {
        cs.boost = stdmax(cs.boost - (100.f / 3) * kTick, 0.f);
        float accel = cs.is_on_ground ? (2975 / 3.f) : (3175 / 3.f);
        add_force(A, bi, accel * kUU2BT * col(brot(A, bi), 0) * kCarMass);
    }
    cs.boost = stdmin(cs.boost, 100.f);
}

// Car::_UpdateJump (Car.cpp:507-554)
DEV void update_jump(ArenaLDS* A, int ci, bool jump_pressed) {
    rlgpu_car& cs = A->s.cars[ci];
    int bi = ci + 1;
    const float JUMP_MIN = 0.025f, JUMP_MAX = 0.2f, PAD = 1 / 40.f;
    if (cs.is_on_ground && !cs.is_jumping) {
        if (cs.has_jumped && cs.jump_time < JUMP_MIN + PAD) {
        } else {
            cs.has_jumped = 0;
            cs.jump_time = 0;
        }
    }
    if (cs.is_jumping) {
        cs.is_jumping = (cs.jump_time < JUMP_MIN || (cs.controls[5] != 0.f && cs.jump_time < JUMP_MAX));
    } else if (cs.is_on_ground && jump_pressed) {
        cs.is_jumping = 1;
        cs.jump_time = 0;
        v3 f = col(brot(A, bi), 2) * (875.f / 3.f) * kUU2BT * kCarMass;
        apply_central_impulse(A, bi, f);
    }
    if (cs.is_jumping) {
        cs.has_jumped = 1;
        v3 total = col(brot(A, bi), 2) * (4375.f / 3.f);
        if (cs.jump_time < JUMP_MIN) total *= 0.62f;
        add_force(A, bi, total * kUU2BT * kCarMass);
    }
    if (cs.is_jumping || cs.has_jumped) cs.jump_time += kTick;
}

// Car::_UpdateAirTorque (Car.cpp:556-641)
DEV void update_air_torque(ArenaLDS* A, int ci, bool update_air_control) {
    rlgpu_car& cs = A->s.cars[ci];
    int bi = ci + 1;
    const float* ctl = cs.controls;
    m3 R = brot(A, bi);
    v3 dir_pitch = -col(R, 1), dir_yaw = col(R, 2), dir_roll = -col(R, 0);
    bool do_air = false;
    if (cs.is_flipping) cs.is_flipping = cs.has_flipped && cs.flip_time < 0.65f;
    if (cs.is_flipping) {
        v3 rel = ld3(cs.flip_rel_torque);
        if (!(rel.x == 0 && rel.y == 0 && rel.z == 0)) {
            float pitch_scale = 1;
            if (rel.y != 0 && ctl[2] != 0) {
                if (sgn(rel.y) == sgn(ctl[2])) {
                    pitch_scale = 1 - stdmin(fabsf(ctl[2]), 1.f);
                    do_air = true;
                }
            }
            rel.y *= pitch_scale;
            v3 dodge = rel * v3{260.f, 224.f, 0};
            add_torque(A, bi, (inverse(A->a.iiw[bi]) * R) * dodge);
        } else {
            do_air = true;
        }
    } else {
        do_air = true;
    }
    do_air &= !cs.is_auto_flipping;
    do_air &= update_air_control;
    if (do_air) {
        float pitch_scale = 1;
        v3 torque = zero3();
        if (ctl[2] != 0 || ctl[3] != 0 || ctl[4] != 0) {
            if (cs.is_flipping)
                pitch_scale = 0;
            else if (cs.has_flipped && cs.flip_time < 0.65f + 0.3f)
                pitch_scale = 0;
            torque = (ctl[2] * dir_pitch * pitch_scale * 130.f) + (ctl[3] * dir_yaw * 95.f) + (ctl[4] * dir_roll * 400.f);
        }
        v3 av = bang(A, bi);
        float damp_pitch = dot(dir_pitch, av) * 30.f * (1 - fabsf(do_air ? (ctl[2] * pitch_scale) : 0));
        float damp_yaw = dot(dir_yaw, av) * 20.f * (1 - fabsf(do_air ? ctl[3] : 0));
        float damp_roll = dot(dir_roll, av) * 50.f;
        v3 damping = (dir_yaw * damp_yaw) + (dir_pitch * damp_pitch) + (dir_roll * damp_roll);
        const float TORQUE_SCALE = (float)(2 * 3.14159265358979323846 / (1 << 16) * 1000);
        add_torque(A, bi, inverse(A->a.iiw[bi]) * (torque - damping) * TORQUE_SCALE);
    }
    if (ctl[0] != 0) add_force(A, bi, col(R, 0) * ctl[0] * (200 / 3.f) * kUU2BT * kCarMass);
}

// Car::_UpdateDoubleJumpOrFlip (Car.cpp:643-761)
DEV void update_double_jump_or_flip(ArenaLDS* A, int ci, bool jump_pressed, float fwd_speed) {
    rlgpu_car& cs = A->s.cars[ci];
    int bi = ci + 1;
    const float* ctl = cs.controls;
    if (cs.is_on_ground) {
        cs.has_double_jumped = 0;
        cs.has_flipped = 0;
        cs.air_time = 0;
        cs.air_time_since_jump = 0;
        cs.flip_time = 0;
    } else {
        cs.air_time += kTick;
        if (cs.has_jumped && !cs.is_jumping)
            cs.air_time_since_jump += kTick;
        else
            cs.air_time_since_jump = 0;
        if (jump_pressed && cs.air_time_since_jump < 1.25f) {
            float mag = fabsf(ctl[3]) + fabsf(ctl[2]) + fabsf(ctl[4]);
            bool flip_input = mag >= 0.5f;
            bool can_use = !cs.has_double_jumped && !cs.has_flipped;
            if (cs.is_auto_flipping) can_use = false;
            if (can_use) {
                if (flip_input) {
                    cs.flip_time = 0;
                    cs.has_flipped = 1;
                    cs.is_flipping = 1;
                    float ratio = fabsf(fwd_speed) / 2300.f;
                    v3 dodge = v3{-ctl[2], ctl[3] + ctl[4], 0};
                    if (fabsf(ctl[3] + ctl[4]) < 0.1f && fabsf(ctl[2]) < 0.1f)
                        dodge = zero3();
                    else
                        dodge = safe_normalized(dodge);
                    st3(cs.flip_rel_torque, v3{-dodge.y, dodge.x, 0});
                    if (fabsf(dodge.x) < 0.1f) dodge.x = 0;
                    if (fabsf(dodge.y) < 0.1f) dodge.y = 0;
                    if (!fuzzy_zero(dodge)) {
                        bool back;
                        if (fabsf(fwd_speed) < 100.0f)
                            back = dodge.x < 0.0f;
                        else
                            back = (dodge.x >= 0.0f) != (fwd_speed >= 0.0f);
                        v3 init = dodge * 500.f;
                        float max_x = back ? 2.5f : 1.f;
                        init.x *= ((max_x - 1) * ratio) + 1.f;
                        init.y *= ((1.9f - 1) * ratio) + 1.f;
                        if (back) init.x *= 16.f / 15.f;
                        v3 fdir = col(brot(A, bi), 0);
                        float ang = rs_atan2f(fdir.y, fdir.x);
                        float sa, ca;
                        rs_sincosf(ang, &sa, &ca);
                        v3 xdir = v3{ca, -sa, 0.f}, ydir = v3{sa, ca, 0.f};
                        v3 dv = v3{dot(init, xdir), dot(init, ydir), 0.f};
                        apply_central_impulse(A, bi, dv * kUU2BT * kCarMass);
                    }
                } else {
                    v3 f = col(brot(A, bi), 2) * (875.f / 3.f) * kUU2BT * kCarMass;
                    apply_central_impulse(A, bi, f);
                    cs.has_double_jumped = 1;
                }
            }
        }
    }
    if (cs.is_flipping) {
        cs.flip_time += kTick;
        if (cs.flip_time <= 0.65f) {
            rlgpu_body* b = body(A, bi);
            if (cs.flip_time >= 0.15f && (b->vel[2] < 0 || cs.flip_time < 0.21f)) b->vel[2] *= (1 - 0.35f);
        }
    } else if (cs.has_flipped) {
        cs.flip_time += kTick;
    }
}

// Car::_UpdateAutoFlip (Car.cpp:763-797)
DEV void update_auto_flip(ArenaLDS* A, int ci, bool jump_pressed) {
    rlgpu_car& cs = A->s.cars[ci];
    int bi = ci + 1;
    m3 m = brot(A, bi);
    if (jump_pressed && cs.world_contact && cs.world_contact_normal[2] > 0.70710678118654752440f) {
        float r0 = rs_atan2f(m.r2.y, m.r2.z);
        // btAsin (btScalar.h): clamp to [-1, 1], then asin
        const float ax = -m.r2.x;
        float pitch_raw = rs_asinf(ax < -1.f ? -1.f : (ax > 1.f ? 1.f : ax));
        if (fabsf(pitch_raw) == kHalfPi) r0 = r0 > 0 ? r0 - kPi : r0 + kPi;
        float roll = -r0;
        float abs_roll = fabsf(roll);
        if (abs_roll > 2.8f) {
            cs.auto_flip_timer = 0.4f * (abs_roll / (float)3.14159265358979323846);
            cs.auto_flip_torque_scale = (roll > 0) ? 1 : -1;
            cs.is_auto_flipping = 1;
            apply_central_impulse(A, bi, -col(m, 2) * 200.f * kUU2BT * kCarMass);
        }
    }
    if (cs.is_auto_flipping) {
        if (cs.auto_flip_timer <= 0) {
            cs.is_auto_flipping = 0;
            cs.auto_flip_timer = 0;
        } else {
            rlgpu_body* b = body(A, bi);
            st3(b->angvel, ld3(b->angvel) + col(m, 0) * 50.f * cs.auto_flip_torque_scale * kTick);
            cs.auto_flip_timer -= kTick;
        }
    }
}

// Car::_UpdateAutoRoll (Car.cpp:799-831)
DEV void update_auto_roll(ArenaLDS* A, int ci, int nwc) {
    rlgpu_car& cs = A->s.cars[ci];
    int bi = ci + 1;
    v3 gup = nwc > 0 ? upwards_dir_from_wheels(A, ci) : ld3(cs.world_contact_normal);
    v3 gdown = -gup;
    m3 R = brot(A, bi);
    v3 fwd = col(R, 0), right = col(R, 1);
    v3 cross_right = cross(gup, fwd);
    v3 cross_fwd = cross(gdown, cross_right);
    float rtf = 1 - stdclamp(dot(right, cross_right), 0.f, 1.f);
    float ftf = 1 - stdclamp(dot(fwd, cross_fwd), 0.f, 1.f);
    v3 tdr = fwd * (dot(right, gup) >= 0 ? -1.f : 1.f);
    v3 tdf = right * (dot(fwd, gup) >= 0 ? 1.f : -1.f);
    v3 tr = tdr * rtf, tf = tdf * ftf;
    add_force(A, bi, gdown * 100.f * kUU2BT * kCarMass);
    add_torque(A, bi, inverse(A->a.iiw[bi]) * (tf + tr) * 80.f);
}

// Car::_PreTickUpdate after the wheel phase (Car.cpp:86-131 + btVehicleRL::updateVehicleSecond), in two parts
// around the per-wheel friction lanes (wheel_friction): car_phase_a up to _UpdateWheels' per-wheel loop, car_phase_b
// from its world-contact force on.  The body's velocity and rotation do not change in between (the wheel forces
// go to the force accumulator), so car_phase_b's forward speed is car_phase_a's.
DEV float car_fwd_speed(ArenaLDS* A, int bi) { return dot(bvel(A, bi), col(brot(A, bi), 0)) * kBT2UU; }
DEV void car_phase_a(ArenaLDS* A, int ci) {
    rlgpu_car& cs = A->s.cars[ci];
    if (cs.is_demoed) return;
    int nwc = 0;
    for (int i = 0; i < 4; i++) {
        cs.wheel_contact[i] = (uint8_t)A->u.wt[ci * 4 + i].in_contact;
        nwc += A->u.wt[ci * 4 + i].in_contact;
    }
    cs.is_on_ground = nwc >= 3;
    update_wheels_pre(A, ci, nwc, car_fwd_speed(A, ci + 1));
}
DEV void car_phase(ArenaLDS* A, int ci) {
    rlgpu_car& cs = A->s.cars[ci];
    if (cs.is_demoed) return;
    int bi = ci + 1;
    float* ctl = cs.controls;
    bool jump_pressed = ctl[5] != 0.f && cs.last_controls[5] == 0.f;
    int nwc = 0;
    for (int i = 0; i < 4; i++) nwc += A->u.wt[ci * 4 + i].in_contact;
    float fwd_speed = car_fwd_speed(A, bi);
    update_wheels_post(A, ci, fwd_speed);
    if (nwc < 3)
        update_air_torque(A, ci, nwc == 0);
    else
        cs.is_flipping = 0;
    update_jump(A, ci, jump_pressed);
    update_auto_flip(A, ci, jump_pressed);
    update_double_jump_or_flip(A, ci, jump_pressed, fwd_speed);
    if (ctl[0] != 0.f && ((nwc > 0 && nwc < 4) || cs.world_contact)) update_auto_roll(A, ci, nwc);
    cs.world_contact = 0;
    for (int i = 0; i < 4; i++) {
        WheelT& W = A->u.wt[ci * 4 + i];
        if (W.in_contact) {
            float force = (C.wheel_rest[i] - W.susp_len) * 500.f * W.clipped_inv;
            float damp = (W.susp_rel_vel < 0) ? 25.f : 40.f;
            float sf = force - (damp * W.susp_rel_vel);
            sf *= C.wheel_force_scale[i];
            if (sf < 0) sf = 0;
            W.susp_rel_vel = sf;  // reuse: suspension force
        } else {
            W.susp_rel_vel = 0;
        }
    }
    // the suspension, then the friction impulses (apply_impulse each, in this order), accumulated in registers
    // and stored once: the same additions as eight read-modify-writes of the body's velocities in LDS
    if (binv_mass(bi) != 0.f) {
        rlgpu_body* b = body(A, bi);
        const v3 P = bpos(A, bi);
        const m3 iiw = A->a.iiw[bi];
        const float im = binv_mass(bi);
        v3 lin = ld3(b->vel), ang = ld3(b->angvel);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const WheelT& W = A->u.wt[ci * 4 + i];
            if (W.susp_rel_vel != 0) {
                const v3 off = W.contact_point - P;
                const float base = (W.susp_rel_vel * kTick) + cs.wheel_extra_pushback[i];
                const v3 imp = W.contact_normal * base;
                lin = lin + imp * im;
                ang = ang + iiw * cross(off, imp);
            }
        }
        const v3 up = col(brot(A, bi), 2);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const WheelT& W = A->u.wt[ci * 4 + i];
            if (!is_zero(W.impulse)) {
                const v3 off = W.contact_point - P;
                const float d = dot(up, off);
                const v3 rel = off - up * d;
                const v3 imp = W.impulse * kTick;
                lin = lin + imp * im;
                ang = ang + iiw * cross(rel, imp);
            }
        }
        st3(b->vel, lin);
        st3(b->angvel, ang);
    }
    update_boost(A, ci);
}

// ------------------------------------------------------------------ car state reset helpers
DEV void default_car(rlgpu_car& cs) {
    // CarState defaults (Car.h:17-100); wheel values and controls survive SetState
    float keep[24 + 8];
    for (int i = 0; i < 4; i++) {
        keep[i] = cs.wheel_steer[i];
        keep[4 + i] = cs.wheel_engine_force[i];
        keep[8 + i] = cs.wheel_brake[i];
        keep[12 + i] = cs.wheel_lat_friction[i];
        keep[16 + i] = cs.wheel_long_friction[i];
        keep[20 + i] = cs.wheel_extra_pushback[i];
    }
    for (int k = 0; k < 8; k++) keep[24 + k] = cs.controls[k];
    __builtin_memset(&cs, 0, sizeof(rlgpu_car));  // (no type-punned stores: they may be reordered)
    for (int i = 0; i < 4; i++) {
        cs.wheel_steer[i] = keep[i];
        cs.wheel_engine_force[i] = keep[4 + i];
        cs.wheel_brake[i] = keep[8 + i];
        cs.wheel_lat_friction[i] = keep[12 + i];
        cs.wheel_long_friction[i] = keep[16 + i];
        cs.wheel_extra_pushback[i] = keep[20 + i];
    }
    for (int k = 0; k < 8; k++) cs.controls[k] = keep[24 + k];
    cs.is_on_ground = 1;
    cs.boost = 100.f / 3.f;
    cs.ball_hit_tick = -1;
    cs.ball_hit_extra_tick = -1;
}

DEV void set_car_state(ArenaLDS* A, int ci, v3 pos_uu, const m3& rot, float boost, bool on_ground) {
    rlgpu_car& cs = A->s.cars[ci];
    default_car(cs);
    cs.boost = boost;
    cs.is_on_ground = on_ground;
    rlgpu_body* b = &cs.body;
    st3(b->pos, pos_uu * kUU2BT);
    stm(b->rot, rot);
    st3(b->vel, zero3());
    st3(b->angvel, zero3());
    update_inertia(A, ci + 1);
}

}  // namespace rl
