// rsim_ref.cpp -- ORACLE (test infrastructure only; never linked into the product).
//
// Scalar, one-arena-at-a-time C++ restatement of the reference hot path:
//   RocketSim arena step   GigaLearnCPP/RLGymCPP/RocketSim/src/Sim/Arena/Arena.cpp:716-812
//   car logic              .../Sim/Car/Car.cpp:58-833
//   vehicle                .../Sim/btVehicleRL/btVehicleRL.cpp:64-421
//   ball / pads            .../Sim/Ball/Ball.cpp:112-138, .../Sim/BoostPad/BoostPad.cpp:51-105,
//                          .../Sim/BoostPad/BoostPadGrid/BoostPadGrid.cpp:5-25
//   contact callbacks      Arena.cpp:218-427
//   Bullet subset          btDiscreteDynamicsWorld.cpp:325-437, btRigidBody.cpp:95-420,
//                          btSequentialImpulseConstraintSolver.cpp:440-1900 (the row functions and the
//                          LinearMath branches of the build selected by g_arith, rsim_math.hpp),
//                          btPersistentManifold.cpp:100-330, btManifoldResult.cpp:110-200,
//                          SphereTriangleDetector.cpp:88-240, btSphereBoxCollisionAlgorithm.cpp,
//                          btConvexPlaneCollisionAlgorithm.cpp:53-90, btContactConstraint.cpp:60-150
//   env                    GigaLearnCPP/RLGymCPP/src/RLGymCPP/EnvSet/EnvSet.cpp:113-354 + the plugin set
//                          of src/ExampleMain.cpp:46-226 (see env_ref.cpp)
//
// Parity status: UNPINNED by the reference (no tests, no runnable binary -- SURVEY.md 8c);
// pinned by known-answer tests of constants/tables/spawn poses (tests/test_env_oracle.py).
// Documented deviations from the reference (also in DESIGN.md):
//   * synthetic arena mesh (include/rlgpu_arena_mesh.h) by default; real .cmf meshes can be
//     loaded (World::set_mesh), one collision object per file;
//   * (box-triangle runs Bullet's GJK / EPA, gjk_ref.hpp; box-box btBoxBoxDetector, boxbox_ref.hpp;
//     mesh triangles are visited in the quantized BVH's order, bvh_ref.hpp)
//   * time-based deactivation (btRigidBody.h:531-545) is not modelled -- only the zero-velocity
//     ball sleep of Arena.cpp:722-727;
//   * pairs are processed in btRSBroadphase's order (per dynamic proxy: its statics, then its pairs with
//     later bodies), except that a cell's dynamic list is taken in body order rather than its insertion
//     history; wheels resting on another dynamic
//     body read that body's tick-start velocity (the reference's order is unordered_set order);
//   * transcendentals use include/rlgpu_detmath.h (shared with the kernels) instead of libm.
#include "rsim_ref.hpp"

#include <algorithm>
#include <cstring>

#include "../include/rlgpu_arena_mesh.h"
#include "../include/rlgpu_detmath.h"
#include "boxbox_ref.hpp"
#include "bvh_ref.hpp"
#include "gjk_ref.hpp"

namespace orc {

// diagnostics: box-triangle GJK queries and penetration-solver (EPA) calls on this thread
thread_local uint64_t gjk_evals[2] = {0, 0};

// ------------------------------------------------------------------ constants (RLConst.h)
const float UU_TO_BT = 1.f / 50.f;  // BulletLink.h:15
const float BT_TO_UU = 50.f;        // BulletLink.h:12
const float TICK_TIME = 1.f / 120.f;
const float CAR_MASS = 180.f;
const float BALL_MASS = CAR_MASS / 6.f;
const float BALL_RADIUS_UU = 91.25f;
const float GRAVITY_Z_UU = -650.f;

// ---------------------------------------------------------------- LinearPieceCurve (Math.cpp:5-34)
struct Curve {
    int n;
    float k[6], v[6];
    float out(float input, float def = 1.f) const {
        if (n == 0) return def;
        if (input <= k[0]) return v[0];
        for (int i = 1; i < n; i++) {
            if (k[i] > input) {
                float range = k[i] - k[i - 1];
                float diff = v[i] - v[i - 1];
                float f = (input - k[i - 1]) / range;
                return v[i - 1] + diff * f;
            }
        }
        return v[n - 1];
    }
};
// RLConst.h:342-437
const Curve STEER_ANGLE_FROM_SPEED = {6, {0, 500, 1000, 1500, 1750, 3000}, {0.53356f, 0.31930f, 0.18203f, 0.10570f, 0.08507f, 0.03454f}};
const Curve POWERSLIDE_STEER_ANGLE = {2, {0, 2500}, {0.39235f, 0.12610f}};
const Curve DRIVE_SPEED_TORQUE_FACTOR = {3, {0, 1400, 1410}, {1.0f, 0.1f, 0.0f}};
const Curve NON_STICKY_FRICTION_FACTOR = {3, {0, 0.7075f, 1}, {0.1f, 0.5f, 1.0f}};
const Curve LAT_FRICTION = {2, {0, 1}, {1.0f, 0.2f}};
const Curve LONG_FRICTION = {0, {}, {}};
const Curve HANDBRAKE_LAT_FRICTION_FACTOR = {1, {0}, {0.1f}};
const Curve HANDBRAKE_LONG_FRICTION_FACTOR = {2, {0, 1}, {0.5f, 0.9f}};
const Curve BALL_CAR_EXTRA_IMPULSE_FACTOR = {4, {0, 500, 2300, 4600}, {0.65f, 0.65f, 0.55f, 0.30f}};
const Curve BUMP_VEL_AMOUNT_GROUND = {3, {0, 1400, 2200}, {5.f / 6.f, 1100.f, 1530.f}};
const Curve BUMP_VEL_AMOUNT_AIR = {3, {0, 1400, 2200}, {5.f / 6.f, 1390.f, 1945.f}};
const Curve BUMP_UPWARD_VEL_AMOUNT = {3, {0, 1400, 2200}, {2.f / 6.f, 278.f, 417.f}};

// -------------------------------------------------------------------- static world
World::World(int arith_) : arith(arith_) {
    ball_radius = BALL_RADIUS_UU * UU_TO_BT;
    // btSphereShape::calculateLocalInertia (btSphereShape.cpp:61-65)
    float elem = 0.4f * BALL_MASS * ball_radius * ball_radius;
    ball_inv_inertia = V(1.f / elem, 1.f / elem, 1.f / elem);
    ball_inv_mass = 1.f / BALL_MASS;
    // Octane (CarConfig.cpp:20-70): box half extents through btBoxShape margin handling
    V hs = V(120.507f, 86.6994f, 38.6591f) * UU_TO_BT;
    V h(hs.x / 2.f, hs.y / 2.f, hs.z / 2.f);
    // btBoxShape(halfExtents) (btBoxShape.cpp:18-26): implicit = half - 0.04 (CONVEX_DISTANCE_MARGIN), then
    // setSafeMargin(half) (btConvexInternalShape.h:63-78) lowers the margin to 0.1 x the smallest half
    // extent when that is below 0.04 (Octane: 0.0386591) and btBoxShape::setMargin (btBoxShape.h:84-92)
    // moves the difference into the implicit dimensions
    const float m0 = 0.04f;
    V impl((h.x - m0), (h.y - m0), (h.z - m0));
    float mn_half = h[h.x < h.y ? (h.x < h.z ? 0 : 2) : (h.y < h.z ? 1 : 2)];  // btVector3::minAxis
    float safe = 0.1f * mn_half;
    car_margin = m0;
    if (safe < car_margin) {
        V with_m = impl + V(m0, m0, m0);
        car_margin = safe;
        impl = with_m - V(safe, safe, safe);
    }
    car_impl = impl;
    car_half = car_impl + V(car_margin, car_margin, car_margin);  // getHalfExtentsWithMargin
    car_offset = V(13.87566f, 0.f, 20.755f) * UU_TO_BT;
    float lx = 2.f * car_half.x, ly = 2.f * car_half.y, lz = 2.f * car_half.z;  // btBoxShape.cpp
    V inertia = V(ly * ly + lz * lz, lx * lx + lz * lz, lx * lx + ly * ly) * (CAR_MASS / 12.f);
    car_inv_inertia = V(1.f / inertia.x, 1.f / inertia.y, 1.f / inertia.z);
    car_inv_mass = 1.f / CAR_MASS;
    // wheels (Car.cpp:231-277)
    for (int i = 0; i < 4; i++) {
        bool front = i < 2, left = i % 2;
        float radius = front ? 12.50f : 15.00f;
        V off = front ? V(51.25f, 25.90f, 20.755f) : V(-33.75f, 29.50f, 20.755f);
        if (left) off.y *= -1;
        float rest = (front ? 38.755f : 37.055f) - 12.f;  // minus MAX_SUSPENSION_TRAVEL
        wheel_conn[i] = off * UU_TO_BT;
        wheel_rest[i] = rest * UU_TO_BT;
        wheel_radius[i] = radius * UU_TO_BT;
        wheel_force_scale[i] = front ? (36.f - (1.f / 4.f)) : (54.f + (1.f / 4.f) + (1.5f / 100.f));
    }
    susp_travel = ((12.f * UU_TO_BT) * 100.f) / 100.f;  // m_maxSuspensionTravelCm / 100
    // contact breaking thresholds (btCollisionShape.cpp:128-158, btCollisionDispatcher.cpp:76-80)
    ball_cbt = (float)((double)ball_radius + 0.08) * 0.02f;
    {
        V mn = car_offset - car_half, mx = car_offset + car_half;
        V c = (mn + mx) * 0.5f;
        float r = len(mx - mn) * 0.5f;
        car_cbt = (r + len(c)) * 0.02f;
    }
    gravity = V(0, 0, GRAVITY_Z_UU) * UU_TO_BT;
    // btPow(1 - 0.03, 1/120): constant per tick (btRigidBody.cpp:153-163); host libm, double
    ball_damp = (float)std::pow((double)(1.f - 0.03f), (double)TICK_TIME);
    // planes (Arena.cpp:1052-1100): normal, point
    plane_n[0] = V(0, 0, 1);
    plane_p[0] = V(0, 0, 0);
    plane_n[1] = V(0, 0, -1);
    plane_p[1] = V(0, 0, 2048) * UU_TO_BT;
    plane_n[2] = V(1, 0, 0);
    plane_p[2] = V(-4096, 0, 2048 / 2) * UU_TO_BT;
    plane_n[3] = V(-1, 0, 0);
    plane_p[3] = V(4096, 0, 2048 / 2) * UU_TO_BT;
    {
        std::vector<float> bt((size_t)RLGPU_MESH_TRIS * 9);
        for (int t = 0; t < RLGPU_MESH_TRIS; t++)
            for (int k = 0; k < 9; k++) bt[(size_t)t * 9 + k] = RLGPU_MESH_UU[t][k] * UU_TO_BT;
        set_mesh(bt.data(), RLGPU_MESH_TRIS, nullptr, 1);
    }
    // spawn / respawn rotations precomputed on the host (RLConst.h:297-338, Arena.cpp:183-186)
    const float spawn_x[5] = {-2048, 2048, -256, 256, 0}, spawn_y[5] = {-2560, -2560, -3840, -3840, -4608};
    const float spawn_yaw[5] = {(float)(M_PI_4 * 1), (float)(M_PI_4 * 3), (float)(M_PI_4 * 2), (float)(M_PI_4 * 2),
                                (float)(M_PI_4 * 2)};
    for (int i = 0; i < 5; i++) {
        kick_x[i] = spawn_x[i];
        kick_y[i] = spawn_y[i];
        kick_rot[0][i] = euler_ypr(spawn_yaw[i], -0.f, -0.f);
        kick_rot[1][i] = euler_ypr(spawn_yaw[i] + (float)M_PI, -0.f, -0.f);
    }
    const float rs_x[4] = {-2304, -2688, 2304, 2688};
    for (int i = 0; i < 4; i++) {
        respawn_x[i] = rs_x[i];
        respawn_y[i] = -4608;
        respawn_rot[0][i] = euler_ypr((float)(M_PI / 2) + 0.f, 0.f, 0.f);
        respawn_rot[1][i] = euler_ypr((float)(M_PI / 2) + (float)M_PI, 0.f, 0.f);
    }
    // pads: big 6 then small 28 (Arena.cpp:532-556)
    const float big[6][3] = {{-3584, 0, 73}, {3584, 0, 73}, {-3072, 4096, 73}, {3072, 4096, 73}, {-3072, -4096, 73}, {3072, -4096, 73}};
    const float small[28][3] = {{0, -4240, 70},    {-1792, -4184, 70}, {1792, -4184, 70}, {-940, -3308, 70},  {940, -3308, 70},
                                {0, -2816, 70},    {-3584, -2484, 70}, {3584, -2484, 70}, {-1788, -2300, 70}, {1788, -2300, 70},
                                {-2048, -1036, 70}, {0, -1024, 70},    {2048, -1036, 70}, {-1024, 0, 70},     {1024, 0, 70},
                                {-2048, 1036, 70}, {0, 1024, 70},      {2048, 1036, 70},  {-1788, 2300, 70},  {1788, 2300, 70},
                                {-3584, 2484, 70}, {3584, 2484, 70},   {0, 2816, 70},     {-940, 3308, 70},   {940, 3308, 70},
                                {-1792, 4184, 70}, {1792, 4184, 70},   {0, 4240, 70}};
    for (int i = 0; i < RLGPU_PADS; i++) {
        const float* p = i < 6 ? big[i] : small[i - 6];
        pad_pos_uu[i] = V(p[0], p[1], p[2]);
        pad_big[i] = i < 6;
        pad_pos_bt[i] = pad_pos_uu[i] * UU_TO_BT;
        float box_rad = (pad_big[i] ? 160.f : 120.f) * UU_TO_BT;  // BoostPad.cpp:44-48
        pad_box_min[i] = pad_pos_bt[i] - V(box_rad, box_rad, 0);
        pad_box_max[i] = pad_pos_bt[i] + V(box_rad, box_rad, 64.f * UU_TO_BT);
        pad_cell_x[i] = (int)(pad_pos_uu[i].x / 1024 + 4);  // BoostPadGrid.cpp:30-31
        pad_cell_y[i] = (int)(pad_pos_uu[i].y / 1024 + 5);
    }
}

void World::set_mesh(const float* p, int n, const int* obj_ntris, int nobjects) {
    ntris = n;
    nobj = obj_ntris ? nobjects : 1;
    tri.resize((size_t)n * 3);
    tri_min.resize(n);
    tri_max.resize(n);
    tri_obj.assign(n, 0);
    for (int t = 0; t < n; t++) {
        for (int k = 0; k < 3; k++) tri[(size_t)t * 3 + k] = V(p[t * 9 + 3 * k], p[t * 9 + 3 * k + 1], p[t * 9 + 3 * k + 2]);
        V mn = tri[(size_t)t * 3], mx = mn;
        for (int k = 1; k < 3; k++)
            for (int a = 0; a < 3; a++) {
                mn[a] = std::min(mn[a], tri[(size_t)t * 3 + k][a]);
                mx[a] = std::max(mx[a], tri[(size_t)t * 3 + k][a]);
            }
        tri_min[t] = mn;
        tri_max[t] = mx;
    }
    if (obj_ntris) {
        int t = 0;
        for (int k = 0; k < nobjects; k++)
            for (int i = 0; i < obj_ntris[k] && t < n; i++) tri_obj[t++] = k;
    }
    // btBvhTriangleMeshShape per object (RocketSim.cpp:167): the order its quantized BVH visits the triangles
    tri_visit.resize(n);
    obj_t0.assign(nobj, 0);
    obj_tree.assign(nobj, bvh::Tree());  // an object without triangles keeps an empty tree
    for (int t0 = 0; t0 < n;) {
        int t1 = t0;
        while (t1 < n && tri_obj[t1] == tri_obj[t0]) t1++;
        const int o = tri_obj[t0];
        std::vector<int> order = bvh::leaf_order(p + (size_t)t0 * 9, t1 - t0, &obj_tree[o]);
        for (int k = 0; k < t1 - t0; k++) tri_visit[t0 + k] = t0 + order[k];
        obj_t0[o] = t0;
        t0 = t1;
    }
    ArithScope scope(arith);
    tri_info = edge::gen_edge_info(tri, tri_obj, tri_visit);  // RocketSim.cpp:166-170
}

const World& world(int arith) {
    static const World w0(RLGPU_ARITH_MSVC_X64), w1(RLGPU_ARITH_GCC_X64), w2(RLGPU_ARITH_SCALAR);
    return arith == RLGPU_ARITH_SCALAR ? w2 : (arith == RLGPU_ARITH_GCC_X64 ? w1 : w0);
}

// ------------------------------------------------------------------ Philox 4x32-10
void philox(uint64_t key, uint32_t c0, uint32_t c1, uint32_t out[4]) {
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
    out[0] = x0;
    out[1] = x1;
    out[2] = x2;
    out[3] = x3;
}

uint32_t rng_next(uint64_t seed, int arena, rlgpu_env_extra& env) {
    uint32_t o[4];
    philox(seed, (uint32_t)arena, env.rng_counter++, o);
    return o[0];
}

// Working copy of a rigid body during a tick (btRigidBody subset).
struct Body {
    V pos, vel, ang, force, torque;
    M rot, inv_inertia_world;
    V inv_inertia_local;
    float inv_mass;
    bool no_rot, active, present;
    V pred_pos;  // interpolation transform (predictUnconstraintMotion) -> broadphase AABB
    M pred_rot;
    void update_inertia() { inv_inertia_world = scaled(rot, inv_inertia_local) * transpose(rot); }
    V vel_at(V rel) const { return vel + cross(ang, rel); }  // getVelocityInLocalPoint
    void apply_central_impulse(V imp) { vel += imp * inv_mass; }
    void apply_torque_impulse(V t) { ang += inv_inertia_world * t; }
    void apply_impulse(V imp, V rel) {
        if (inv_mass != 0.f) {
            apply_central_impulse(imp);
            apply_torque_impulse(cross(rel, imp));
        }
    }
    float impulse_denominator(V pos_w, V n) const {  // btRigidBody::computeImpulseDenominator
        V r0 = pos_w - pos;
        V c0 = cross(r0, n);
        V vec = cross(vmul(c0, inv_inertia_world), r0);
        return inv_mass + dot(n, vec);
    }
};

// ---------------------------------------------------------------- arena working set
struct Sim {
    const World& w;
    rlgpu_arena_state& s;
    uint64_t seed;
    int arena_index;
    Body b[5];  // 0 ball, 1..4 cars
    // per-tick transient vehicle data
    struct WheelTick {
        V hard_point, wheel_dir, axle, contact_point, contact_normal, wt_col1;
        float susp_len, susp_rel_vel, clipped_inv, susp_force;
        bool in_contact, contact_world;
        int ground;  // -1 none, 0 ball, 1..4 cars, 10 static
        V impulse;
    } wt[4][4];
    Body snap[5];  // tick-start snapshot for wheel-on-dynamic-body friction
    // event sink for the env layer
    bool ev_bump[4], ev_demo[4];

    Sim(const World& w_, rlgpu_arena_state& s_, uint64_t seed_, int idx) : w(w_), s(s_), seed(seed_), arena_index(idx) {}

    rlgpu_car& car(int i) { return s.cars[i]; }  // i = 0..3
    static bool car_team_orange(int i) { return i & 1; }  // creation order B,O,B,O (ExampleMain.cpp:204-208)
    static uint32_t car_id(int i) { return (uint32_t)(i + 1); }

    void load_bodies() {
        const World& W = w;
        Body& ball = b[0];
        ball.pos = ld3(s.ball.pos);
        ball.rot = ldm(s.ball.rot);
        ball.vel = ld3(s.ball.vel);
        ball.ang = ld3(s.ball.angvel);
        ball.inv_mass = W.ball_inv_mass;
        ball.inv_inertia_local = W.ball_inv_inertia;
        ball.no_rot = true;
        ball.present = true;
        ball.force = ball.torque = V();
        ball.update_inertia();
        for (int i = 0; i < 4; i++) {
            Body& c = b[i + 1];
            rlgpu_car& cs = car(i);
            c.pos = ld3(cs.body.pos);
            c.rot = ldm(cs.body.rot);
            c.vel = ld3(cs.body.vel);
            c.ang = ld3(cs.body.angvel);
            c.inv_mass = W.car_inv_mass;
            c.inv_inertia_local = W.car_inv_inertia;
            c.no_rot = false;
            c.present = true;
            c.force = c.torque = V();
            c.update_inertia();
        }
    }
    void store_bodies() {
        st3(s.ball.pos, b[0].pos);
        stm(s.ball.rot, b[0].rot);
        st3(s.ball.vel, b[0].vel);
        st3(s.ball.angvel, b[0].ang);
        for (int i = 0; i < 4; i++) {
            rlgpu_car& cs = car(i);
            st3(cs.body.pos, b[i + 1].pos);
            stm(cs.body.rot, b[i + 1].rot);
            st3(cs.body.vel, b[i + 1].vel);
            st3(cs.body.angvel, b[i + 1].ang);
        }
    }

    // -------------------------------------------------------------- shapes / AABBs
    V car_box_center(int bi) const { return b[bi].pos + b[bi].rot * w.car_offset; }
    void body_aabb(int bi, V pos, const M& rot, V& mn, V& mx) const {
        if (bi == 0) {
            float m = w.ball_radius + 0.08f;  // btSphereShape.cpp:55 (RocketSim change)
            mn = pos - V(m, m, m);
            mx = pos + V(m, m, m);
        } else {  // btCompoundShape::getAabb
            V center = pos + rot * w.car_offset;
            V e;
            for (int r = 0; r < 3; r++)
                e[r] = std::fabs(rot.r[r].x) * w.car_half.x + std::fabs(rot.r[r].y) * w.car_half.y +
                       std::fabs(rot.r[r].z) * w.car_half.z;
            mn = center - e;
            mx = center + e;
        }
    }
    // broadphase AABB: current + predicted transform, expanded by gContactBreakingThreshold
    void broad_aabb(int bi, V& mn, V& mx) const {
        V a0, a1, p0, p1;
        body_aabb(bi, b[bi].pos, b[bi].rot, a0, a1);
        body_aabb(bi, b[bi].pred_pos, b[bi].pred_rot, p0, p1);
        for (int k = 0; k < 3; k++) {
            mn[k] = std::min(a0[k], p0[k]) - 0.02f;
            mx[k] = std::max(a1[k], p1[k]) + 0.02f;
        }
    }

    // ---------------------------------------------------------------- ray tests
    // btVector3::setInterpolate3 (btVector3.h:496-520)
    static V interpolate3(V v0, V v1, float rt) {
        const float s = 1.f - rt;
        return V(s * v0.x + rt * v1.x, s * v0.y + rt * v1.y, s * v0.z + rt * v1.z);
    }
    // btTriangleRaycastCallback::processTriangle (btRaycastCallback.cpp:35-117), flags 0: the fraction of a
    // hit inside the triangle (edge tolerance) strictly closer than `best`, else -1; n faces `from`
    static float ray_triangle(const V& v0, const V& v1, const V& v2, V from, V to, float best, V& n) {
        const V tn = cross(v1 - v0, v2 - v0);
        const float dist = dot(v0, tn);
        const float da = dot(tn, from) - dist;
        const float db = dot(tn, to) - dist;
        if (da * db >= 0.f) return -1.f;
        const float f = da / (da - db);
        if (!(f < best)) return -1.f;
        const float tol = len2(tn) * -0.0001f;
        const V pt = interpolate3(from, to, f);
        const V v0p = v0 - pt, v1p = v1 - pt;
        if (!(dot(cross(v0p, v1p), tn) >= tol)) return -1.f;
        const V v2p = v2 - pt;
        if (!(dot(cross(v1p, v2p), tn) >= tol)) return -1.f;
        const V cp2 = cross(v2p, v0p);
        if (!(dot(cp2, tn) >= tol)) return -1.f;
        const V u = bt_normalize(tn);  // triangleNormal.normalize()
        n = da <= 0.f ? -u : u;
        return f;
    }
    // Closest hit of segment [from,to] against the world (btCollisionWorld::rayTest +
    // ClosestRayResultCallback), ignoring body `self`.  Returns hit object id:
    // -1 none, 0 ball, 1..4 car, 10 static.  (btDefaultVehicleRaycaster.cpp:32-52)
    int ray_cast(V from, V to, int self, V& hit_point, V& hit_normal, float& frac) {
        float best = 1.0f;
        int obj = -1;
        V nrm;
        // the ray cell's statics in creation order (btRSBroadphase::rayTest): mesh objects, then planes;
        // every object keeps a hit only when strictly closer, so the first one wins a tie
        // mesh triangles in BVH visit order (btBvhTriangleMeshShape::performRaycast ->
        // walkStacklessQuantizedTreeAgainstRay), objects in creation order; the walk is pruned by the
        // segment's box grown by 0.1 (more than the edge tolerance can reach outside a triangle)
        const V rmn(std::min(from.x, to.x) - 0.1f, std::min(from.y, to.y) - 0.1f, std::min(from.z, to.z) - 0.1f);
        const V rmx(std::max(from.x, to.x) + 0.1f, std::max(from.y, to.y) + 0.1f, std::max(from.z, to.z) + 0.1f);
        for (size_t o = 0; o < w.obj_tree.size(); o++)
            w.obj_tree[o].walk(rmn, rmx, [&](int k) {
                const int t = w.tri_visit[w.obj_t0[o] + k];
                V n;
                const float f = ray_triangle(w.tri[(size_t)t * 3], w.tri[(size_t)t * 3 + 1], w.tri[(size_t)t * 3 + 2],
                                             from, to, best, n);
                if (f >= 0.f) {
                    best = f;
                    obj = 10;
                    nrm = n;
                }
            });
        // static planes: btStaticPlaneShape(normal, 0) at plane_p (identity basis); processAllTriangles
        // (btStaticPlaneShape.cpp:56-82) spans two triangles over the ray's AABB in the plane's frame
        for (int p = 0; p < 4; p++) {
            const V pn = w.plane_n[p], fl = from - w.plane_p[p], tl = to - w.plane_p[p];
            V amn = fl, amx = fl;
            for (int a = 0; a < 3; a++) {
                if (tl[a] < amn[a]) amn[a] = tl[a];  // btSetMin
                if (amx[a] < tl[a]) amx[a] = tl[a];  // btSetMax
            }
            const V he = (amx - amn) * 0.5f;
            const float radius = std::sqrt(he.x * he.x + he.y * he.y + he.z * he.z);  // length()
            const V c = (amx + amn) * 0.5f;
            V t0, t1;
            if (std::fabs(pn.z) > 0.7071067811865475244008443621048490f) {  // btPlaneSpace1
                const float a = pn.y * pn.y + pn.z * pn.z, k = 1.f / std::sqrt(a);
                t0 = V(0.f, -pn.z * k, pn.y * k);
                t1 = V(a * k, -pn.x * t0.z, pn.x * t0.y);
            } else {
                const float a = pn.x * pn.x + pn.y * pn.y, k = 1.f / std::sqrt(a);
                t0 = V(-pn.y * k, pn.x * k, 0.f);
                t1 = V(-pn.z * t0.y, pn.z * t0.x, a * k);
            }
            const V pc = c - pn * ((pn.x * c.x + pn.y * c.y + pn.z * c.z) - 0.f);
            const V ta = t0 * radius, tb = t1 * radius;
            const V tri[2][3] = {{(pc + ta) + tb, (pc + ta) - tb, (pc - ta) - tb}, {(pc - ta) - tb, (pc - ta) + tb, (pc + ta) + tb}};
            for (int q = 0; q < 2; q++) {
                V n;
                const float f = ray_triangle(tri[q][0], tri[q][1], tri[q][2], fl, tl, best, n);
                if (f >= 0.f) {
                    best = f;
                    obj = 10;
                    nrm = n;
                }
            }
        }
        // the dynamic bodies of the ray's cell in the cell list's order (list_key), the wheel's own car skipped
        // (ClosestRayResultCallback's ignore object): btSubsimplexConvexCast of the ray's point against the ball's
        // sphere or the car compound's box child (childWorldTrans = the body's transform * the hitbox offset,
        // btCollisionWorld.cpp:339-400 without a dynamic AABB tree), kept when strictly closer and its normal is
        // long enough (btCollisionWorld.cpp:285-307).  Every dynamic within reach is in the cell's list: a body
        // sits in the 3x3x3 cells around its home cell (btRSBroadphase.cpp:182-200), wider than any wheel ray.
        int order[5] = {0, 1, 2, 3, 4};
        std::sort(order, order + 5, [&](int x, int y) { return list_key(x) < list_key(y); });
        for (int k = 0; k < 5; k++) {
            const int bi = order[k];
            if (bi == self || best == 0.f) continue;  // btSingleRayCallback::process stops at fraction 0
            float f;
            V n;
            const bool hit = bi == 0 ? gjk::ray_convex_cast(from, to, w.ball_radius, V(), b[0].rot, b[0].pos, f, n)
                                     : gjk::ray_convex_cast(from, to, 0.f, w.car_half, b[bi].rot, car_box_center(bi), f, n);
            if (!hit || !(len2(n) > 0.0001f) || !(f < best)) continue;
            best = f;
            obj = bi;
            nrm = bt_normalize(n);  // castResult.m_normal.normalize()
        }
        if (obj < 0) return -1;
        frac = best;
        hit_point = interpolate3(from, to, best);  // ClosestRayResultCallback: setInterpolate3
        hit_normal = bt_normalize(nrm);
        if (obj >= 1 && obj <= 4 && !b[obj].active) return -1;  // CF_NO_CONTACT_RESPONSE
        return obj;
    }

    // ------------------------------------------------------------------ vehicle
    // btVehicleRL::updateWheelTransform / updateWheelTransformsWS (btVehicleRL.cpp:64-113)
    void wheel_transforms(int ci) {
        Body& c = b[ci + 1];
        rlgpu_car& cs = car(ci);
        for (int i = 0; i < 4; i++) {
            WheelTick& W = wt[ci][i];
            W.hard_point = c.rot * w.wheel_conn[i] + c.pos;
            W.wheel_dir = c.rot * V(0, 0, -1);
            W.axle = c.rot * V(0, -1, 0);
            V up = -W.wheel_dir;
            V right = W.axle;
            Q q = quat_axis_angle(up, cs.wheel_steer[i]);
            M steer = mat_from_quat(q);
            // basis2 column 1 (right axis) = -right; column 1 of steer*basis2 = steer * (-right)
            W.wt_col1 = steer * (-right);
        }
    }

    // btVehicleRL::rayCast (btVehicleRL.cpp:118-207)
    void wheel_ray(int ci, int i) {
        Body& c = b[ci + 1];
        rlgpu_car& cs = car(ci);
        WheelTick& W = wt[ci][i];
        W.in_contact = false;
        W.contact_world = false;
        float rest = w.wheel_rest[i], radius = w.wheel_radius[i], travel = w.susp_travel;
        float ray_len = rest + travel + radius - 0.05f;
        V source = W.hard_point;
        V target = source + W.wheel_dir * ray_len;
        W.contact_point = target;
        W.ground = -1;
        V hp, hn;
        float frac = 1.f;
        int obj = ray_cast(source, target, ci + 1, hp, hn, frac);
        V upv = c.rot.col(2);
        if (obj >= 0) {
            W.contact_point = hp;
            W.contact_normal = hn;
            W.in_contact = true;
            W.contact_world = (obj == 10);
            W.ground = obj;
            float trace = dot(W.hard_point - W.contact_point, upv);
            W.susp_len = trace - radius;
            W.susp_len = std::clamp(W.susp_len, rest - travel, rest + travel);
            float denom = dot(W.contact_normal, upv);
            V relpos = W.contact_point - c.pos;
            V vel_at = c.vel_at(relpos);
            float proj = dot(W.contact_normal, vel_at);
            if (denom > 0.1f) {
                float inv = 1.f / denom;
                W.susp_rel_vel = proj * inv;
                W.clipped_inv = inv;
            } else {
                W.susp_rel_vel = 0.f;
                W.clipped_inv = 10.f;
            }
            if (obj == 10) {  // static: extra pushback (resolveSingleCollision, btContactConstraint.cpp:60-105)
                float thresh = (rest + radius) - 0.05f;
                if (trace < thresh) {
                    float dist = trace - thresh;
                    V rel1 = hp - c.pos;
                    V v1 = c.vel_at(rel1);
                    float rel_vel = dot(hn, v1);
                    float pos_err = 0.2f * -dist / TICK_TIME;
                    float vel_err = -(1.0f + 0.f) * rel_vel;
                    float denom0 = c.impulse_denominator(hp, hn);
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
    }

    // ground body data for friction: velocity / mass / inertia (static -> zero)
    void ground_info(int g, V rel, V& vel, float& inv_mass, V& inv_iner, M& rot, V& com) {
        if (g >= 0 && g <= 4) {
            const Body& o = snap[g];
            vel = o.vel_at(rel);
            inv_mass = o.inv_mass;
            inv_iner = o.inv_inertia_local;
            rot = o.rot;
            com = o.pos;
        } else {
            vel = V();
            inv_mass = 0.f;
            inv_iner = V();
            rot = M::ident();
            com = V();
        }
    }

    // btVehicleRL::calcFrictionImpulses (btVehicleRL.cpp:308-369)
    void calc_friction(int ci) {
        Body& c = b[ci + 1];
        rlgpu_car& cs = car(ci);
        const float friction_scale = CAR_MASS / 3;
        for (int i = 0; i < 4; i++) {
            WheelTick& W = wt[ci][i];
            if (W.ground < 0) {
                W.impulse = V();
                continue;
            }
            V axle = W.wt_col1;
            V n = W.contact_normal;
            float proj = dot(axle, n);
            axle -= n * proj;
            axle = safe_normalized(axle);
            V fwd = safe_normalized(cross(n, axle));
            // resolveSingleBilateral (btContactConstraint.cpp:108-150)
            float side;
            {
                V cp = W.contact_point;
                V rel1 = cp - c.pos;
                V gvel;
                float g_inv_mass;
                V g_iner, g_com;
                M g_rot;
                ground_info(W.ground, V(), gvel, g_inv_mass, g_iner, g_rot, g_com);
                V rel2 = cp - g_com;
                V v1 = c.vel_at(rel1);
                V v2 = (W.ground >= 0 && W.ground <= 4) ? snap[W.ground].vel_at(rel2) : V();
                V vel = v1 - v2;
                V aJ = transpose(c.rot) * cross(rel1, axle);
                V bJ = transpose(g_rot) * cross(rel2, -axle);
                V m0 = c.inv_inertia_local * aJ;
                V m1 = g_iner * bJ;
                float adiag = c.inv_mass + dot(m0, aJ) + g_inv_mass + dot(m1, bJ);
                float jinv = 1.f / adiag;
                float rel_vel = dot(axle, vel);
                side = -0.2f * rel_vel * jinv;
            }
            float rolling;
            if (cs.wheel_engine_force[i] == 0.f) {
                if (cs.wheel_brake[i] != 0.f) {
                    V cp = W.contact_point;
                    V car_rel = cp - c.pos;
                    V v1 = c.vel_at(car_rel);
                    V v2 = (W.ground >= 0 && W.ground <= 4) ? snap[W.ground].vel_at(car_rel) : V();
                    float rel_vel = dot(v1 - v2, fwd);
                    const float MAGIC = 113.73963f;
                    rolling = std::clamp(-rel_vel * MAGIC, -cs.wheel_brake[i], cs.wheel_brake[i]);
                } else {
                    rolling = 0.f;
                }
            } else {
                rolling = -cs.wheel_engine_force[i] / friction_scale;
            }
            V total = (fwd * rolling * cs.wheel_long_friction[i]) + (axle * side * cs.wheel_lat_friction[i]);
            W.impulse = total * friction_scale;
        }
    }

    V upwards_dir_from_wheels(int ci) {
        V sum;
        for (int i = 0; i < 4; i++)
            if (wt[ci][i].in_contact) sum += wt[ci][i].contact_normal;
        if (sum.x == 0 && sum.y == 0 && sum.z == 0) return b[ci + 1].rot.col(2);
        return safe_normalized(sum);
    }

    // Car::_PreTickUpdate demo block (Car.cpp:66-84), hoisted in front of all cars' pre-ticks so
    // the vehicle phase can run car-parallel; RNG draws stay in car order.
    void demo_timers() {
        for (int ci = 0; ci < 4; ci++) {
            rlgpu_car& cs = car(ci);
            if (cs.is_demoed) {
                cs.demo_respawn_timer = std::max(cs.demo_respawn_timer - TICK_TIME, 0.f);
                if (cs.demo_respawn_timer == 0.f) respawn(ci);
            }
        }
    }

    // ---------------------------------------------------------------- Car::_PreTickUpdate
    void car_pre_tick(int ci) {
        Body& c = b[ci + 1];
        rlgpu_car& cs = car(ci);
        float* ctl = cs.controls;
        for (int k = 0; k < 5; k++) ctl[k] = std::clamp(ctl[k], -1.f, 1.f);  // ClampFix
        // c.active (DISABLE_SIMULATION / CF_NO_CONTACT_RESPONSE) was decided at tick start and the
        // demo timer / respawn ran for every car before any pre-tick (see demo_timers()).
        if (cs.is_demoed) return;

        wheel_transforms(ci);
        for (int i = 0; i < 4; i++) wheel_ray(ci, i);
        calc_friction(ci);

        bool jump_pressed = ctl[5] != 0.f && cs.last_controls[5] == 0.f;
        int nwc = 0;
        for (int i = 0; i < 4; i++) {
            cs.wheel_contact[i] = wt[ci][i].in_contact;
            nwc += wt[ci][i].in_contact;
        }
        cs.is_on_ground = nwc >= 3;
        float fwd_speed = dot(c.vel, c.rot.col(0)) * BT_TO_UU;
        update_wheels(ci, nwc, fwd_speed);
        if (nwc < 3)
            update_air_torque(ci, nwc == 0);
        else
            cs.is_flipping = false;
        update_jump(ci, jump_pressed);
        update_auto_flip(ci, jump_pressed);
        update_double_jump_or_flip(ci, jump_pressed, fwd_speed);
        if (ctl[0] != 0.f && ((nwc > 0 && nwc < 4) || cs.world_contact)) update_auto_roll(ci, nwc);
        cs.world_contact = 0;
        // updateVehicleSecond: updateSuspension + applyFrictionImpulses (btVehicleRL.cpp:237-306,372-389)
        for (int i = 0; i < 4; i++) {
            WheelTick& W = wt[ci][i];
            if (W.in_contact) {
                float force = (w.wheel_rest[i] - W.susp_len) * 500.f * W.clipped_inv;
                float damp = (W.susp_rel_vel < 0) ? 25.f : 40.f;
                W.susp_force = force - (damp * W.susp_rel_vel);
                W.susp_force *= w.wheel_force_scale[i];
                if (W.susp_force < 0) W.susp_force = 0;
            } else {
                W.susp_force = 0;
            }
        }
        for (int i = 0; i < 4; i++) {
            WheelTick& W = wt[ci][i];
            if (W.susp_force != 0) {
                V off = W.contact_point - c.pos;
                float base = (W.susp_force * TICK_TIME) + cs.wheel_extra_pushback[i];
                c.apply_impulse(W.contact_normal * base, off);
            }
        }
        {
            V up = c.rot.col(2);
            for (int i = 0; i < 4; i++) {
                WheelTick& W = wt[ci][i];
                if (!is_zero(W.impulse)) {
                    V off = W.contact_point - c.pos;
                    float d = dot(up, off);
                    V rel = off - up * d;
                    c.apply_impulse(W.impulse * TICK_TIME, rel);
                }
            }
        }
        update_boost(ci);
    }

    // Car::_UpdateWheels (Car.cpp:330-475)
    void update_wheels(int ci, int nwc, float fwd_speed) {
        Body& c = b[ci + 1];
        rlgpu_car& cs = car(ci);
        const float* ctl = cs.controls;
        float abs_fwd = std::fabs(fwd_speed);
        bool world_contact = false;
        for (int i = 0; i < 4; i++) world_contact |= wt[ci][i].contact_world;
        if (ctl[7] != 0.f)
            cs.handbrake_val += 5.f * TICK_TIME;
        else
            cs.handbrake_val -= 2.f * TICK_TIME;
        cs.handbrake_val = std::clamp(cs.handbrake_val, 0.f, 1.f);
        float real_throttle = ctl[0];
        float real_brake = 0;
        if (ctl[6] != 0.f && cs.boost > 0) real_throttle = 1;
        {
            float drive_scale = DRIVE_SPEED_TORQUE_FACTOR.out(abs_fwd);
            float engine_throttle = real_throttle;
            if (ctl[7] != 0.f) {
            } else {
                float abs_throttle = std::fabs(real_throttle);
                if (abs_throttle >= 0.001f) {
                    auto sgn = [](float x) { return x > 0 ? 1 : (x < 0 ? -1 : 0); };  // RS_SGN
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
            float engine = engine_throttle * (CAR_MASS * 400.f * UU_TO_BT) * drive_scale;
            float brake = real_brake * (CAR_MASS * (14.25f + (1.f / 3.f)) * UU_TO_BT);
            for (int i = 0; i < 4; i++) {
                cs.wheel_engine_force[i] = engine;
                cs.wheel_brake[i] = brake;
            }
        }
        {
            float steer = STEER_ANGLE_FROM_SPEED.out(abs_fwd);
            if (cs.handbrake_val != 0.f) steer += (POWERSLIDE_STEER_ANGLE.out(abs_fwd) - steer) * cs.handbrake_val;
            steer *= ctl[1];
            cs.wheel_steer[0] = steer;
            cs.wheel_steer[1] = steer;
        }
        for (int i = 0; i < 4; i++) {
            WheelTick& W = wt[ci][i];
            if (W.ground >= 0) {
                V lat_dir = W.wt_col1;
                V long_dir = cross(lat_dir, W.contact_normal);
                float fin = 0;
                V delta = W.hard_point - c.pos;
                V cv = (cross(c.ang, delta) + c.vel) * BT_TO_UU;
                float base = std::fabs(dot(cv, lat_dir));
                if (base > 5) fin = base / (std::fabs(dot(cv, long_dir)) + base);
                float lat = LAT_FRICTION.out(fin);
                float lon = LONG_FRICTION.out(fin);
                if (cs.handbrake_val != 0.f) {
                    float hb = cs.handbrake_val;
                    lat *= (HANDBRAKE_LAT_FRICTION_FACTOR.out(fin) - 1) * hb + 1;
                    lon *= (HANDBRAKE_LONG_FRICTION_FACTOR.out(fin) - 1) * hb + 1;
                } else {
                    lon = 1;
                }
                bool sticky = real_throttle != 0;
                if (!sticky) {
                    float ns = NON_STICKY_FRICTION_FACTOR.out(W.contact_normal.z);
                    lat *= ns;
                    lon *= ns;
                }
                cs.wheel_lat_friction[i] = lat;
                cs.wheel_long_friction[i] = lon;
            }
        }
        if (world_contact) {
            V up = upwards_dir_from_wheels(ci);
            bool full = (real_throttle != 0) || (abs_fwd > 25.f);
            float scale = 0.5f;
            if (full) scale += 1 - std::fabs(up.z);
            c.force += up * scale * (GRAVITY_Z_UU * UU_TO_BT) * CAR_MASS;
        }
    }

    // Car::_UpdateBoost (Car.cpp:477-505)
    void update_boost(int ci) {
        Body& c = b[ci + 1];
        rlgpu_car& cs = car(ci);
        bool boosting = cs.controls[6] != 0.f;
        if (cs.time_spent_boosting > 0) {
            if (!boosting && cs.time_spent_boosting >= 0.1f)
                cs.time_spent_boosting = 0;
            else
                cs.time_spent_boosting += TICK_TIME;
        } else {
            if (boosting) cs.time_spent_boosting = TICK_TIME;
        }
        if (cs.boost > 0 && cs.time_spent_boosting > 0) {
            cs.boost = std::max(cs.boost - (100.f / 3) * TICK_TIME, 0.f);
            float accel = cs.is_on_ground ? (2975 / 3.f) : (3175 / 3.f);
            c.force += accel * UU_TO_BT * c.rot.col(0) * CAR_MASS;
        }
        cs.boost = std::min(cs.boost, 100.f);
    }

    // Car::_UpdateJump (Car.cpp:507-554)
    void update_jump(int ci, bool jump_pressed) {
        Body& c = b[ci + 1];
        rlgpu_car& cs = car(ci);
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
            V f = c.rot.col(2) * (875.f / 3.f) * UU_TO_BT * CAR_MASS;
            c.apply_central_impulse(f);
        }
        if (cs.is_jumping) {
            cs.has_jumped = 1;
            V total = c.rot.col(2) * (4375.f / 3.f);
            if (cs.jump_time < JUMP_MIN) total *= 0.62f;
            c.force += total * UU_TO_BT * CAR_MASS;
        }
        if (cs.is_jumping || cs.has_jumped) cs.jump_time += TICK_TIME;
    }

    // Car::_UpdateAirTorque (Car.cpp:556-641)
    void update_air_torque(int ci, bool update_air_control) {
        Body& c = b[ci + 1];
        rlgpu_car& cs = car(ci);
        const float* ctl = cs.controls;
        V dir_pitch = -c.rot.col(1), dir_yaw = c.rot.col(2), dir_roll = -c.rot.col(0);
        bool do_air = false;
        if (cs.is_flipping) cs.is_flipping = cs.has_flipped && cs.flip_time < 0.65f;
        if (cs.is_flipping) {
            V rel = ld3(cs.flip_rel_torque);
            if (!(rel.x == 0 && rel.y == 0 && rel.z == 0)) {
                float pitch_scale = 1;
                if (rel.y != 0 && ctl[2] != 0) {
                    auto sgn = [](float x) { return x > 0 ? 1 : (x < 0 ? -1 : 0); };
                    if (sgn(rel.y) == sgn(ctl[2])) {
                        pitch_scale = 1 - std::min(std::fabs(ctl[2]), 1.f);
                        do_air = true;
                    }
                }
                rel.y *= pitch_scale;
                V dodge = rel * V(260.f, 224.f, 0);
                c.torque += (inverse(c.inv_inertia_world) * c.rot) * dodge;
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
            V torque;
            if (ctl[2] != 0 || ctl[3] != 0 || ctl[4] != 0) {
                if (cs.is_flipping)
                    pitch_scale = 0;
                else if (cs.has_flipped && cs.flip_time < 0.65f + 0.3f)
                    pitch_scale = 0;
                torque = (ctl[2] * dir_pitch * pitch_scale * 130.f) + (ctl[3] * dir_yaw * 95.f) + (ctl[4] * dir_roll * 400.f);
            }
            V av = c.ang;
            float damp_pitch = dot(dir_pitch, av) * 30.f * (1 - std::fabs(do_air ? (ctl[2] * pitch_scale) : 0));
            float damp_yaw = dot(dir_yaw, av) * 20.f * (1 - std::fabs(do_air ? ctl[3] : 0));
            float damp_roll = dot(dir_roll, av) * 50.f;
            V damping = (dir_yaw * damp_yaw) + (dir_pitch * damp_pitch) + (dir_roll * damp_roll);
            const float TORQUE_SCALE = (float)(2 * M_PI / (1 << 16) * 1000);
            c.torque += inverse(c.inv_inertia_world) * (torque - damping) * TORQUE_SCALE;
        }
        if (ctl[0] != 0) c.force += c.rot.col(0) * ctl[0] * (200 / 3.f) * UU_TO_BT * CAR_MASS;
    }

    // Car::_UpdateDoubleJumpOrFlip (Car.cpp:643-761)
    void update_double_jump_or_flip(int ci, bool jump_pressed, float fwd_speed) {
        Body& c = b[ci + 1];
        rlgpu_car& cs = car(ci);
        const float* ctl = cs.controls;
        if (cs.is_on_ground) {
            cs.has_double_jumped = 0;
            cs.has_flipped = 0;
            cs.air_time = 0;
            cs.air_time_since_jump = 0;
            cs.flip_time = 0;
        } else {
            cs.air_time += TICK_TIME;
            if (cs.has_jumped && !cs.is_jumping)
                cs.air_time_since_jump += TICK_TIME;
            else
                cs.air_time_since_jump = 0;
            if (jump_pressed && cs.air_time_since_jump < 1.25f) {
                float mag = std::fabs(ctl[3]) + std::fabs(ctl[2]) + std::fabs(ctl[4]);
                bool flip_input = mag >= 0.5f;  // CarConfig::dodgeDeadzone
                bool can_use = !cs.has_double_jumped && !cs.has_flipped;
                if (cs.is_auto_flipping) can_use = false;
                if (can_use) {
                    if (flip_input) {
                        cs.flip_time = 0;
                        cs.has_flipped = 1;
                        cs.is_flipping = 1;
                        float ratio = std::fabs(fwd_speed) / 2300.f;
                        V dodge(-ctl[2], ctl[3] + ctl[4], 0);
                        if (std::fabs(ctl[3] + ctl[4]) < 0.1f && std::fabs(ctl[2]) < 0.1f)
                            dodge = V();
                        else
                            dodge = safe_normalized(dodge);
                        st3(cs.flip_rel_torque, V(-dodge.y, dodge.x, 0));
                        if (std::fabs(dodge.x) < 0.1f) dodge.x = 0;
                        if (std::fabs(dodge.y) < 0.1f) dodge.y = 0;
                        if (!fuzzy_zero(dodge)) {
                            bool back;
                            if (std::fabs(fwd_speed) < 100.0f)
                                back = dodge.x < 0.0f;
                            else
                                back = (dodge.x >= 0.0f) != (fwd_speed >= 0.0f);
                            V init = dodge * 500.f;
                            float max_x = back ? 2.5f : 1.f;
                            init.x *= ((max_x - 1) * ratio) + 1.f;
                            init.y *= ((1.9f - 1) * ratio) + 1.f;
                            if (back) init.x *= 16.f / 15.f;
                            V fdir = c.rot.col(0);
                            float ang = rs_atan2f_at(fdir.y, fdir.x, RS_SITE_FLIP);
                            float sa, ca;
                            rs_sincosf_at(ang, &sa, &ca, RS_SITE_FLIP);
                            V xdir(ca, -sa, 0.f), ydir(sa, ca, 0.f);
                            V dv(dot(init, xdir), dot(init, ydir), 0.f);
                            c.apply_central_impulse(dv * UU_TO_BT * CAR_MASS);
                        }
                    } else {
                        V f = c.rot.col(2) * (875.f / 3.f) * UU_TO_BT * CAR_MASS;
                        c.apply_central_impulse(f);
                        cs.has_double_jumped = 1;
                    }
                }
            }
        }
        if (cs.is_flipping) {
            cs.flip_time += TICK_TIME;
            if (cs.flip_time <= 0.65f) {
                if (cs.flip_time >= 0.15f && (c.vel.z < 0 || cs.flip_time < 0.21f)) {
                    // powf(1 - 0.35, tickTime / (1/120)) == 0.65^1 at 120 tps
                    c.vel.z *= (1 - 0.35f);
                }
            }
        } else if (cs.has_flipped) {
            cs.flip_time += TICK_TIME;
        }
    }

    // Car::_UpdateAutoFlip (Car.cpp:763-797)
    void update_auto_flip(int ci, bool jump_pressed) {
        Body& c = b[ci + 1];
        rlgpu_car& cs = car(ci);
        if (jump_pressed && cs.world_contact && cs.world_contact_normal[2] > (float)M_SQRT1_2) {
            // Angle::FromRotMat -> btMatrix3x3::getEulerYPR roll, negated (MathTypes.cpp:62-71)
            const M& m = c.rot;
            float r0 = rs_atan2f_at(m.r[2].y, m.r[2].z, RS_SITE_EULER);
            // btAsin (btScalar.h): clamp to [-1, 1], then asin
            const float ax = -m.r[2].x;
            float pitch_raw = rs_asinf_at(ax < -1.f ? -1.f : (ax > 1.f ? 1.f : ax), RS_SITE_EULER);
            if (std::fabs(pitch_raw) == SIMD_HALF_PI) r0 = r0 > 0 ? r0 - SIMD_PI : r0 + SIMD_PI;
            float roll = -r0;
            float abs_roll = std::fabs(roll);
            if (abs_roll > 2.8f) {
                cs.auto_flip_timer = 0.4f * (abs_roll / (float)M_PI);
                cs.auto_flip_torque_scale = (roll > 0) ? 1 : -1;
                cs.is_auto_flipping = 1;
                c.apply_central_impulse(-c.rot.col(2) * 200.f * UU_TO_BT * CAR_MASS);
            }
        }
        if (cs.is_auto_flipping) {
            if (cs.auto_flip_timer <= 0) {
                cs.is_auto_flipping = 0;
                cs.auto_flip_timer = 0;
            } else {
                c.ang += c.rot.col(0) * 50.f * cs.auto_flip_torque_scale * TICK_TIME;
                cs.auto_flip_timer -= TICK_TIME;
            }
        }
    }

    // Car::_UpdateAutoRoll (Car.cpp:799-831)
    void update_auto_roll(int ci, int nwc) {
        Body& c = b[ci + 1];
        rlgpu_car& cs = car(ci);
        V gup = nwc > 0 ? upwards_dir_from_wheels(ci) : ld3(cs.world_contact_normal);
        V gdown = -gup;
        V fwd = c.rot.col(0), right = c.rot.col(1);
        V cross_right = cross(gup, fwd);
        V cross_fwd = cross(gdown, cross_right);
        float rtf = 1 - std::clamp(dot(right, cross_right), 0.f, 1.f);
        float ftf = 1 - std::clamp(dot(fwd, cross_fwd), 0.f, 1.f);
        V tdr = fwd * (dot(right, gup) >= 0 ? -1.f : 1.f);
        V tdf = right * (dot(fwd, gup) >= 0 ? 1.f : -1.f);
        V tr = tdr * rtf, tf = tdf * ftf;
        c.force += gdown * 100.f * UU_TO_BT * CAR_MASS;
        c.torque += inverse(c.inv_inertia_world) * (tf + tr) * 80.f;
    }

    // Car::Respawn (Car.cpp:43-56)
    void respawn(int ci) {
        rlgpu_car& cs = car(ci);
        int idx = (int)(rng_next(seed, arena_index, s.env) % 4u);
        bool orange = car_team_orange(ci);
        V pos(w.respawn_x[idx], w.respawn_y[idx] * (orange ? -1.f : 1.f), 36.f);
        set_car_state(ci, pos, w.respawn_rot[orange][idx], 100.f / 3.f, false);
    }

    // Car::SetState with a default CarState (Car.h defaults) at pos/rot.
    void set_car_state(int ci, V pos_uu, const M& rot, float boost, bool on_ground) {
        rlgpu_car& cs = car(ci);
        float steer[4], eng[4], brk[4], lat[4], lon[4], push[4];
        float ctl[8];
        std::memcpy(steer, cs.wheel_steer, sizeof steer);
        std::memcpy(eng, cs.wheel_engine_force, sizeof eng);
        std::memcpy(brk, cs.wheel_brake, sizeof brk);
        std::memcpy(lat, cs.wheel_lat_friction, sizeof lat);
        std::memcpy(lon, cs.wheel_long_friction, sizeof lon);
        std::memcpy(push, cs.wheel_extra_pushback, sizeof push);
        std::memcpy(ctl, cs.controls, sizeof ctl);  // controls are not part of CarState
        default_car(cs);
        std::memcpy(cs.wheel_steer, steer, sizeof steer);
        std::memcpy(cs.wheel_engine_force, eng, sizeof eng);
        std::memcpy(cs.wheel_brake, brk, sizeof brk);
        std::memcpy(cs.wheel_lat_friction, lat, sizeof lat);
        std::memcpy(cs.wheel_long_friction, lon, sizeof lon);
        std::memcpy(cs.wheel_extra_pushback, push, sizeof push);
        std::memcpy(cs.controls, ctl, sizeof ctl);
        cs.boost = boost;
        cs.is_on_ground = on_ground;
        Body& c = b[ci + 1];
        c.pos = pos_uu * UU_TO_BT;
        c.rot = rot;
        c.vel = V();
        c.ang = V();
        c.update_inertia();
    }

    // ------------------------------------------------------------------ manifolds
    // Manifolds live for one tick: RocketSim's broadphase removes every overlapping pair before the
    // collision pass and re-adds the overlapping ones (btRSBroadphase.cpp:392-465); removing a pair
    // destroys its algorithm and manifold (btOverlappingPairCache.cpp:36-46,
    // btConvexConvexAlgorithm.cpp:198-205, btConvexConcaveCollisionAlgorithm.cpp:60-64).  Pairs are
    // processed in ascending key order, so a pair's manifold is the last one created.
    //
    // Keys: dynamic-static body*KSTAT + s, s = mesh object 0..KOBJ-1 then KOBJ + plane (meshes
    // are created before the planes, Arena.cpp:1015-1100, and the broadphase cell keeps static
    // proxies in creation order, btRSBroadphase.cpp:160-176); dynamic-dynamic KDYN + a*8 + b,
    // a < b (manifold A = the lower body: the ball for ball-car pairs, which Bullet creates as
    // (sphere, box), btSphereBoxCollisionAlgorithm.cpp:30-37).
    static constexpr int KOBJ = RLGPU_MAX_MESH_OBJECTS, KSTAT = KOBJ + 4, KDYN = 5 * KSTAT;
    rlgpu_manifold mf[RLGPU_MANIFOLDS];
    int nmf = 0;
    rlgpu_manifold* find_manifold(int key) {
        return (nmf > 0 && mf[nmf - 1].key == key) ? &mf[nmf - 1] : nullptr;
    }
    rlgpu_manifold* get_or_new_manifold(int key) {
        rlgpu_manifold* m = find_manifold(key);
        if (m) return m;
        if (nmf >= RLGPU_MANIFOLDS) return nullptr;
        mf[nmf].key = key;
        mf[nmf].count = 0;
        return &mf[nmf++];
    }
    static void key_bodies(int key, int& a, int& bb) {  // bb: body index, or 10+static slot
        if (key >= KDYN) {
            a = (key - KDYN) / 8;
            bb = (key - KDYN) % 8;
        } else {
            a = key / KSTAT;
            bb = 10 + key % KSTAT;
        }
    }
    // body transform of a manifold side
    void side_transform(int id, V& p, M& r) const {
        if (id >= 10) {
            p = V();
            r = M::ident();
        } else {
            p = b[id].pos;
            r = b[id].rot;
        }
    }
    float pair_cbt(int a, int bb) const {
        float ta = a == 0 ? w.ball_cbt : w.car_cbt;
        if (bb >= 10) return ta;
        float tb = bb == 0 ? w.ball_cbt : w.car_cbt;
        return std::min(ta, tb);
    }

    // btPersistentManifold::sortCachedPoints (btPersistentManifold.cpp:110-198), area3 variant
    static int sort_cached(const rlgpu_manifold& m, const rlgpu_contact& pt) {
        int max_idx = -1;
        float max_pen = pt.dist;
        for (int i = 0; i < 4; i++)
            if (m.pts[i].dist < max_pen) {
                max_idx = i;
                max_pen = m.pts[i].dist;
            }
        float res[4] = {0, 0, 0, 0};
        auto la = [&](int i) { return ld3(m.pts[i].localA); };
        V p = ld3(pt.localA);
        if (max_idx != 0) res[0] = len2(cross(p - la(1), la(3) - la(2)));
        if (max_idx != 1) res[1] = len2(cross(p - la(0), la(3) - la(2)));
        if (max_idx != 2) res[2] = len2(cross(p - la(0), la(3) - la(1)));
        if (max_idx != 3) res[3] = len2(cross(p - la(0), la(2) - la(1)));
        // btVector4::closestAxis4 -> absolute().maxAxis4()
        int best = -1;
        float mx = -1e30f;
        for (int i = 0; i < 4; i++) {
            float v = std::fabs(res[i]);
            if (v > mx) {
                best = i;
                mx = v;
            }
        }
        return best;
    }

    // btManifoldResult::addContactPoint + contact-added callback (Arena.cpp:218-281); t >= 0: the
    // mesh triangle of the point (btAdjustInternalEdgeContacts ends the callback, Arena.cpp:275-279)
    void add_contact(int key, V normal_b, V point_b, float depth, int t = -1) {
        int a, bb;
        key_bodies(key, a, bb);
        float cbt = pair_cbt(a, bb);
        if (depth > cbt) return;
        rlgpu_manifold* m = get_or_new_manifold(key);
        if (!m) {
            s.env.manifold_overflow++;
            return;
        }
        V pa = point_b + normal_b * depth;
        V ta_p, tb_p;
        M ta_r, tb_r;
        side_transform(a, ta_p, ta_r);
        side_transform(bb, tb_p, tb_r);
        rlgpu_contact c;
        std::memset(&c, 0, sizeof c);
        st3(c.localA, vmul(pa - ta_p, ta_r));  // invXform
        st3(c.localB, vmul(point_b - tb_p, tb_r));
        st3(c.normalB, normal_b);
        c.dist = depth;
        c.applied = 0.f;
        // combined friction / restitution (btManifoldResult.cpp:59-82, RocketSim variant)
        bool stat = bb >= 10;
        float fa = a == 0 ? 0.35f : 0.3f, ra = a == 0 ? 0.6f : 0.1f;
        float fb = stat ? 0.6f : (bb == 0 ? 0.35f : 0.3f), rb = stat ? 0.3f : (bb == 0 ? 0.6f : 0.1f);
        c.friction = stat ? std::min(fa, fb) : fa * fb;
        c.restitution = stat ? std::max(ra, rb) : ra * rb;
        int idx;
        if (m->count == 4) {
            idx = sort_cached(*m, c);
        } else {
            idx = m->count;
            m->count++;
        }
        if (idx < 0) idx = 0;
        m->pts[idx] = c;
        contact_callback(a, bb, m->pts[idx]);
        if (t >= 0) {
            rlgpu_contact& cp = m->pts[idx];
            V n = ld3(cp.normalB), lb = ld3(cp.localB);
            edge::adjust_edge(&w.tri[(size_t)t * 3], w.tri_info[t], n, lb, pa, cp.dist);
            st3(cp.normalB, n);
            st3(cp.localB, lb);
        }
    }

    // Arena::_BulletContactAddedCallback (Arena.cpp:218-281): bodies ordered car < ball < world
    void contact_callback(int a, int bb, rlgpu_contact& cp) {
        if (a >= 1 && a <= 4) {
            int ci = a - 1;
            if (bb >= 1 && bb <= 4) {
                car_car_hit(ci, bb - 1, cp);
            } else if (bb >= 10) {  // car-world (Arena.cpp:417-427)
                rlgpu_car& cs = car(ci);
                cs.world_contact = 1;
                std::memcpy(cs.world_contact_normal, cp.normalB, sizeof(float) * 3);
                cp.friction = 0.3f;
                cp.restitution = 0.3f;
            }
        } else if (a == 0) {
            if (bb >= 1 && bb <= 4)
                car_ball_hit(bb - 1, cp);  // manifold A = ball: the callback swaps to (car, ball)
            else if (bb >= 10)
                cp.special = 1;  // ball-world (Arena.cpp:265-273)
        }
    }

    // Arena::_BtCallback_OnCarBallCollision (Arena.cpp:283-333)
    void car_ball_hit(int ci, rlgpu_contact& cp) {
        rlgpu_car& cs = car(ci);
        const Body& c = b[ci + 1];
        const Body& ball = b[0];
        cp.friction = 2.0f;
        cp.restitution = 0.0f;
        V ball_pos = ball.pos * BT_TO_UU, car_pos = c.pos * BT_TO_UU;
        V ball_vel = ball.vel * BT_TO_UU, car_vel = c.vel * BT_TO_UU;
        cs.ball_hit_valid = 1;
        st3(cs.ball_hit_rel_pos, ld3(cp.localA) * BT_TO_UU);  // ballIsBodyA (Arena.cpp:297)
        cs.ball_hit_tick = s.env.tick_count;
        st3(cs.ball_hit_ball_pos, ball_pos);
        st3(cs.ball_hit_extra_vel, V());
        int64_t tick = s.env.tick_count;
        int64_t ex = cs.ball_hit_extra_tick;
        // unsigned comparison of the reference (~0ULL == never)
        uint64_t uex = (uint64_t)ex, ut = (uint64_t)tick;
        if ((ut > uex + 1) || (uex > ut)) {
            cs.ball_hit_extra_tick = tick;
        } else {
            return;
        }
        V fwd = c.rot.col(0);
        V rel_pos = ball_pos - car_pos;
        V rel_vel = ball_vel - car_vel;
        float rel_speed = std::min(len(rel_vel), 4600.f);
        if (rel_speed > 0) {
            V hit_dir = safe_normalized(rel_pos * V(1, 1, 0.35f));
            V adj = fwd * dot(hit_dir, fwd) * (1 - 0.65f);
            hit_dir = safe_normalized(hit_dir - adj);
            V added = (hit_dir * rel_speed) * BALL_CAR_EXTRA_IMPULSE_FACTOR.out(rel_speed) * 1.f;
            st3(cs.ball_hit_extra_vel, added);
            V cache = ld3(s.ball_vel_impulse_cache);
            cache += added * UU_TO_BT;
            st3(s.ball_vel_impulse_cache, cache);
        }
    }

    // Arena::_BtCallback_OnCarCarCollision (Arena.cpp:335-415)
    void car_car_hit(int c1, int c2, rlgpu_contact& cp) {
        cp.friction = 0.09f;
        cp.restitution = 0.1f;
        for (int i = 0; i < 2; i++) {
            bool swapped = i == 1;
            int a = swapped ? c2 : c1, o = swapped ? c1 : c2;
            rlgpu_car& sa = car(a);
            rlgpu_car& so = car(o);
            if (sa.is_demoed || so.is_demoed) return;
            if (sa.car_contact_other_id == car_id(o) && sa.car_contact_cooldown > 0) continue;
            V pa = b[a + 1].pos * BT_TO_UU, po = b[o + 1].pos * BT_TO_UU;
            V va = b[a + 1].vel * BT_TO_UU, vo = b[o + 1].vel * BT_TO_UU;
            V delta = po - pa;
            if (dot(va, delta) > 0) {
                V vel_dir = rs_norm(va);  // RocketSim Vec::Normalized
                V dir_to = rs_norm(delta);
                float speed_towards = dot(va, dir_to);
                float other_away = dot(vo, vel_dir);
                if (speed_towards > other_away) {
                    V lp = swapped ? ld3(cp.localB) : ld3(cp.localA);
                    bool bumper = (lp.x * BT_TO_UU) > 64.5f;
                    if (bumper) {
                        bool demo = sa.is_supersonic;
                        if (demo) demo = car_team_orange(a) != car_team_orange(o);  // enableTeamDemos=false
                        if (demo) {
                            so.is_demoed = 1;
                            so.demo_respawn_timer = 3.f;
                        } else {
                            bool ground = so.is_on_ground;
                            float base = (ground ? BUMP_VEL_AMOUNT_GROUND : BUMP_VEL_AMOUNT_AIR).out(speed_towards);
                            V up = so.is_on_ground ? b[o + 1].rot.col(2) : V(0, 0, 1);
                            V imp = vel_dir * base + up * BUMP_UPWARD_VEL_AMOUNT.out(speed_towards) * 1.f;
                            V cache = ld3(so.vel_impulse_cache);
                            cache += imp * UU_TO_BT;
                            st3(so.vel_impulse_cache, cache);
                        }
                        sa.car_contact_other_id = car_id(o);
                        sa.car_contact_cooldown = 0.25f;
                        // EnvSet _BumpCallback (EnvSet.cpp:31-42): only across teams
                        if (car_team_orange(a) != car_team_orange(o)) {
                            s.env.ev_bump[a] = 1;
                            s.env.ev_bumped[o] = 1;
                            if (demo) {
                                s.env.ev_demo[a] = 1;
                                s.env.ev_demoed[o] = 1;
                            }
                        }
                    }
                }
            }
        }
    }

    // btPersistentManifold::refreshContactPoints (btPersistentManifold.cpp:265-330)
    void refresh(int key) {
        rlgpu_manifold* m = find_manifold(key);
        if (!m) return;
        int a, bb;
        key_bodies(key, a, bb);
        float cbt = pair_cbt(a, bb);
        V pa_, pb_;
        M ra, rb;
        side_transform(a, pa_, ra);
        side_transform(bb, pb_, rb);
        V wa[4], wb[4];
        for (int i = m->count - 1; i >= 0; i--) {
            rlgpu_contact& p = m->pts[i];
            wa[i] = ra * ld3(p.localA) + pa_;
            wb[i] = rb * ld3(p.localB) + pb_;
            p.dist = dot(wa[i] - wb[i], ld3(p.normalB));
        }
        for (int i = m->count - 1; i >= 0; i--) {
            rlgpu_contact& p = m->pts[i];
            bool remove;
            if (!(p.dist <= cbt)) {
                remove = true;
            } else {
                V proj = wa[i] - ld3(p.normalB) * p.dist;
                V diff = wb[i] - proj;
                remove = dot(diff, diff) > cbt * cbt;
            }
            if (remove) {  // removeContactPoint: move last into i
                int last = m->count - 1;
                if (i != last) {
                    m->pts[i] = m->pts[last];
                    wa[i] = wa[last];
                    wb[i] = wb[last];
                }
                m->count--;
            }
        }
    }

    // --------------------------------------------------------------- narrowphase
    void collide_sphere_plane(int key, int p) {
        V n = w.plane_n[p];
        V c = b[0].pos;
        V vtx = c + (-n) * w.ball_radius;  // support vertex (btSphereShape margin = radius)
        float dist = dot(n, vtx - w.plane_p[p]);
        V on_plane = vtx - n * dist;
        float cbt = pair_cbt(0, 10);
        if (dist < cbt) add_contact(key, n, on_plane, dist);
    }
    // triangles [t0, t1) of one mesh object, in BVH visit order (btConvexTriangleCallback)
    void collide_sphere_mesh(int key, int o) {
        V c = b[0].pos;
        float r = w.ball_radius;
        float ext = r + 0.08f;
        float cbt = pair_cbt(0, 10);
        // the object's triangles whose box overlaps the sphere's, in BVH visit order
        w.obj_tree[o].walk(c - V(ext, ext, ext), c + V(ext, ext, ext), [&](int k) {
            const int t = w.tri_visit[w.obj_t0[o] + k];
            V pt, nrm;
            float depth;
            if (sphere_triangle(c, r, t, cbt, pt, nrm, depth)) add_contact(key, nrm, pt, depth, t);
        });
    }
    static bool aabb_overlap(V a0, V a1, V b0, V b1) {
        return !(a0.x > b1.x || a1.x < b0.x || a0.y > b1.y || a1.y < b0.y || a0.z > b1.z || a1.z < b0.z);
    }
    // SphereTriangleDetector::collide (SphereTriangleDetector.cpp:139-240)
    bool sphere_triangle(V center, float radius, int t, float cbt, V& point, V& normal_out, float& depth) const {
        const V* v = &w.tri[(size_t)t * 3];
        float rwt = radius + cbt;
        V normal = cross(v[1] - v[0], v[2] - v[0]);
        float l2 = len2(normal);
        bool has = false;
        V cp;
        if (l2 >= SIMD_EPSILON * SIMD_EPSILON) {
            normal = normal / std::sqrt(l2);
            V p1c = center - v[0];
            float dfp = dot(p1c, normal);
            if (dfp < 0.f) {
                dfp *= -1.f;
                normal = normal * -1.f;
            }
            if (dfp < rwt) {
                if (point_in_triangle(v, normal, center)) {
                    has = true;
                    cp = center - normal * dfp;
                } else {
                    V near = closest_point_triangle(center, v[0], v[1], v[2]);
                    float d2 = len2(near - center);
                    if (d2 < rwt * rwt) {
                        has = true;
                        cp = near;
                    }
                }
            }
        }
        if (!has) return false;
        V c2c = center - cp;
        float d2 = len2(c2c);
        if (!(d2 < rwt * rwt)) return false;
        if (d2 > SIMD_EPSILON) {
            float d = std::sqrt(d2);
            normal_out = bt_normalize(c2c);
            point = cp;
            depth = -(radius - d);
        } else {
            normal_out = normal;
            point = cp;
            depth = -radius;
        }
        return true;
    }
    // SphereTriangleDetector::pointInTriangle (edge-plane test)
    static bool point_in_triangle(const V* v, V normal, V p) {
        V e1 = v[1] - v[0], e2 = v[2] - v[1], e3 = v[0] - v[2];
        V n1 = cross(e1, normal), n2 = cross(e2, normal), n3 = cross(e3, normal);
        float r1 = dot(p, n1) - dot(v[0], n1);
        float r2 = dot(p, n2) - dot(v[1], n2);
        float r3 = dot(p, n3) - dot(v[2], n3);
        if (r1 > 0 && r2 > 0 && r3 > 0) return true;
        if (r1 <= 0 && r2 <= 0 && r3 <= 0) return true;
        return false;
    }
    // closestPointTriangle (SphereTriangleDetector.cpp:88-137)
    static V closest_point_triangle(V p, V a, V b_, V c) {
        V ab = b_ - a, ac = c - a, ap = p - a;
        float d1 = dot(ab, ap), d2 = dot(ac, ap);
        if (d1 <= 0.f && d2 <= 0.f) return a;
        V bp = p - b_;
        float d3 = dot(ab, bp), d4 = dot(ac, bp);
        if (d3 >= 0.f && d4 <= d3) return b_;
        V cp = p - c;
        float d5 = dot(ab, cp), d6 = dot(ac, cp);
        if (d6 >= 0.f && d5 <= d6) return c;
        float vc = d1 * d4 - d3 * d2;
        if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) {
            float vv = d1 / (d1 - d3);
            return a + ab * vv;
        }
        float vb = d5 * d2 - d1 * d6;
        if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) {
            float vv = d2 / (d2 - d6);
            return a + ac * vv;
        }
        float va = d3 * d6 - d5 * d4;
        if (va <= 0.f && (d4 - d3) >= 0.f && (d5 - d6) >= 0.f) {
            float vv = (d4 - d3) / ((d4 - d3) + (d5 - d6));
            return b_ + (c - b_) * vv;
        }
        float denom = 1.f / (va + vb + vc);
        float vv = vb * denom, ww = vc * denom;
        return a + ab * vv + ac * ww;
    }
    // box (car hitbox) vs plane: support vertex (btConvexPlaneCollisionAlgorithm.cpp:53-90)
    void collide_box_plane(int key, int bi, int p) {
        V n = w.plane_n[p];
        const M& R = b[bi].rot;
        V c = car_box_center(bi);
        V dl = vmul(-n, R);  // direction in box frame
        V lv(dl.x >= 0 ? w.car_half.x : -w.car_half.x, dl.y >= 0 ? w.car_half.y : -w.car_half.y,
             dl.z >= 0 ? w.car_half.z : -w.car_half.z);
        V vtx = R * lv + c;
        float dist = dot(n, vtx - w.plane_p[p]);
        V on_plane = vtx - n * dist;
        if (dist < pair_cbt(bi, 10)) add_contact(key, n, on_plane, dist);
    }
    // box vs one triangle: btConvexTriangleCallback::processTriangle's normal early out, then GJK with
    // margins and the GJK/EPA penetration solver (gjk_ref.hpp)
    bool box_triangle(int bi, int t, float cbt, V& nrm, V& point_b, float& depth) {
        gjk::Shapes sh;
        sh.impl = w.car_impl;
        sh.margin = w.car_margin;
        const V* v = &w.tri[(size_t)t * 3];
        sh.tri[0] = v[0];
        sh.tri[1] = v[1];
        sh.tri[2] = v[2];
        return gjk::box_triangle(b[bi].rot, car_box_center(bi), sh, cbt, nrm, point_b, depth, gjk_evals);
    }
    void collide_box_mesh(int key, int bi, int o) {
        V mn, mx;
        body_aabb(bi, b[bi].pos, b[bi].rot, mn, mx);
        float cbt = pair_cbt(bi, 10);
        // the object's triangles whose box overlaps the body's, in BVH visit order
        w.obj_tree[o].walk(mn, mx, [&](int k) {
            const int t = w.tri_visit[w.obj_t0[o] + k];
            V n, pb;
            float d;
            if (box_triangle(bi, t, cbt, n, pb, d)) add_contact(key, n, pb, d, t);
        });
    }
    // btSphereBoxCollisionAlgorithm::getSphereDistance (box = the car), manifold A = ball, B = car
    void collide_car_ball(int key, int bi) {
        const M& R = b[bi].rot;
        V c = car_box_center(bi);
        const float margin = w.car_margin;  // boxShape->getMargin() (btSphereBoxCollisionAlgorithm.cpp:82-90)
        V he = w.car_impl;                  // getHalfExtentsWithoutMargin
        V rel = vmul(b[0].pos - c, R);
        V cp(std::max(-he.x, std::min(he.x, rel.x)), std::max(-he.y, std::min(he.y, rel.y)),
             std::max(-he.z, std::min(he.z, rel.z)));
        float r = w.ball_radius;
        float inter = r + margin;
        float cbt = pair_cbt(bi, 0);
        float contact_dist = inter + cbt;
        V normal = rel - cp;
        float d2 = len2(normal);
        if (d2 > contact_dist * contact_dist) return;
        float distance;
        if (d2 <= SIMD_EPSILON) {
            // getSpherePenetration: deepest face
            float fd[6] = {he.x - rel.x, he.x + rel.x, he.y - rel.y, he.y + rel.y, he.z - rel.z, he.z + rel.z};
            int bf = 0;
            for (int k = 1; k < 6; k++)
                if (fd[k] < fd[bf]) bf = k;
            V nn;
            cp = rel;
            int axis = bf / 2;
            float sg = (bf % 2 == 0) ? 1.f : -1.f;
            cp[axis] = sg * he[axis];
            nn[axis] = sg;
            normal = nn;
            distance = -fd[bf];
        } else {
            distance = len(normal);
            normal = normal / distance;
        }
        V point_on_box = R * (cp + normal * margin) + c;
        float pen = distance - inter;
        V nw = R * normal;  // from box towards sphere
        // addContactPoint(normalOnSurfaceB, pOnBox, depth) into the (sphere, box) manifold, unswapped
        // (btSphereBoxCollisionAlgorithm.cpp:30-37,66-75, btManifoldResult.cpp:118-135)
        add_contact(key, nw, point_on_box, pen);
    }
    // car hitbox vs car hitbox: btBoxBoxDetector / dBoxBox2 (boxbox_ref.hpp), A = car a, B = car b; sides
    // 2 x the half extents with margin (btBoxBoxDetector.cpp:758-766); up to 4 points
    void collide_car_car(int key, int ba, int bb) {
        const V side = w.car_half * 2.f;
        boxbox::box_box(car_box_center(ba), b[ba].rot, side, car_box_center(bb), b[bb].rot, side,
                        [&](V n, V p, float d) { add_contact(key, n, p, d); });
    }

    // btRSBroadphase's grid (Arena.cpp:466-471 with ArenaConfig.h:20-29, HEAVY; btRSBroadphase.cpp:43-84) and
    // GetCellIndices (btRSBroadphase.h:90-99): the home cell of a dynamic proxy is the cell of its AABB min
    int home_cell(V mn) const {
        const float uu = 1.f / 50.f;
        const V lo(-4500.f * uu, -6000.f * uu, 0.f * uu), hi(4500.f * uu, 6000.f * uu, 2500.f * uu);
        const float cs = 370.f * uu * 1.f;
        const V range = hi - lo;
        int n[3];
        for (int a = 0; a < 3; a++) n[a] = std::max(1, (int)std::ceil(range[a] / cs));
        const V f = (mn - lo) * (1.f / cs);
        int c[3];
        for (int a = 0; a < 3; a++) c[a] = std::min(std::max((int)f[a], 0), n[a] - 1);
        return (c[0] * n[1] + c[1]) * n[2] + c[2];
    }
    // The cells' dynamic lists (btRSBroadphase.cpp:160-176, 284-320): setAabb (from updateAabbs, bodies in
    // creation order) removes a proxy whose home cell changed from the 27 cells around the old one and appends
    // it to the 27 around the new one, so each list is in the order of the members' last home change --
    // kept as s.env.bp_rank (all zero: creation order) with s.env.bp_cell = home cell + 1 (0: not placed).
    int list_key(int bi) const { return s.env.bp_rank[bi] * 8 + bi; }
    void broadphase_update() {
        for (int bi = 0; bi < 5; bi++) {
            V mn, mx;
            broad_aabb(bi, mn, mx);
            const int cell = home_cell(mn) + 1;
            if (cell == s.env.bp_cell[bi]) continue;
            s.env.bp_cell[bi] = (uint16_t)cell;
            std::vector<std::pair<int, int>> order;  // (list key, body); bi goes to the end
            for (int c = 0; c < 5; c++) order.push_back({c == bi ? 1000 : list_key(c), c});
            std::sort(order.begin(), order.end());
            for (int r = 0; r < 5; r++) s.env.bp_rank[order[r].second] = (uint8_t)r;
        }
    }
    void collision_detection(bool ball_awake) {
        nmf = 0;  // last tick's pairs (and manifolds) were removed by the broadphase
        // the broadphase's pair order (btRSBroadphase.cpp:392-465): per dynamic proxy in creation order
        // (ball, cars 1-4), its static pairs (mesh objects, then the 4 planes; skipped when the body is
        // inactive, needsCollision(inactive, static) == false), then its dynamic pairs with the later
        // bodies, in its home cell's dynamic-list order, while the AABBs overlap
        for (int bi = 0; bi < 5; bi++) {
            bool active = bi == 0 ? ball_awake : b[bi].active;
            if (active) {
                for (int o = 0; o < w.nobj; o++) {
                    int key = bi * KSTAT + o;
                    if (bi == 0)
                        collide_sphere_mesh(key, o);
                    else
                        collide_box_mesh(key, bi, o);
                    refresh(key);
                }
                for (int p = 0; p < 4; p++) {
                    int key = bi * KSTAT + KOBJ + p;
                    if (bi == 0)
                        collide_sphere_plane(key, p);
                    else
                        collide_box_plane(key, bi, p);
                    refresh(key);
                }
            }
            const int a = bi;
            std::vector<std::pair<int, int>> later;  // (list key, body) of the later bodies
            for (int c = a + 1; c < 5; c++) later.push_back({list_key(c), c});
            std::sort(later.begin(), later.end());
            for (const auto& lc : later) {
                const int c2 = lc.second;
                int ka = a == 0 ? c2 : a, kb = a == 0 ? 0 : c2;  // the car first for ball pairs
                int key = KDYN + a * 8 + c2;
                bool dem = (ka >= 1 && !b[ka].active) || (kb >= 1 && !b[kb].active);
                V m0, m1, n0, n1;
                broad_aabb(ka, m0, m1);
                broad_aabb(kb, n0, n1);
                if (dem || !aabb_overlap(m0, m1, n0, n1)) continue;
                bool act_a = ka == 0 ? ball_awake : b[ka].active;
                bool act_b = kb == 0 ? ball_awake : b[kb].active;
                if (!act_a && !act_b) continue;
                if (kb == 0)
                    collide_car_ball(key, ka);
                else
                    collide_car_car(key, ka, kb);
                refresh(key);
            }
        }
    }

    // -------------------------------------------------------------------- solver
    struct SBody {
        V dlin, dang, push, turn, lin, ang, ext_f, ext_t, inv_mass;
        bool real;
        int idx;
    };
    struct Row {
        int a, bb;  // solver body ids
        V n1, n2, rc1, rc2, angA, angB;
        float jinv, rhs, rhs_pen, cfm, lower, upper, applied, applied_push, friction;
        int friction_index;
        bool special;
        rlgpu_contact* orig;
    };

    void solve(bool ball_awake) {
        // solver bodies: 0..4 as bodies (if active), 5 = fixed
        SBody sb[6];
        bool in_solver[5];
        for (int i = 0; i < 5; i++) {
            bool act = i == 0 ? ball_awake : b[i].active;
            in_solver[i] = act;
            SBody& x = sb[i];
            x.dlin = x.dang = x.push = x.turn = V();
            x.real = act;
            x.idx = i;
            if (act) {
                x.inv_mass = V(b[i].inv_mass, b[i].inv_mass, b[i].inv_mass);
                x.lin = b[i].vel;
                x.ang = b[i].ang;
                x.ext_f = b[i].force * b[i].inv_mass * TICK_TIME;
                x.ext_t = vmul(b[i].torque, b[i].inv_inertia_world) * TICK_TIME;
            } else {
                x.inv_mass = V();
                x.lin = x.ang = x.ext_f = x.ext_t = V();
            }
        }
        SBody& fixed = sb[5];
        fixed.dlin = fixed.dang = fixed.push = fixed.turn = fixed.lin = fixed.ang = fixed.ext_f = fixed.ext_t = fixed.inv_mass = V();
        fixed.real = false;
        fixed.idx = -1;

        std::vector<Row> rows, frows;
        struct Special {
            int num = 0;
            float friction = 0, restitution = 0;
            V total_n;
            float total_d = 0;
        } spec[5];

        auto setup_contact = [&](Row& row, int ia, int ib, const rlgpu_contact& cp, V rel1, V rel2, float dist) {
            SBody& A = sb[ia];
            SBody& B = sb[ib];
            const Body* rb0 = A.real ? &b[A.idx] : nullptr;
            const Body* rb1 = B.real ? &b[B.idx] : nullptr;
            V n = ld3(cp.normalB);
            V t0 = cross(rel1, n);
            row.angA = rb0 ? rb0->inv_inertia_world * t0 : V();
            V t1 = cross(rel2, n);
            row.angB = rb1 ? rb1->inv_inertia_world * -t1 : V();
            float d0 = 0, d1 = 0;
            if (rb0) d0 = rb0->inv_mass + dot(n, cross(row.angA, rel1));
            if (rb1) d1 = rb1->inv_mass + dot(n, cross(-row.angB, rel2));
            row.jinv = 1.f / (d0 + d1 + 0.f);
            row.n1 = rb0 ? n : V();
            row.rc1 = rb0 ? t0 : V();
            row.n2 = rb1 ? -n : V();
            row.rc2 = rb1 ? -t1 : V();
            float penetration = dist + 0.f;
            V v1 = rb0 ? rb0->vel_at(rel1) : V();
            V v2 = rb1 ? rb1->vel_at(rel2) : V();
            float rel_vel = dot(n, v1 - v2);
            row.friction = cp.friction;
            float restitution = std::fabs(rel_vel) < 0.2f ? 0.f : cp.restitution * -rel_vel;
            if (restitution <= 0.f) restitution = 0.f;
            row.applied = cp.applied * 0.85f;  // warm start
            if (rb0) {
                A.dlin += row.n1 * A.inv_mass * row.applied;
                A.dang += row.angA * row.applied;
            }
            if (rb1) {
                B.dlin += (-row.n2 * B.inv_mass) * -row.applied;
                B.dang += -row.angB * -row.applied;
            }
            row.applied_push = 0;
            float v1n = dot(row.n1, A.lin + (A.real ? A.ext_f : V())) + dot(row.rc1, A.ang + (A.real ? A.ext_t : V()));
            float v2n = dot(row.n2, B.lin + (B.real ? B.ext_f : V())) + dot(row.rc2, B.ang + (B.real ? B.ext_t : V()));
            float rv = v1n + v2n;
            float pos_err = 0, vel_err = restitution - rv;
            if (penetration > 0) {
                pos_err = 0;
            } else {
                pos_err = -penetration * 0.8f * (1.f / TICK_TIME);
            }
            float pen_imp = pos_err * row.jinv, vel_imp = vel_err * row.jinv;
            row.rhs = vel_imp;  // split impulse always (threshold 1e30, Arena.cpp:486)
            row.rhs_pen = pen_imp;
            row.cfm = 0.f * row.jinv;
            row.lower = 0;
            row.upper = 1e10f;
        };
        auto add_friction = [&](int ia, int ib, const rlgpu_contact& cp, V rel1, V rel2, int contact_index, float friction) {
            SBody& A = sb[ia];
            SBody& B = sb[ib];
            const Body* rb0 = A.real ? &b[A.idx] : nullptr;
            const Body* rb1 = B.real ? &b[B.idx] : nullptr;
            V n = ld3(cp.normalB);
            V va = A.real ? A.lin + A.ext_f + cross(A.ang + A.ext_t, rel1) : V();
            V vb = B.real ? B.lin + B.ext_f + cross(B.ang + B.ext_t, rel2) : V();
            V vel = va - vb;
            float rel_vel = dot(n, vel);
            V dir = vel - n * rel_vel;
            float lat = len2(dir);
            if (lat > SIMD_EPSILON) {
                dir = dir * (1.f / std::sqrt(lat));
            } else {  // btPlaneSpace1
                V p, q;
                if (std::fabs(n.z) > 0.7071067811865475244008443621048490f) {
                    float a = n.y * n.y + n.z * n.z;
                    float k = 1.f / std::sqrt(a);
                    p = V(0, -n.z * k, n.y * k);
                } else {
                    float a = n.x * n.x + n.y * n.y;
                    float k = 1.f / std::sqrt(a);
                    p = V(-n.y * k, n.x * k, 0);
                }
                dir = p;
            }
            Row f;
            f.a = ia;
            f.bb = ib;
            f.friction = friction;
            f.orig = nullptr;
            f.special = false;
            f.applied = 0;
            f.applied_push = 0;
            f.friction_index = contact_index;
            if (rb0) {
                f.n1 = dir;
                V ta = cross(rel1, dir);
                f.rc1 = ta;
                f.angA = rb0->inv_inertia_world * ta;
            } else {
                f.n1 = f.rc1 = f.angA = V();
            }
            if (rb1) {
                f.n2 = -dir;
                V tb = cross(rel2, f.n2);
                f.rc2 = tb;
                f.angB = rb1->inv_inertia_world * tb;
            } else {
                f.n2 = f.rc2 = f.angB = V();
            }
            float d0 = 0, d1 = 0;
            if (rb0) d0 = rb0->inv_mass + dot(dir, cross(f.angA, rel1));
            if (rb1) d1 = rb1->inv_mass + dot(dir, cross(-f.angB, rel2));
            f.jinv = 1.f / (d0 + d1);
            float v1n = dot(f.n1, rb0 ? A.lin + A.ext_f : V()) + dot(f.rc1, rb0 ? A.ang : V());
            float v2n = dot(f.n2, rb1 ? B.lin + B.ext_f : V()) + dot(f.rc2, rb1 ? B.ang : V());
            f.rhs = (0.f - (v1n + v2n)) * f.jinv;
            f.rhs_pen = 0;
            f.cfm = 0;
            f.lower = -friction;
            f.upper = friction;
            frows.push_back(f);
        };

        // manifolds in creation order = ascending key order (the dispatcher's manifold array)
        for (int oi = 0; oi < nmf; oi++) {
            rlgpu_manifold& mf = this->mf[oi];
            if (mf.count == 0) continue;
            int a, bb;
            key_bodies(mf.key, a, bb);
            bool aact = a < 10 && in_solver[a];
            bool bact = bb < 10 && in_solver[bb];
            if (!aact && !bact) continue;  // sleeping island / both static
            int ia = aact ? a : 5, ib = bact ? bb : 5;
            V pa_, pb_;
            M ra, rb;
            side_transform(a, pa_, ra);
            side_transform(bb, pb_, rb);
            for (int j = 0; j < mf.count; j++) {
                if ((int)rows.size() >= RLGPU_MAX_SOLVER_ROWS) {  // build limit shared with the kernel
                    s.env.manifold_overflow++;
                    continue;
                }
                rlgpu_contact& cp = mf.pts[j];
                V wa = ra * ld3(cp.localA) + pa_;  // positions from the last refresh
                V wb = rb * ld3(cp.localB) + pb_;
                V rel1 = wa - pa_;
                V rel2 = wb - (bb >= 10 ? V() : pb_);
                Row row;
                row.a = ia;
                row.bb = ib;
                row.orig = &cp;
                row.special = cp.special != 0;
                setup_contact(row, ia, ib, cp, rel1, rel2, cp.dist);
                int cidx = (int)rows.size();
                row.friction_index = (int)frows.size();
                if (cp.special) {
                    for (int side = 0; side < 2; side++) {
                        int bid = side ? bb : a;
                        if (bid < 10) {
                            Special& sp = spec[bid];
                            sp.num++;
                            sp.friction = cp.friction;
                            sp.restitution = cp.restitution;
                            sp.total_n += ld3(cp.normalB);
                            sp.total_d += len(side ? rel2 : rel1);
                        }
                    }
                }
                rows.push_back(row);
                add_friction(ia, ib, cp, rel1, rel2, cidx, cp.friction);
            }
        }
        // RocketSim special contacts: one averaged row per body vs the fixed body
        for (int i = 0; i < 5; i++) {
            if (spec[i].num <= 0 || !in_solver[i]) continue;
            if ((int)rows.size() >= RLGPU_MAX_SOLVER_ROWS) {
                s.env.manifold_overflow++;
                continue;
            }
            float distance = spec[i].total_d / spec[i].num;
            V normal = spec[i].total_n / (float)spec[i].num;
            rlgpu_contact tmp;
            std::memset(&tmp, 0, sizeof tmp);
            tmp.dist = distance;
            st3(tmp.normalB, normal);
            tmp.friction = spec[i].friction;
            tmp.restitution = spec[i].restitution;
            V rel1 = normal * -distance, rel2 = V();
            Row row;
            row.a = i;
            row.bb = 5;
            row.orig = nullptr;
            row.special = false;
            setup_contact(row, i, 5, tmp, rel1, rel2, distance);
            int cidx = (int)rows.size();
            row.friction_index = (int)frows.size();
            rows.push_back(row);
            add_friction(i, 5, tmp, rel1, rel2, cidx, tmp.friction);
        }

        // The row functions the reference build selects (setupSolverFunctions, btSequentialImpulseConstraintSolver.cpp:
        // 359-382): _scalar_reference (:46-100, 283-313) without SSE; _sse2 (:149-177, 207-233, 315-350) on x86;
        // MSVC on an SSE4.1 + FMA3 CPU replaces the contact and friction rows by _sse4_1_fma3 (:180-205, 235-260).
        // The dots: btSimdDot3 x + (y + z) (:106-110) in _sse2, _mm_dp_ps(.., 0x7f) = (x + y) + (z + 0) in
        // _sse4_1_fma3, btVector3::dot (x + y) + z in the scalar rows.
        const int ar = g_arith;
        auto rdot = [](V a, V b, int how) {
            const float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z;
            if (how == 1) return x + (y + z);
            if (how == 2) return (x + y) + (z + 0.f);
            return (x + y) + z;
        };
        auto resolve_lower = [&](Row& c, bool generic) {
            SBody& A = sb[c.a];
            SBody& B = sb[c.bb];
            const bool fma3 = ar == RLGPU_ARITH_MSVC_X64;
            const int how = fma3 ? 2 : (ar == RLGPU_ARITH_GCC_X64 ? 1 : 0);
            float di = c.rhs - c.applied * c.cfm;
            float dv1 = rdot(c.n1, A.dlin, how) + rdot(c.rc1, A.dang, how);
            float dv2 = rdot(c.n2, B.dlin, how) + rdot(c.rc2, B.dang, how);
            if (fma3) {  // FMNADD(deltaVelDotn, jacDiagABInv, deltaImpulse) = -(a * b) + c, one rounding
                di = std::fma(-dv1, c.jinv, di);
                di = std::fma(-dv2, c.jinv, di);
            } else {
                di -= dv1 * c.jinv;
                di -= dv2 * c.jinv;
            }
            const float applied = c.applied, sum = applied + di;
            if (fma3) {
                // masks sum > lower and upper > sum; _mm_blendv_ps keeps the in-range values
                const bool above = sum > c.lower, below = !generic || c.upper > sum;
                di = above ? (below ? di : c.upper - applied) : c.lower - applied;
                c.applied = above ? (below ? sum : c.upper) : c.lower;
            } else if (ar == RLGPU_ARITH_GCC_X64) {
                // resultLowerLess = sum < lower, resultUpperLess = sum < upper, applied as and / andnot selects
                const bool low = sum < c.lower;
                float d = low ? c.lower - applied : di, ap = low ? c.lower : sum;
                if (generic && !(sum < c.upper)) {
                    d = c.upper - applied;
                    ap = c.upper;
                }
                di = d;
                c.applied = ap;
            } else if (sum < c.lower) {
                di = c.lower - applied;
                c.applied = c.lower;
            } else if (generic && sum > c.upper) {
                di = c.upper - applied;
                c.applied = c.upper;
            } else {
                c.applied = sum;
            }
            if (fma3) {  // FMADD(n * invMass, deltaImpulse, deltaLinearVelocity), FMADD(angularComponent, ...)
                if (A.real) {
                    const V la = c.n1 * A.inv_mass;
                    A.dlin = V(std::fma(la.x, di, A.dlin.x), std::fma(la.y, di, A.dlin.y), std::fma(la.z, di, A.dlin.z));
                    A.dang = V(std::fma(c.angA.x, di, A.dang.x), std::fma(c.angA.y, di, A.dang.y), std::fma(c.angA.z, di, A.dang.z));
                }
                if (B.real) {
                    const V lb = c.n2 * B.inv_mass;
                    B.dlin = V(std::fma(lb.x, di, B.dlin.x), std::fma(lb.y, di, B.dlin.y), std::fma(lb.z, di, B.dlin.z));
                    B.dang = V(std::fma(c.angB.x, di, B.dang.x), std::fma(c.angB.y, di, B.dang.y), std::fma(c.angB.z, di, B.dang.z));
                }
            } else {
                if (A.real) {
                    A.dlin += c.n1 * A.inv_mass * di;
                    A.dang += c.angA * di;
                }
                if (B.real) {
                    B.dlin += c.n2 * B.inv_mass * di;
                    B.dang += c.angB * di;
                }
            }
        };
        auto resolve_split = [&](Row& c) {  // _scalar_reference or _sse2: only the dot order differs
            float di = 0.f;
            if (c.rhs_pen != 0.f) {
                SBody& A = sb[c.a];
                SBody& B = sb[c.bb];
                const int how = ar == RLGPU_ARITH_SCALAR ? 0 : 1;
                di = c.rhs_pen - c.applied_push * c.cfm;
                float dv1 = rdot(c.n1, A.push, how) + rdot(c.rc1, A.turn, how);
                float dv2 = rdot(c.n2, B.push, how) + rdot(c.rc2, B.turn, how);
                di -= dv1 * c.jinv;
                di -= dv2 * c.jinv;
                float sum = c.applied_push + di;
                if (sum < c.lower) {
                    di = c.lower - c.applied_push;
                    c.applied_push = c.lower;
                } else {
                    c.applied_push = sum;
                }
                if (A.real) {
                    A.push += c.n1 * A.inv_mass * di;
                    A.turn += c.angA * di;
                }
                if (B.real) {
                    B.push += c.n2 * B.inv_mass * di;
                    B.turn += c.angB * di;
                }
            }
            return (float)((double)di * (1. / (double)c.jinv));  // deltaImpulse * (1. / m_jacDiagABInv)
        };
        // split-impulse iterations (btSequentialImpulseConstraintSolver.cpp:1762-1795)
        for (int it = 0; it < 10; it++) {
            float lsr = 0.f;
            for (auto& r : rows) {
                float res = resolve_split(r);
                lsr = std::max(lsr, res * res);
            }
            if (lsr <= 0.f || it >= 9) break;
        }
        // main iterations (:1640-1760, non-interleaved path, special rows skipped)
        for (int it = 0; it < 10; it++) {
            for (auto& r : rows) {
                if (r.special) continue;
                resolve_lower(r, false);
            }
            for (auto& f : frows) {
                float total = rows[f.friction_index].applied;
                if (total > 0.f) {
                    f.lower = -(f.friction * total);
                    f.upper = f.friction * total;
                    resolve_lower(f, true);
                }
            }
        }
        // write back contacts and bodies (:1830-1900)
        for (auto& r : rows)
            if (r.orig) r.orig->applied = r.applied;
        for (int i = 0; i < 5; i++) {
            if (!in_solver[i]) continue;
            SBody& x = sb[i];
            Body& bd = b[i];
            x.lin += x.dlin;
            x.ang += x.dang;
            if (!(x.push.x == 0 && x.push.y == 0 && x.push.z == 0 && x.turn.x == 0 && x.turn.y == 0 && x.turn.z == 0)) {
                if (bd.no_rot) {
                    bd.pos = bd.pos + x.push * TICK_TIME;
                } else {
                    V np;
                    M nr;
                    integrate_transform(bd.pos, bd.rot, x.push, x.turn * 0.1f, TICK_TIME, np, nr);
                    bd.pos = np;
                    bd.rot = nr;
                }
            }
            bd.vel = x.lin + x.ext_f;
            bd.ang = x.ang + x.ext_t;
        }
    }

    // ------------------------------------------------------------ Arena::Step (1 tick)
    void tick() {
        const World& W = w;
        // ball zero-vel sleeping (Arena.cpp:722-727)
        bool ball_sleep = len2(b[0].vel) == 0 && len2(b[0].ang) == 0;
        s.ball_sleeping = ball_sleep;
        b[0].active = true;
        for (int ci = 0; ci < 4; ci++) b[ci + 1].active = !car(ci).is_demoed;  // Car.cpp:66-81
        for (int i = 0; i < 5; i++) snap[i] = b[i];
        demo_timers();
        for (int ci = 0; ci < 4; ci++) car_pre_tick(ci);
        for (int i = 0; i < RLGPU_PADS; i++) {  // BoostPad::_PreTickUpdate
            rlgpu_pad& p = s.pads[i];
            if (p.cooldown > 0) p.cooldown = std::max(p.cooldown - TICK_TIME, 0.f);
            p.is_active = p.cooldown == 0;
        }
        int locked[RLGPU_PADS];
        for (int i = 0; i < RLGPU_PADS; i++) locked[i] = -1;
        // stepSimulation: applyGravity
        b[0].force += W.gravity * BALL_MASS;
        for (int ci = 0; ci < 4; ci++) b[ci + 1].force += W.gravity * CAR_MASS;
        // predictUnconstraintMotion: damping + predicted transform
        b[0].vel *= W.ball_damp;
        b[0].ang *= 1.f;  // angular damping 0 -> pow(1, dt) == 1
        for (int i = 0; i < 5; i++) {
            if (i == 0 && b[0].no_rot) {
                b[0].pred_pos = b[0].pos + b[0].vel * TICK_TIME;
                b[0].pred_rot = b[0].rot;
            } else {
                integrate_transform(b[i].pos, b[i].rot, b[i].vel, b[i].ang, TICK_TIME, b[i].pred_pos, b[i].pred_rot);
            }
        }
        broadphase_update();  // updateAabbs -> btRSBroadphase::setAabb
        // ball island activity: awake if moving, or sharing an island (overlapping broadphase pair)
        bool ball_awake = !ball_sleep;
        if (ball_sleep) {
            V m0, m1;
            broad_aabb(0, m0, m1);
            for (int ci = 1; ci <= 4; ci++) {
                if (!b[ci].active) continue;
                V n0, n1;
                broad_aabb(ci, n0, n1);
                if (aabb_overlap(m0, m1, n0, n1)) ball_awake = true;
            }
        }
        collision_detection(ball_awake);
        solve(ball_awake);
        // integrateTransforms (btDiscreteDynamicsWorld.cpp:889-985), active bodies only
        for (int i = 0; i < 5; i++) {
            bool act = i == 0 ? ball_awake : b[i].active;
            if (!act) continue;
            if (b[i].no_rot) {
                b[i].pos = b[i].pos + b[i].vel * TICK_TIME;
            } else {
                V np;
                M nr;
                integrate_transform(b[i].pos, b[i].rot, b[i].vel, b[i].ang, TICK_TIME, np, nr);
                b[i].pos = np;
                b[i].rot = nr;
            }
            b[i].update_inertia();
        }
        for (int i = 0; i < 5; i++) b[i].force = b[i].torque = V();
        // cars: post tick, finish, pad collide (Arena.cpp:785-800)
        for (int ci = 0; ci < 4; ci++) {
            rlgpu_car& cs = car(ci);
            Body& c = b[ci + 1];
            if (!cs.is_demoed) {
                // _PostTickUpdate (Car.cpp:133-163)
                float sp2 = len2(c.vel * BT_TO_UU);
                if (cs.is_supersonic && cs.supersonic_time < 1.f)
                    cs.is_supersonic = sp2 >= 2100.f * 2100.f;
                else
                    cs.is_supersonic = sp2 >= 2200.f * 2200.f;
                if (cs.is_supersonic)
                    cs.supersonic_time += TICK_TIME;
                else
                    cs.supersonic_time = 0;
                if (cs.car_contact_cooldown > 0) cs.car_contact_cooldown = std::max(cs.car_contact_cooldown - TICK_TIME, 0.f);
                std::memcpy(cs.last_controls, cs.controls, sizeof cs.controls);
                // _FinishPhysicsTick (Car.cpp:165-193)
                V cache = ld3(cs.vel_impulse_cache);
                if (!is_zero(cache)) {
                    c.vel += cache;
                    st3(cs.vel_impulse_cache, V());
                }
                const float maxv = 2300.f * UU_TO_BT;
                if (len2(c.vel) > maxv * maxv) c.vel = bt_normalize(c.vel) * maxv;
                if (len2(c.ang) > 5.5f * 5.5f) c.ang = bt_normalize(c.ang) * 5.5f;
            }
            // BoostPadGrid::CheckCollision (BoostPadGrid.cpp:5-25)
            if (cs.is_demoed || cs.boost >= 100) continue;
            V pos_uu = c.pos * BT_TO_UU;
            if (pos_uu.z > 95.f + 250.f) continue;
            int ix = (int)(pos_uu.x / 1024 + 4), iy = (int)(pos_uu.y / 1024 + 5);
            for (int p = 0; p < RLGPU_PADS; p++) {
                int px = W.pad_cell_x[p], py = W.pad_cell_y[p];
                if (px < std::max(ix - 1, 0) || px > std::min(ix + 1, 7) || py < std::max(iy - 1, 0) || py > std::min(iy + 1, 9))
                    continue;
                rlgpu_pad& pd = s.pads[p];
                bool col = false;
                if (pd.prev_locked_car_id == car_id(ci)) {
                    V mn, mx;
                    body_aabb(ci + 1, c.pos, c.rot, mn, mx);
                    col = (W.pad_box_max[p].x > mn.x && W.pad_box_max[p].y > mn.y && W.pad_box_max[p].z > mn.z) &&
                          (W.pad_box_min[p].x < mx.x && W.pad_box_min[p].y < mx.y && W.pad_box_min[p].z < mx.z);
                } else {
                    float rad = (W.pad_big[p] ? 208.f : 144.f) * UU_TO_BT;
                    float dx = c.pos.x - W.pad_pos_bt[p].x, dy = c.pos.y - W.pad_pos_bt[p].y;
                    if (dx * dx + dy * dy < rad * rad) col = std::fabs(c.pos.z - W.pad_pos_bt[p].z) < (95.f * UU_TO_BT);
                }
                if (col) locked[p] = ci;
            }
        }
        // BoostPad::_PostTickUpdate (BoostPad.cpp:88-105)
        for (int p = 0; p < RLGPU_PADS; p++) {
            rlgpu_pad& pd = s.pads[p];
            uint32_t lid = 0;
            if (locked[p] >= 0) {
                lid = car_id(locked[p]);
                if (pd.is_active) {
                    rlgpu_car& cs = car(locked[p]);
                    cs.boost = std::min(cs.boost + (W.pad_big[p] ? 100.f : 12.f), 100.f);
                    pd.is_active = 0;
                    pd.cooldown = W.pad_big[p] ? 10.f : 4.f;
                }
            }
            pd.prev_locked_car_id = lid;
        }
        // Ball::_FinishPhysicsTick (Ball.cpp:112-138)
        {
            Body& ball = b[0];
            V cache = ld3(s.ball_vel_impulse_cache);
            if (!is_zero(cache)) {
                ball.vel += cache;
                st3(s.ball_vel_impulse_cache, V());
            }
            const float maxv = 6000.f * UU_TO_BT;
            if (len2(ball.vel) > maxv * maxv) ball.vel = bt_normalize(ball.vel) * maxv;
            if (len2(ball.ang) > 6.f * 6.f) ball.ang = bt_normalize(ball.ang) * 6.f;
        }
        s.env.tick_count++;
    }

    void step(int ticks) {
        load_bodies();
        for (int t = 0; t < ticks; t++) tick();
        store_bodies();
    }
};

void default_car(rlgpu_car& cs) {
    // CarState defaults (Car.h:17-100)
    std::memset(&cs, 0, sizeof cs);
    stm(cs.body.rot, M::ident());
    cs.is_on_ground = 1;
    cs.boost = 100.f / 3.f;  // BOOST_SPAWN_AMOUNT
    cs.ball_hit_tick = -1;
    cs.ball_hit_extra_tick = -1;
}

// Arena::ResetToRandomKickoff (Arena.cpp:112-216) with Philox draws for std::shuffle; fuzz: then
// FuzzedKickoffState::ResetArena (FuzzedKickoffState.h:17-25): per car GetState (pos, vel x BT_TO_UU),
// pos += RandFloat(-0.1, 0.1) per axis (Math.cpp:54-57, a 24-bit Philox fraction in place of the engine's),
// SetState (x UU_TO_BT, Car.cpp:23-36).
void kickoff(rlgpu_arena_state& s, uint64_t seed, int arena_index, bool fuzz) {
    const World& W = world();
    int order[5] = {0, 1, 2, 3, 4};
    for (int i = 4; i > 0; i--) {  // Fisher-Yates
        int j = (int)(rng_next(seed, arena_index, s.env) % (uint32_t)(i + 1));
        std::swap(order[i], order[j]);
    }
    Sim sim(W, s, seed, arena_index);
    sim.load_bodies();
    for (int i = 0; i < 2; i++) {  // two cars per team: blue = cars 0,2; orange = cars 1,3
        int k = order[i];
        for (int team = 0; team < 2; team++) {
            int ci = 2 * i + team;
            V pos(W.kick_x[k], W.kick_y[k], 17.f);
            if (team == 1) pos = pos * V(-1, -1, 1);
            sim.set_car_state(ci, pos, W.kick_rot[team][k], 100.f / 3.f, true);
        }
    }
    if (fuzz)
        for (int ci = 0; ci < 4; ci++) {
            Body& c = sim.b[ci + 1];
            for (int k = 0; k < 3; k++) {
                const float u = (float)(rng_next(seed, arena_index, s.env) >> 8) * (1.f / 16777216.f);
                const float r = -0.1f + u * (0.1f - -0.1f);
                c.pos[k] = (c.pos[k] * BT_TO_UU + r) * UU_TO_BT;
                c.vel[k] = (c.vel[k] * BT_TO_UU) * UU_TO_BT;
            }
        }
    // ball: BallState() at rest (pos 0,0,BALL_REST_Z)
    sim.b[0].pos = V(0, 0, 93.15f) * UU_TO_BT;
    sim.b[0].rot = M::ident();
    sim.b[0].vel = sim.b[0].ang = V();
    sim.store_bodies();
    for (int i = 0; i < 3; i++) s.ball_vel_impulse_cache[i] = 0;
    for (int p = 0; p < RLGPU_PADS; p++) {
        s.pads[p].is_active = 1;
        s.pads[p].cooldown = 0;
        s.pads[p].prev_locked_car_id = 0;
    }
}

void arena_step(const World& w, rlgpu_arena_state& s, uint64_t seed, int arena_index, int ticks) {
    Sim sim(w, s, seed, arena_index);
    sim.step(ticks);
}

}  // namespace orc

// ---------------------------------------------------------------- checker entry points (tests only)
extern "C" {
// The Octane hitbox as btBoxShape holds it: implicit half extents, margin, half extents with margin.
void oracle_car_box_shape(float* impl3, float* margin, float* half3) {
    const orc::World& w = orc::world();
    for (int i = 0; i < 3; i++) {
        impl3[i] = w.car_impl[i];
        half3[i] = w.car_half[i];
    }
    *margin = w.car_margin;
}
// n box-triangle queries (gjk_ref.hpp box_triangle): per query rot[9] (rows), centre[3], tri[9] (3
// vertices), cbt; the box shape is the Octane's.  out[8 per query] = {hit, normal xyz, point xyz, depth}.
// counts[2] (optional) += GJK queries and penetration-solver calls.
void oracle_box_triangle(int n, const float* rot, const float* centre, const float* tri, const float* cbt, float* out,
                         uint64_t* counts, int arith) {
    orc::ArithScope scope(arith);
    const orc::World& w = orc::world();
    orc::gjk::Shapes sh;
    sh.impl = w.car_impl;
    sh.margin = w.car_margin;
    uint64_t ev[2] = {0, 0};
    for (int i = 0; i < n; i++) {
        orc::M R;
        for (int r = 0; r < 3; r++) R.r[r] = orc::V(rot[9 * i + 3 * r], rot[9 * i + 3 * r + 1], rot[9 * i + 3 * r + 2]);
        orc::V c(centre[3 * i], centre[3 * i + 1], centre[3 * i + 2]);
        for (int k = 0; k < 3; k++) sh.tri[k] = orc::V(tri[9 * i + 3 * k], tri[9 * i + 3 * k + 1], tri[9 * i + 3 * k + 2]);
        orc::V nrm, pt;
        float d = 0;
        bool hit = orc::gjk::box_triangle(R, c, sh, cbt[i], nrm, pt, d, ev);
        float* o = out + 8 * i;
        o[0] = hit ? 1.f : 0.f;
        o[1] = hit ? nrm.x : 0.f;
        o[2] = hit ? nrm.y : 0.f;
        o[3] = hit ? nrm.z : 0.f;
        o[4] = hit ? pt.x : 0.f;
        o[5] = hit ? pt.y : 0.f;
        o[6] = hit ? pt.z : 0.f;
        o[7] = hit ? d : 0.f;
    }
    if (counts) {
        counts[0] += ev[0];
        counts[1] += ev[1];
    }
}
// this thread's box-triangle GJK queries / penetration-solver calls inside arena steps, then EPA runs, EPA
// iterations, most iterations of one run, most faces one run took (reset after reading)
void oracle_gjk2_counts(uint64_t* out3) {
    for (int i = 0; i < 3; i++) {
        out3[i] = orc::gjk::gjk2_stats[i];
        orc::gjk::gjk2_stats[i] = 0;
    }
}
void oracle_gjk_counts(uint64_t* out6) {
    out6[0] = orc::gjk_evals[0];
    out6[1] = orc::gjk_evals[1];
    orc::gjk_evals[0] = orc::gjk_evals[1] = 0;
    for (int i = 0; i < 4; i++) {
        out6[2 + i] = orc::gjk::epa_stats[i];
        orc::gjk::epa_stats[i] = 0;
    }
}
}  // extern "C"

extern "C" {
// n car-vs-car hitbox queries (boxbox_ref.hpp): per query rot_a[9], centre_a[3], rot_b[9], centre_b[3];
// the Octane box for both.  out[n][1 + 4 * 7] = {count, then per point: normal xyz, point xyz, depth}.
void oracle_box_box(int n, const float* rot_a, const float* centre_a, const float* rot_b, const float* centre_b,
                    float* out) {
    const orc::World& w = orc::world();
    const orc::V side = w.car_half * 2.f;
    for (int i = 0; i < n; i++) {
        orc::M Ra, Rb;
        for (int r = 0; r < 3; r++) {
            Ra.r[r] = orc::V(rot_a[9 * i + 3 * r], rot_a[9 * i + 3 * r + 1], rot_a[9 * i + 3 * r + 2]);
            Rb.r[r] = orc::V(rot_b[9 * i + 3 * r], rot_b[9 * i + 3 * r + 1], rot_b[9 * i + 3 * r + 2]);
        }
        orc::V ca(centre_a[3 * i], centre_a[3 * i + 1], centre_a[3 * i + 2]);
        orc::V cb(centre_b[3 * i], centre_b[3 * i + 1], centre_b[3 * i + 2]);
        float* o = out + (size_t)i * 29;
        for (int k = 0; k < 29; k++) o[k] = 0.f;
        int cnt = 0;
        orc::boxbox::box_box(ca, Ra, side, cb, Rb, side, [&](orc::V nn, orc::V p, float d) {
            float* q = o + 1 + 7 * cnt++;
            q[0] = nn.x; q[1] = nn.y; q[2] = nn.z; q[3] = p.x; q[4] = p.y; q[5] = p.z; q[6] = d;
        });
        o[0] = (float)cnt;
    }
}
}  // extern "C"

extern "C" {
// Bullet's BVH visit order of one mesh's triangles (bvh_ref.hpp): out[k] = triangle visited k-th.
void oracle_bvh_order(const float* tris, int ntris, int32_t* out) {
    std::vector<int> o = orc::bvh::leaf_order(tris, ntris);
    for (int k = 0; k < ntris; k++) out[k] = o[k];
}
}  // extern "C"

// ---------------------------------------------------------------- x86 instruction checks (tests only)
// The x86 modes restate three instructions: rsqrtss (executed here, looked up from this host's table on the
// device), DPPS with mask 0x7f ((x + y) + (z + 0)) and the FMA3 fused multiply-add (std::fma).  These run
// the instructions themselves on arrays so the tests can compare them with the restatements.
#include <immintrin.h>
extern "C" {
void oracle_rsqrtss(const float* x, int64_t n, float* out) {
    for (int64_t i = 0; i < n; i++) out[i] = orc::x86_rsqrtss(x[i]);
}
// 1 when the host has SSE4.1 and FMA3 (the MSVC build's _sse4_1_fma3 rows run only there)
int oracle_has_sse41_fma3() { return __builtin_cpu_supports("sse4.1") && __builtin_cpu_supports("fma") ? 1 : 0; }
__attribute__((target("sse4.1"))) void oracle_dpps(const float* a, const float* b, int64_t n, float* out) {
    for (int64_t i = 0; i < n; i++) {
        const __m128 va = _mm_set_ps(0.f, a[3 * i + 2], a[3 * i + 1], a[3 * i]);
        const __m128 vb = _mm_set_ps(0.f, b[3 * i + 2], b[3 * i + 1], b[3 * i]);
        out[i] = _mm_cvtss_f32(_mm_dp_ps(va, vb, 0x7f));
    }
}
__attribute__((target("fma"))) void oracle_fmadd(const float* a, const float* b, const float* c, int64_t n, float* out) {
    for (int64_t i = 0; i < n; i++) out[i] = _mm_cvtss_f32(_mm_fmadd_ss(_mm_set_ss(a[i]), _mm_set_ss(b[i]), _mm_set_ss(c[i])));
}
// the restatements, for comparison: DPPS order and std::fma
void oracle_dpps_restated(const float* a, const float* b, int64_t n, float* out) {
    for (int64_t i = 0; i < n; i++) {
        const float x = a[3 * i] * b[3 * i], y = a[3 * i + 1] * b[3 * i + 1], z = a[3 * i + 2] * b[3 * i + 2];
        out[i] = (x + y) + (z + 0.f);
    }
}
void oracle_fma_restated(const float* a, const float* b, const float* c, int64_t n, float* out) {
    for (int64_t i = 0; i < n; i++) out[i] = std::fma(a[i], b[i], c[i]);
}
// LinearMath operations of one arithmetic mode (rsim_math.hpp) on arrays, for the device comparison
// (rlgpu_linear_math_queries, dmath.hpp): op 0 normalize v[3] -> v[3]; 1 setRotation q[4] -> m[9];
// 2 getRotation m[9] -> q[4]; 3 quaternion product a[4] b[4] -> q[4]; 4 integrateTransform of rot[9] pos[3]
// linvel[3] angvel[3] over 1/120 s -> pos[3] rot[9].  Input stride 24 floats, output stride 12.
void oracle_linear_math(int op, int arith, const float* in, int64_t n, float* out) {
    orc::ArithScope scope(arith);
    using orc::V;
    using orc::M;
    using orc::Q;
    for (int64_t i = 0; i < n; i++) {
        const float* p = in + 24 * i;
        float* o = out + 12 * i;
        M m;
        for (int r = 0; r < 3; r++) m.r[r] = V(p[3 * r], p[3 * r + 1], p[3 * r + 2]);
        if (op == 0) {
            const V v = orc::bt_normalize(V(p[0], p[1], p[2]));
            o[0] = v.x, o[1] = v.y, o[2] = v.z;
        } else if (op == 1) {
            const M r = orc::mat_from_quat(Q{p[0], p[1], p[2], p[3]});
            for (int k = 0; k < 9; k++) o[k] = r.r[k / 3][k % 3];
        } else if (op == 2) {
            const Q q = orc::quat_from_mat(m);
            o[0] = q.x, o[1] = q.y, o[2] = q.z, o[3] = q.w;
        } else if (op == 3) {
            const Q q = orc::qmul(Q{p[0], p[1], p[2], p[3]}, Q{p[4], p[5], p[6], p[7]});
            o[0] = q.x, o[1] = q.y, o[2] = q.z, o[3] = q.w;
        } else if (op == 4) {
            V np;
            M nr;
            orc::integrate_transform(V(p[9], p[10], p[11]), m, V(p[12], p[13], p[14]), V(p[15], p[16], p[17]), 1.f / 120.f,
                                     np, nr);
            o[0] = np.x, o[1] = np.y, o[2] = np.z;
            for (int k = 0; k < 9; k++) o[3 + k] = nr.r[k / 3][k % 3];
        } else if (op == 6) {  // rsqrtss itself
            for (int k = 0; k < 12; k++) o[k] = orc::x86_rsqrtss(p[k]);
        } else {  // a wheel ray's btSubsimplexConvexCast (layout: rlgpu_linear_math_queries op 5)
            float f = 0.f;
            V n(0.f, 0.f, 0.f);
            const bool hit = orc::gjk::ray_convex_cast(V(p[9], p[10], p[11]), V(p[12], p[13], p[14]), p[21],
                                                       V(p[18], p[19], p[20]), m, V(p[15], p[16], p[17]), f, n);
            o[0] = hit ? 1.f : 0.f, o[1] = f, o[2] = n.x, o[3] = n.y, o[4] = n.z;
        }
    }
}
}  // extern "C"
