// rsim_ref.hpp -- ORACLE (test infrastructure only).  See rsim_ref.cpp for the reference map.
#pragma once
#include <cstdint>
#include <vector>

#include "../include/rlgpu_env.h"
#include "bvh_ref.hpp"
#include "edge_ref.hpp"
#include "rsim_math.hpp"

namespace orc {

extern const float UU_TO_BT, BT_TO_UU, TICK_TIME, CAR_MASS, BALL_MASS;

// Static configuration of a SOCCAR arena with 2v2 Octanes (bullet units).
struct World {
    float ball_radius, ball_inv_mass, car_inv_mass, ball_cbt, car_cbt, ball_damp, susp_travel;
    V ball_inv_inertia, car_half, car_offset, car_inv_inertia, gravity;
    V car_impl;        // btBoxShape m_implicitShapeDimensions (half extents without the margin)
    float car_margin;  // btBoxShape margin after setSafeMargin (0.1 x the smallest half extent)
    V wheel_conn[4];
    float wheel_rest[4], wheel_radius[4], wheel_force_scale[4];
    V plane_n[4], plane_p[4];
    // arena collision meshes (Arena::_SetupArenaCollisionShapes): triangles in load order, object
    // by object (3 vertices each, bullet units), their AABBs and owning object
    int ntris = 0, nobj = 1;
    std::vector<V> tri, tri_min, tri_max;
    std::vector<int> tri_obj;
    std::vector<TriInfo> tri_info;  // internal-edge records (btGenerateInternalEdgeInfo, edge_ref.hpp)
    std::vector<int> tri_visit;     // each object's triangles in Bullet's BVH visit order (bvh_ref.hpp)
    std::vector<int> obj_t0;        // first triangle of each object
    std::vector<bvh::Tree> obj_tree;  // each object's BVH nodes (the walk that finds a query's triangles)
    int arith = RLGPU_ARITH_MSVC_X64;  // the build whose arithmetic the edge records are made in (rsim_math.hpp)
    void set_mesh(const float* tris_bt, int n, const int* obj_ntris, int nobjects);
    float kick_x[5], kick_y[5];
    M kick_rot[2][5];
    float respawn_x[4], respawn_y[4];
    M respawn_rot[2][4];
    V pad_pos_uu[RLGPU_PADS], pad_pos_bt[RLGPU_PADS], pad_box_min[RLGPU_PADS], pad_box_max[RLGPU_PADS];
    bool pad_big[RLGPU_PADS];
    int pad_cell_x[RLGPU_PADS], pad_cell_y[RLGPU_PADS];
    explicit World(int arith = RLGPU_ARITH_MSVC_X64);
};
// the built-in world of an arithmetic mode (synthetic mesh; its edge records depend on the mode)
const World& world(int arith = g_arith);

inline V ld3(const float* p) { return V(p[0], p[1], p[2]); }
inline V ld3v(const float* p) { return V(p[0], p[1], p[2]); }
inline void st3(float* p, V v) {
    p[0] = v.x;
    p[1] = v.y;
    p[2] = v.z;
}
inline M ldm(const float* p) {
    M m;
    for (int i = 0; i < 3; i++) m.r[i] = V(p[3 * i], p[3 * i + 1], p[3 * i + 2]);
    return m;
}
inline void stm(float* p, const M& m) {
    for (int i = 0; i < 3; i++) {
        p[3 * i] = m.r[i].x;
        p[3 * i + 1] = m.r[i].y;
        p[3 * i + 2] = m.r[i].z;
    }
}

void philox(uint64_t key, uint32_t c0, uint32_t c1, uint32_t out[4]);
uint32_t rng_next(uint64_t seed, int arena, rlgpu_env_extra& env);
void default_car(rlgpu_car& cs);
void kickoff(rlgpu_arena_state& s, uint64_t seed, int arena_index, bool fuzz = false);
void arena_step(const World& w, rlgpu_arena_state& s, uint64_t seed, int arena_index, int ticks);

}  // namespace orc
