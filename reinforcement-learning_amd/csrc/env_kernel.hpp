// env_kernel.hpp -- device-side arena simulation for MI355X (gfx950).
//
// Layout: each arena is one rlgpu_arena_state record (include/rlgpu_env.h) in HBM.  A
// 64-thread workgroup (one wavefront) owns kArenas = 4 arenas; the 16 lanes of a quarter-wave
// ("team") own one arena.  At launch the record is copied whole into LDS with coalesced
// 16-byte loads, all ticks of the env step run against LDS, and the record is written back
// once -- HBM traffic is ~2 x 2 KB per arena per env step plus the obs/mask/reward rows and the
// (L2-resident) arena mesh.
//
// Inside a tick the team runs the phases of Arena::Step
// (GigaLearnCPP/RLGymCPP/RocketSim/src/Sim/Arena/Arena.cpp:716-812) with lane-level parallelism
// where the reference has independent work:
//   * 16 lanes = 4 cars x 4 wheels for the btVehicleRL wheel transforms / suspension rays /
//     friction impulses (btVehicleRL.cpp:64-369);
//   * 4 lanes = cars for Car::_PreTickUpdate (Car.cpp:58-131) while 12 lanes tick boost pads;
//   * 16 lanes over the 35 canonical body pairs for the narrowphase (body-vs-mesh pairs split
//     over several lanes, triangles found through the uniform-grid index of MeshView), whose
//     contact candidates are then committed to this tick's manifolds in canonical order by one
//     lane (contact callbacks mutate shared state and Bullet processes pairs serially);
//   * one lane per arena for the order-dependent sequential-impulse solver
//     (btSequentialImpulseConstraintSolver.cpp:1540-1900), rows staged in LDS;
//   * 5 lanes = bodies for integration, 34 pads over 16 lanes for pickups.
// The arithmetic is the CPU oracle's (oracle/rsim_ref.cpp) operation for operation: the
// product and the oracle are independent implementations of the same reference algorithm,
// so a strict-FP build makes them agree bit for bit on every tick.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rlgpu_env.h"
#include "dmath.hpp"
#include "gjk.hpp"

namespace rl {

constexpr int kTeam = 16;           // lanes per arena
constexpr int kArenas = 4;                         // arenas per workgroup (one wavefront)
constexpr int kWG = kArenas * kTeam;               // threads per workgroup
static_assert(kWG <= 64, "one wavefront per workgroup");
constexpr int kMaxCand = 64;        // narrowphase candidates per tick per arena
constexpr int kMaxRows = RLGPU_MAX_SOLVER_ROWS;  // solver contact rows per arena (+ as many friction rows)
constexpr int kPairs = 35;          // 25 dynamic-static + 10 dynamic-dynamic work items ("ranks")
constexpr int kMeshChunks = 6;      // lanes per body-vs-mesh pair in the narrowphase
constexpr int kQueue = 64;          // box-triangle queries queued per arena and tick (more run at once)
// Manifold keys, ascending in Bullet's pair order (rsim_ref.cpp pair_key restates the same):
//   dynamic-static  body * kStat + s, s = mesh object 0..kMaxObj-1, then kMaxObj + plane 0..3
//                   (meshes are created before the planes, Arena.cpp:1015-1100, and a cell's static
//                   list keeps creation order, btRSBroadphase.cpp:160-176)
//   dynamic-dynamic kDynKey + a * 8 + b, a < b
constexpr int kMaxObj = RLGPU_MAX_MESH_OBJECTS;
constexpr int kStat = kMaxObj + 4;
constexpr int kDynKey = 5 * kStat;
constexpr float kTick = 1.f / 120.f;
constexpr float kUU2BT = 1.f / 50.f;
constexpr float kBT2UU = 50.f;
constexpr float kCarMass = 180.f;
constexpr float kBallMass = kCarMass / 6.f;

// Static arena / car constants computed once on the host (env.hip: make_env_const).
struct EnvConst {
    float ball_radius, ball_inv_mass, car_inv_mass, ball_cbt, car_cbt, ball_damp, susp_travel;
    v3 ball_inv_inertia, car_half, car_offset, car_inv_inertia, gravity;
    v3 car_impl;       // btBoxShape implicit half extents (without the margin)
    float car_margin;  // btBoxShape margin after setSafeMargin
    v3 bp_min;         // btRSBroadphase grid (Arena.cpp:466-471, ArenaConfig.h:20-29): minPos, 1 / cellSize, cells
    float bp_inv_cell;
    int bp_cells[3];
    v3 wheel_conn[4];
    float wheel_rest[4], wheel_radius[4], wheel_force_scale[4];
    v3 plane_n[4], plane_p[4];
    int plane_axis[4];  // k when plane_n[p] is the unit axis +-e_k, else -1 (ray_cast's side test)
    float kick_x[5], kick_y[5];
    m3 kick_rot[2][5];
    float respawn_x[4], respawn_y[4];
    m3 respawn_rot[2][4];
    v3 pad_pos_uu[RLGPU_PADS], pad_pos_bt[RLGPU_PADS], pad_box_min[RLGPU_PADS], pad_box_max[RLGPU_PADS];
    int pad_big[RLGPU_PADS], pad_cell_x[RLGPU_PADS], pad_cell_y[RLGPU_PADS];
    int pad_map[RLGPU_PADS];           // CommonValues::BOOST_LOCATIONS -> arena pad (GameState.cpp:11-51)
    v3 boost_loc[RLGPU_PADS];          // CommonValues::BOOST_LOCATIONS (uu)
    float action[RLGPU_ACTIONS][8];    // DefaultAction table
    uint8_t mask_ground[RLGPU_ACTIONS], mask_air[RLGPU_ACTIONS], mask_jump[RLGPU_ACTIONS], mask_boost[RLGPU_ACTIONS];
    uint8_t mask_bits[RLGPU_ACTIONS];  // the four tables as bits: ground 1, air 2, jump 4, boost 8 (one load per mask byte)
};

// The env set's reward / terminal registry (rlgpu_envset_config rewards / terminals), one device copy
// per set, read with uniform (scalar) loads by every workgroup.
struct Plugins {
    int nr, nt;
    rlgpu_reward_spec rw[RLGPU_MAX_REWARDS];
    rlgpu_terminal_spec tc[RLGPU_MAX_TERMINALS];
};

struct WheelT {
    v3 hard_point, wheel_dir, contact_point, contact_normal, wt_col1, impulse;
    float susp_len, susp_rel_vel, clipped_inv;
    int ground, in_contact, contact_world;
    v3 rc_nrm;     // the ray's closest static hit before the dynamic bodies' casts: normal,
    float rc_best; // fraction (1: none)
    int rc_obj;    // and object (-1: none)
};
// A wheel ray's convex cast against one dynamic body (ball / car), dealt over the workgroup's lanes
// between the two halves of the wheel phase (wheel_casts)
struct CastJob {
    float f, nx, ny, nz;
    uint8_t wheel, body, hit, pad_;
};
constexpr int kCastJobs = 16 * 4;  // 16 rays x (ball + 3 other cars)

struct Cand {
    float n[3], p[3], depth;
    int order;  // (pair rank << 20) | triangle (= its BVH visit position, mesh.hpp): commit order
    int key;    // manifold key
};

// Arena collision mesh on the device (built by mesh.cpp from the config's triangle list): the
// triangles in load order (3 float4: v0|object, v1, v2 -- bullet units) and a uniform grid over
// their bounding box whose cells list, in CSR form, every triangle whose AABB (grown by kGridPad)
// touches the cell.  Queries are conservative: the exact AABB / edge tests of the reference run
// on every triangle the grid returns, so results equal a scan of all triangles.
constexpr int kMaxTris = 1 << 20;   // triangle index fits the low 20 bits of Cand::order
struct MeshView {
    const float4* cell_tri;  // [entries * 3]: the triangles of every cell inline, ascending index
                             // (v0 | object, v1 | triangle index, v2 | cell x; mesh.hpp MeshGrid)
    const int* cell_start;   // [ncell + 1]
    const float4* tri;       // [ntris * 3]: v0 | object, v1, v2 of triangle t (BVH visit order, mesh.hpp)
    const float4* edge;      // [ntris]: internal-edge record (edge_info.hpp EdgeInfo)
    gjk::GjkScratch* gjk;    // [grid lanes]: box-triangle penetration-solver scratch (gjk.hpp)
    float ox, oy, oz, inv_cell;
    int nx, ny, nz, ntris;
    int empty[6];  // cells x0..x1, y0..y1, z0..z1 that list no triangle (MeshGrid::empty; x0 > x1: none)
};

struct SB {  // btSolverBody subset
    v3 dlin, dang, push, turn, lin, ang, ext_f, ext_t;
    float inv_mass;
    int real;
};
struct CRow {  // contact row (btSolverConstraint subset)
    v3 n1, n2, rc1, rc2, angA, angB;
    float jinv, rhs, rhs_pen, applied, applied_push, friction;
    int a, b, special;
};
struct FRow {  // friction row
    v3 n1, n2, rc1, rc2, angA, angB;
    float jinv, rhs, applied, friction, lower, upper;
    int a, b, cidx;
};
struct Solver {
    SB sb[6];
    CRow rows[kMaxRows];
    FRow frows[kMaxRows];
    int nrows;
    int nmrows;                   // rows from manifold points (the first nmrows)
    int nlev;                     // sweep levels (solve_lanes)
    unsigned in_solver;           // bit i: body i takes part
    int blev[6];                  // level scan: last level that touched each body
    int8_t rmf[kMaxRows], rpt[kMaxRows];  // row -> (manifold, point)
    int8_t lvl[kMaxRows];         // row -> sweep level
    int spec_num[5];
    float spec_fric[5], spec_rest[5], spec_d[5];
    v3 spec_n[5];
};

struct Aux {
    v3 force[5], torque[5];
    m3 iiw[5];
    v3 pred_pos[5];
    m3 pred_rot[5];
    v3 snap_vel[5], snap_ang[5];
    int active[5];
    int ball_awake, ball_sleep, ncand, nmf;
    int epa_lock;  // the arena's LDS penetration-solver set is in use (gjk.hpp box_triangle)
    int npen;      // penetration-solver calls this launch (profiling: prof[28], per-workgroup slot 23)
    int nq;        // this tick's queued box-triangle queries (q: triangle | object << 20 | body << 25)
    uint32_t q[kQueue];
    int locked[RLGPU_PADS];
    int touched[4];
    int goal;
    int traj_term;
    float all_rewards[4];
    int arith;     // the set's arithmetic mode (rlgpu_envset_config.arith, include/rlgpu_arith.h)
    float real_throttle[4];  // T2: each car's Car::_UpdateWheels throttle, for its four wheels' friction lanes
};

union Scratch {
    WheelT wt[16];
    struct {
        WheelT wt_[16];  // = wt
        CastJob job[kCastJobs];
        int njob;
    } wc;
    struct {
        v3 mn[5], mx[5];  // T4: the bodies' broadphase AABBs
        int cell[5];      //     and home cells + 1 (bp_home), one lane per body
    } bp;
    Cand cand[kMaxCand];
    // narrowphase: the candidates, then the small penetration-solver set (gjk::lds_view)
    char narrow[sizeof(Cand) * kMaxCand + gjk::kSmallBytes];
    Solver sv;
    struct {
        float obs[4][RLGPU_OBS];
        uint8_t masks[4][RLGPU_ACTIONS];
    } out;
};

constexpr int kRec = (int)((sizeof(rlgpu_arena_state) + 15) / 16 * 16);  // HBM record stride

struct alignas(16) ArenaLDS {
    rlgpu_arena_state s;
    char pad_[kRec - sizeof(rlgpu_arena_state)];
    Aux a;
    rlgpu_manifold mf[RLGPU_MANIFOLDS];  // this tick's manifolds, in creation (= key) order
    Scratch u;
};

// Optional per-phase cycle accounting (StepArgs::prof != null): thread 0 of every workgroup adds
// the s_memtime delta since the previous mark to prof[phase] (all workgroups) and to
// prof[kProfWG + blockIdx.x * kProfPhases + phase] (this workgroup: the kernel ends with its slowest
// workgroup, so the spread matters as much as the mean).  Used by tools/env_phase_profile.py.
constexpr int kProfPhases = 35, kProfWG = 64;  // per workgroup: phases 0-22 and 30-31, slot 23 = penetration-solver calls
// workgroup barrier (a workgroup is one wave of 4 arenas): LDS writes before it are visible after it
__device__ __forceinline__ void sync() { __syncthreads(); }
struct Prof {
    unsigned long long* p;
    long long t;
    __device__ __forceinline__ void mark(int k) {
        if (p) {
            long long now = clock64();
            if (threadIdx.x == 0) {
                atomicAdd(&p[k], (unsigned long long)(now - t));
                p[kProfWG + (size_t)blockIdx.x * kProfPhases + k] += (unsigned long long)(now - t);
            }
            t = clock64();  // after the bookkeeping: its global read-modify-write is no phase's time
        }
    }
};
__device__ __forceinline__ void pmark(Prof* P, int k) {
    if (P && threadIdx.x == 0) P->mark(k);
}

}  // namespace rl
