// env.hip -- the MI355X arena-set kernel and its C ABI (include/rlgpu_env.h).
//
// One launch = one (half) env step for every arena: LDS-resident arena records, quarter-wave
// teams per arena (env_kernel.hpp), phases of Arena::Step separated by workgroup barriers.
#include <mutex>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"
#include "env_step.hpp"
#include "mesh.hpp"
#include "../../include/rlgpu_gamestate.h"

namespace rl {
// the specialised env kernels (env_k0.hip .. env_k2.hip, one per RLGPU_ARITH_* mode)
void env_k0_upload(const EnvConst& k, const RsqrtLut* lut);
void env_k1_upload(const EnvConst& k, const RsqrtLut* lut);
void env_k2_upload(const EnvConst& k, const RsqrtLut* lut);
void env_k0_launch(const StepArgs& g, int blocks, hipStream_t s);
void env_k1_launch(const StepArgs& g, int blocks, hipStream_t s);
void env_k2_launch(const StepArgs& g, int blocks, hipStream_t s);

// ------------------------------------------------------------------ host: constants
static m3 host_euler_ypr(float yaw, float pitch, float roll) {  // btMatrix3x3::setEulerYPR
    float ci = std::cos(roll), cj = std::cos(pitch), ch = std::cos(yaw);
    float si = std::sin(roll), sj = std::sin(pitch), sh = std::sin(yaw);
    float cc = ci * ch, cs = ci * sh, sc = si * ch, ss = si * sh;
    return m3{v3{cj * ch, sj * sc - cs, sj * cc + ss}, v3{cj * sh, sj * ss + cc, sj * cs - sc}, v3{-sj, cj * si, cj * ci}};
}

static EnvConst make_env_const() {
    EnvConst k;
    std::memset(&k, 0, sizeof k);
    const float UU = 1.f / 50.f;
    k.ball_radius = 91.25f * UU;
    float elem = 0.4f * kBallMass * k.ball_radius * k.ball_radius;  // btSphereShape::calculateLocalInertia
    k.ball_inv_inertia = v3{1.f / elem, 1.f / elem, 1.f / elem};
    k.ball_inv_mass = 1.f / kBallMass;
    v3 hs = v3{120.507f, 86.6994f, 38.6591f} * UU;  // Octane hitbox (CarConfig.cpp:20-70)
    v3 h = v3{hs.x / 2.f, hs.y / 2.f, hs.z / 2.f};
    // btBoxShape (btBoxShape.cpp:18-26): implicit = half - 0.04, then setSafeMargin(half)
    // (btConvexInternalShape.h:63-78) lowers the margin to 0.1 x the smallest half extent (Octane:
    // 0.0386591) and btBoxShape::setMargin (btBoxShape.h:84-92) moves the difference into the implicit
    // half extents
    const float m0 = 0.04f;
    v3 impl = v3{h.x - m0, h.y - m0, h.z - m0};
    const float mn_half = h.x < h.y ? (h.x < h.z ? h.x : h.z) : (h.y < h.z ? h.y : h.z);  // btVector3::minAxis
    const float safe = 0.1f * mn_half;
    k.car_margin = m0;
    if (safe < k.car_margin) {
        const v3 with_m = impl + v3{m0, m0, m0};
        k.car_margin = safe;
        impl = with_m - v3{safe, safe, safe};
    }
    k.car_impl = impl;
    {  // btRSBroadphase(minPos * UU_TO_BT, maxPos * UU_TO_BT, maxAABBLen * UU_TO_BT * 1 (HEAVY)), btRSBroadphase.cpp:43-84
        const v3 mn = v3{-4500.f * UU, -6000.f * UU, 0.f * UU}, mx = v3{4500.f * UU, 6000.f * UU, 2500.f * UU};
        const float cell = 370.f * UU * 1.f;
        const v3 range = mx - mn;
        k.bp_min = mn;
        k.bp_inv_cell = 1.f / cell;
        k.bp_cells[0] = std::max(1, (int)std::ceil(range.x / cell));
        k.bp_cells[1] = std::max(1, (int)std::ceil(range.y / cell));
        k.bp_cells[2] = std::max(1, (int)std::ceil(range.z / cell));
    }
    k.car_half = impl + v3{k.car_margin, k.car_margin, k.car_margin};  // getHalfExtentsWithMargin
    k.car_offset = v3{13.87566f, 0.f, 20.755f} * UU;
    float lx = 2.f * k.car_half.x, ly = 2.f * k.car_half.y, lz = 2.f * k.car_half.z;
    v3 inertia = v3{ly * ly + lz * lz, lx * lx + lz * lz, lx * lx + ly * ly} * (kCarMass / 12.f);
    k.car_inv_inertia = v3{1.f / inertia.x, 1.f / inertia.y, 1.f / inertia.z};
    k.car_inv_mass = 1.f / kCarMass;
    for (int i = 0; i < 4; i++) {  // Car.cpp:231-277
        bool front = i < 2, left = i % 2;
        float radius = front ? 12.50f : 15.00f;
        v3 off = front ? v3{51.25f, 25.90f, 20.755f} : v3{-33.75f, 29.50f, 20.755f};
        if (left) off.y *= -1;
        float rest = (front ? 38.755f : 37.055f) - 12.f;
        k.wheel_conn[i] = off * UU;
        k.wheel_rest[i] = rest * UU;
        k.wheel_radius[i] = radius * UU;
        k.wheel_force_scale[i] = front ? (36.f - (1.f / 4.f)) : (54.f + (1.f / 4.f) + (1.5f / 100.f));
    }
    k.susp_travel = ((12.f * UU) * 100.f) / 100.f;
    k.ball_cbt = (float)((double)k.ball_radius + 0.08) * 0.02f;
    {
        v3 mn = k.car_offset - k.car_half, mx = k.car_offset + k.car_half;
        v3 c = (mn + mx) * 0.5f;
        float r = len(mx - mn) * 0.5f;
        k.car_cbt = (r + len(c)) * 0.02f;
    }
    k.gravity = v3{0, 0, -650.f} * UU;
    k.ball_damp = (float)std::pow((double)(1.f - 0.03f), (double)(1.f / 120.f));
    k.plane_n[0] = v3{0, 0, 1};
    k.plane_p[0] = v3{0, 0, 0};
    k.plane_n[1] = v3{0, 0, -1};
    k.plane_p[1] = v3{0, 0, 2048} * UU;
    k.plane_n[2] = v3{1, 0, 0};
    k.plane_p[2] = v3{-4096, 0, 2048 / 2} * UU;
    k.plane_n[3] = v3{-1, 0, 0};
    k.plane_p[3] = v3{4096, 0, 2048 / 2} * UU;
    for (int p = 0; p < 4; p++) {
        const v3 n = k.plane_n[p];
        k.plane_axis[p] = -1;
        if (std::fabs(n.x) == 1.f && n.y == 0.f && n.z == 0.f) k.plane_axis[p] = 0;
        if (n.x == 0.f && std::fabs(n.y) == 1.f && n.z == 0.f) k.plane_axis[p] = 1;
        if (n.x == 0.f && n.y == 0.f && std::fabs(n.z) == 1.f) k.plane_axis[p] = 2;
    }
    const float sx[5] = {-2048, 2048, -256, 256, 0}, sy[5] = {-2560, -2560, -3840, -3840, -4608};
    const float syaw[5] = {(float)(M_PI_4 * 1), (float)(M_PI_4 * 3), (float)(M_PI_4 * 2), (float)(M_PI_4 * 2), (float)(M_PI_4 * 2)};
    for (int i = 0; i < 5; i++) {  // RLConst.h:297-303, orange mirrored (Arena.cpp:183-186)
        k.kick_x[i] = sx[i];
        k.kick_y[i] = sy[i];
        k.kick_rot[0][i] = host_euler_ypr(syaw[i], -0.f, -0.f);
        k.kick_rot[1][i] = host_euler_ypr(syaw[i] + (float)M_PI, -0.f, -0.f);
    }
    const float rx[4] = {-2304, -2688, 2304, 2688};
    for (int i = 0; i < 4; i++) {  // RLConst.h:326-332
        k.respawn_x[i] = rx[i];
        k.respawn_y[i] = -4608;
        k.respawn_rot[0][i] = host_euler_ypr((float)(M_PI / 2) + 0.f, 0.f, 0.f);
        k.respawn_rot[1][i] = host_euler_ypr((float)(M_PI / 2) + (float)M_PI, 0.f, 0.f);
    }
    const float big[6][3] = {{-3584, 0, 73}, {3584, 0, 73}, {-3072, 4096, 73}, {3072, 4096, 73}, {-3072, -4096, 73}, {3072, -4096, 73}};
    const float small[28][3] = {{0, -4240, 70},     {-1792, -4184, 70}, {1792, -4184, 70}, {-940, -3308, 70},  {940, -3308, 70},
                                {0, -2816, 70},     {-3584, -2484, 70}, {3584, -2484, 70}, {-1788, -2300, 70}, {1788, -2300, 70},
                                {-2048, -1036, 70}, {0, -1024, 70},     {2048, -1036, 70}, {-1024, 0, 70},     {1024, 0, 70},
                                {-2048, 1036, 70},  {0, 1024, 70},      {2048, 1036, 70},  {-1788, 2300, 70},  {1788, 2300, 70},
                                {-3584, 2484, 70},  {3584, 2484, 70},   {0, 2816, 70},     {-940, 3308, 70},   {940, 3308, 70},
                                {-1792, 4184, 70},  {1792, 4184, 70},   {0, 4240, 70}};
    for (int i = 0; i < RLGPU_PADS; i++) {  // RLConst.h:212-264 (big first, Arena.cpp:532-556)
        const float* p = i < 6 ? big[i] : small[i - 6];
        k.pad_pos_uu[i] = v3{p[0], p[1], p[2]};
        k.pad_big[i] = i < 6;
        k.pad_pos_bt[i] = k.pad_pos_uu[i] * UU;
        float box_rad = (k.pad_big[i] ? 160.f : 120.f) * UU;
        k.pad_box_min[i] = k.pad_pos_bt[i] - v3{box_rad, box_rad, 0};
        k.pad_box_max[i] = k.pad_pos_bt[i] + v3{box_rad, box_rad, 64.f * UU};
        k.pad_cell_x[i] = (int)(k.pad_pos_uu[i].x / 1024 + 4);
        k.pad_cell_y[i] = (int)(k.pad_pos_uu[i].y / 1024 + 5);
    }
    const float loc[RLGPU_PADS][3] = {  // CommonValues::BOOST_LOCATIONS (CommonValues.h:47-82)
        {0.f, -4240.0, 70.0},    {-1792.0, -4184.0, 70.0}, {1792.0, -4184.0, 70.0},  {-3072.0, -4096.0, 73.0}, {3072.0, -4096.0, 73.0},
        {-940.0, -3308.0, 70.0}, {940.0, -3308.0, 70.0},   {0.0, -2816.0, 70.0},     {-3584.0, -2484.0, 70.0}, {3584.0, -2484.0, 70.0},
        {-1788.0, -2300.0, 70.0}, {1788.0, -2300.0, 70.0}, {-2048.0, -1036.0, 70.0}, {0.0, -1024.0, 70.0},     {2048.0, -1036.0, 70.0},
        {-3584.0, 0.0, 73.0},    {-1024.0, 0.0, 70.0},     {1024.0, 0.0, 70.0},      {3584.0, 0.0, 73.0},      {-2048.0, 1036.0, 70.0},
        {0.0, 1024.0, 70.0},     {2048.0, 1036.0, 70.0},   {-1788.0, 2300.0, 70.0},  {1788.0, 2300.0, 70.0},   {-3584.0, 2484.0, 70.0},
        {3584.0, 2484.0, 70.0},  {0.0, 2816.0, 70.0},      {-940.0, 3310.0, 70.0},   {940.0, 3308.0, 70.0},    {-3072.0, 4096.0, 73.0},
        {3072.0, 4096.0, 73.0},  {-1792.0, 4184.0, 70.0},  {1792.0, 4184.0, 70.0},   {0.0, 4240.0, 70.0}};
    for (int i = 0; i < RLGPU_PADS; i++) {
        k.boost_loc[i] = v3{loc[i][0], loc[i][1], loc[i][2]};
        k.pad_map[i] = -1;
        for (int j = 0; j < RLGPU_PADS; j++) {
            float dx = k.pad_pos_uu[j].x - loc[i][0], dy = k.pad_pos_uu[j].y - loc[i][1];
            if (dx * dx + dy * dy < 10) {
                k.pad_map[i] = j;
                break;
            }
        }
    }
    {  // DefaultAction (DefaultAction.cpp:3-89)
        const float RB[2] = {0, 1}, RF[3] = {-1, 0, 1};
        int n = 0;
        for (float th : RF)
            for (float st : RF)
                for (float bo : RB)
                    for (float hb : RB) {
                        if (bo == 1 && th != 1) continue;
                        float v[8] = {th, st, 0, st, 0, 0, bo, hb};
                        std::memcpy(k.action[n++], v, sizeof v);
                    }
        int ng = n;
        for (float pi : RF)
            for (float ya : RF)
                for (float ro : RF)
                    for (float ju : RB)
                        for (float bo : RB) {
                            if (ju == 1 && ya != 0) continue;
                            if (pi == ro && ro == ju && ju == 0) continue;
                            float hb = (ju == 1) && (pi != 0 || ya != 0 || ro != 0);
                            float v[8] = {bo, ya, pi, ya, ro, ju, bo, hb};
                            std::memcpy(k.action[n++], v, sizeof v);
                        }
        for (int i = 0; i < n; i++) {
            const float* x = k.action[i];
            k.mask_jump[i] = x[5] != 0;
            k.mask_boost[i] = x[6] != 0;
            k.mask_ground[i] = i < ng;
            k.mask_air[i] = (i > ng && x[5] == 0);
            if (i < ng && x[0] == x[6] && ((x[3] != 0) == (x[7] != 0))) k.mask_air[i] = 1;
            k.mask_bits[i] = (uint8_t)(k.mask_ground[i] | k.mask_air[i] << 1 | k.mask_jump[i] << 2 | k.mask_boost[i] << 3);
        }
    }
    return k;
}

}  // namespace rl

namespace rlgpu {
void boost_pad_index_map(int out[RLGPU_PADS_FOR_MAP]) {
    static_assert(RLGPU_PADS_FOR_MAP == RLGPU_PADS, "pad count");
    const rl::EnvConst k = rl::make_env_const();
    for (int i = 0; i < RLGPU_PADS; i++) out[i] = k.pad_map[i];
}
}  // namespace rlgpu

// ------------------------------------------------------------------ C ABI
struct rlgpu_envset {
    rlgpu_envset_config cfg;
    int num_players;
    char* d_arenas = nullptr;
    float *d_obs = nullptr, *d_rewards = nullptr, *d_last_rewards = nullptr, *d_trunc_obs = nullptr;
    uint8_t *d_masks = nullptr, *d_terminals = nullptr;
    unsigned long long* d_prof = nullptr;
    double* d_metrics = nullptr;   // StepCallback slots [num_arenas][RLGPU_STEP_METRIC_SLOTS] or null
    uint64_t metric_calls = 0;     // ExampleMain's stepCounter
    bool metric_players = false;   // this step's player-metrics flag (rlgpu_envset_step_range)
    bool output_only = false;      // rlgpu_envset_set_output_only: rows given in rlgpu_step_outputs go only there
    void *d_cell_tri = nullptr, *d_cell_start = nullptr, *d_tri = nullptr, *d_edge = nullptr;  // arena mesh (MeshView)
    void* d_gjk = nullptr;  // per-lane box-triangle penetration-solver scratch (MeshView::gjk)
    rl::MeshView mesh{};
    rl::Plugins plug{};                 // host copy of the reward / terminal registry
    rl::Plugins* d_plug = nullptr;      // its device copy (StepArgs::plug)
    int32_t* d_player_start = nullptr;  // EnvState::arenaPlayerStartIdx
    float* d_reward_values = nullptr;   // [players][nr] per-reward values (rlgpu_envset_enable_reward_values) or null
    int pen_slots = rl::kPenSave;       // saved deferred penetration queries per workgroup and tick (tests:
                                        // RLGPU_DEBUG_PEN_SAVE_SLOTS at create, 0..kPenSave, exercises the restart path)
};

namespace {
// src/ExampleMain.cpp:132-187: the 13 weighted rewards and NoTouchCondition(8) + ScoreLimitCondition(3)
void example_main_plugins(rl::Plugins& p) {
    std::memset(&p, 0, sizeof p);
    struct R {
        int type;
        float w, p0, p1;
        int zs;
        float ts, os;
    };
    const R list[RLGPU_REWARDS] = {
        {RLGPU_RW_AIR, 0.25f, 0, 0, 0, 0, 0},
        {RLGPU_RW_WAVEDASH, 0.12f, 0, 0, 0, 0, 0},
        {RLGPU_RW_KICKOFF_PROXIMITY_2V2, 5.f, 0, 0, 0, 0, 0},
        {RLGPU_RW_VELOCITY_PLAYER_TO_BALL, 4.f, 0, 0, 0, 0, 0},
        {RLGPU_RW_STRONG_TOUCH, 60, 20, 120, 0, 0, 0},
        {RLGPU_RW_TOUCH_ACCEL, 6.f, 0, 0, 0, 0, 0},
        {RLGPU_RW_VELOCITY_BALL_TO_GOAL, 8.0f, 0, 0, 1, 1, 1},   // ZeroSumReward(child, 1)
        {RLGPU_RW_PICKUP_BOOST, 0.1f, 0, 0, 0, 0, 0},
        {RLGPU_RW_SAVE_BOOST, 0.010f, 0.5f, 0, 0, 0, 0},
        {RLGPU_RW_BUMP, 20, 0, 0, 1, 0.5f, 1},                   // ZeroSumReward(child, 0.5f)
        {RLGPU_RW_DEMO, 80, 0, 0, 1, 0.5f, 1},
        {RLGPU_RW_GOAL, 150, -1, 0, 1, 1, 1},                    // GoalReward() concedeScale -1
        {RLGPU_RW_LOSING_PENALTY, 1.0f, 0.02f, 0, 0, 0, 0}};
    p.nr = RLGPU_REWARDS;
    for (int i = 0; i < RLGPU_REWARDS; i++) {
        rlgpu_reward_spec& r = p.rw[i];
        r.type = list[i].type;
        r.weight = list[i].w;
        r.params[0] = list[i].p0;
        r.params[1] = list[i].p1;
        r.zero_sum = list[i].zs;
        r.zero_sum_team_spirit = list[i].ts;
        r.zero_sum_opponent_scale = list[i].os;
    }
    p.nt = 2;
    p.tc[0] = rlgpu_terminal_spec{RLGPU_TC_NO_TOUCH, 8.f};
    p.tc[1] = rlgpu_terminal_spec{RLGPU_TC_SCORE_LIMIT, 3.f};
}

// the config's lists, validated (before any device work: a rejected config allocates nothing)
rl::Plugins plugins_from(const rlgpu_envset_config* cfg) {
    rl::Plugins p;
    example_main_plugins(p);
    if (cfg->rewards) {
        RLGPU_REQUIRE(cfg->n_rewards >= 0 && cfg->n_rewards <= RLGPU_MAX_REWARDS,
                      "rlgpu_envset_create: n_rewards must be in [0, " + std::to_string(RLGPU_MAX_REWARDS) + "]");
        p.nr = cfg->n_rewards;
        for (int i = 0; i < p.nr; i++) {
            const rlgpu_reward_spec& r = cfg->rewards[i];
            if (r.type < 0 || r.type >= RLGPU_NUM_REWARD_TYPES)
                throw rlgpu::Error(RLGPU_ERR_UNSUPPORTED,
                                   "rlgpu_envset_create: reward " + std::to_string(i) + " has unknown type " +
                                       std::to_string(r.type) + " (the device registry holds types 0.." +
                                       std::to_string(RLGPU_NUM_REWARD_TYPES - 1) + ", include/rlgpu_env.h RLGPU_RW_*)");
            p.rw[i] = r;
        }
    } else {
        RLGPU_REQUIRE(cfg->n_rewards == 0, "rlgpu_envset_create: n_rewards without a rewards list");
    }
    if (cfg->terminals) {
        RLGPU_REQUIRE(cfg->n_terminals >= 0 && cfg->n_terminals <= RLGPU_MAX_TERMINALS,
                      "rlgpu_envset_create: n_terminals must be in [0, " + std::to_string(RLGPU_MAX_TERMINALS) + "]");
        p.nt = cfg->n_terminals;
        for (int i = 0; i < p.nt; i++) {
            const rlgpu_terminal_spec& t = cfg->terminals[i];
            if (t.type < 0 || t.type >= RLGPU_NUM_TERMINAL_TYPES)
                throw rlgpu::Error(RLGPU_ERR_UNSUPPORTED,
                                   "rlgpu_envset_create: terminal condition " + std::to_string(i) + " has unknown type " +
                                       std::to_string(t.type) + " (the device registry holds types 0.." +
                                       std::to_string(RLGPU_NUM_TERMINAL_TYPES - 1) + ", include/rlgpu_env.h RLGPU_TC_*)");
            p.tc[i] = t;
        }
    } else {
        RLGPU_REQUIRE(cfg->n_terminals == 0, "rlgpu_envset_create: n_terminals without a terminals list");
    }
    return p;
}
}  // namespace

extern "C" int rlgpu_envset_default_plugins(rlgpu_reward_spec* rewards, int32_t* n_rewards, rlgpu_terminal_spec* terminals,
                                            int32_t* n_terminals) {
    return rlgpu::guarded([&] {
        rl::Plugins p;
        example_main_plugins(p);
        if (rewards) std::memcpy(rewards, p.rw, sizeof(rlgpu_reward_spec) * p.nr);
        if (n_rewards) *n_rewards = p.nr;
        if (terminals) std::memcpy(terminals, p.tc, sizeof(rlgpu_terminal_spec) * p.nt);
        if (n_terminals) *n_terminals = p.nt;
    });
}

namespace {
// the kernels' __constant__ symbols live once per device: uploaded the first time a set is created on a
// device, under one lock (sets may be created from several threads, on several devices of one process)
std::mutex g_init_mu;
std::vector<char> g_const_ready, g_rsqrt_ready;  // indexed by HIP device

bool device_flag(std::vector<char>& v, int* dev) {
    RLGPU_CHECK_HIP(hipGetDevice(dev));
    if ((int)v.size() <= *dev) v.resize(*dev + 1, 0);
    return v[*dev] != 0;
}

// the x86 modes' rsqrtss: this host's table (host/x86_arith.cpp) in device memory, its pointer in the
// kernels' kRsqrtLut (once per device; the table is the host CPU's, the same for every set)
void ensure_rsqrt() {
    std::lock_guard<std::mutex> lk(g_init_mu);
    int dev = 0;
    if (device_flag(g_rsqrt_ready, &dev)) return;
    int bits = 0;
    const std::vector<uint32_t>& t = rlgpu::x86_rsqrt_table_or_throw(&bits);
    uint32_t* d = nullptr;
    RLGPU_CHECK_HIP(hipMalloc(&d, t.size() * sizeof(uint32_t)));
    RLGPU_CHECK_HIP(hipMemcpy(d, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    const rl::RsqrtLut L{d, bits};
    RLGPU_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(rl::kRsqrtLut), &L, sizeof L));
    const rl::EnvConst k = rl::make_env_const();
    rl::env_k0_upload(k, &L);
    rl::env_k1_upload(k, &L);
    g_rsqrt_ready[dev] = 1;
}

void ensure_const() {
    std::lock_guard<std::mutex> lk(g_init_mu);
    int dev = 0;
    if (device_flag(g_const_ready, &dev)) return;
    rl::EnvConst k = rl::make_env_const();
    RLGPU_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(rl::C), &k, sizeof k));
    rl::env_k0_upload(k, nullptr);
    rl::env_k1_upload(k, nullptr);
    rl::env_k2_upload(k, nullptr);
    g_const_ready[dev] = 1;
}

// rlgpu_envset_set_output_only: the rows a step appends to its outputs are not also written to the set's own
// buffers (the kernel skips a copy whose pointer is null)
void output_only_rows(const rlgpu_envset* e, rl::StepArgs& g) {
    if (!e->output_only) return;
    if (g.out_obs) g.obs = nullptr;
    if (g.out_masks) g.masks = nullptr;
    if (g.out_trunc) g.trunc_obs = nullptr;
}

void launch(rlgpu_envset* e, rl::StepArgs g, hipStream_t s) {
    g.arenas = e->d_arenas;
    g.n = e->cfg.num_arenas;
    g.obs = e->d_obs;
    g.masks = e->d_masks;
    g.rewards = e->d_rewards;
    g.terminals = e->d_terminals;
    g.last_rewards = e->cfg.save_rewards ? e->d_last_rewards : nullptr;
    g.trunc_obs = e->d_trunc_obs;
    g.seed = e->cfg.seed;
    g.max_episode_steps = e->cfg.max_episode_steps;
    g.prof = e->d_prof;
    g.mesh = e->mesh;
    g.plug = e->d_plug;
    g.arith = e->cfg.arith;
    g.arena_offset = e->cfg.arena_offset;
    g.fuzz = e->cfg.state_setter == RLGPU_SS_FUZZED_KICKOFF;
    g.pen_slots = e->pen_slots;
    g.reward_values = g.build ? e->d_reward_values : nullptr;
    output_only_rows(e, g);
    if (g.build && e->d_metrics) {  // one StepCallback call (Learner.cpp:796-797, ExampleMain.cpp:236-237)
        g.metrics = e->d_metrics;
        g.metrics_players = (++e->metric_calls % 4) == 0;
    }
    unsigned blocks = rlgpu::ceil_div(g.n, rl::kArenas);
    switch (e->cfg.arith) {  // the kernel specialised for the set's arithmetic
        case RLGPU_ARITH_MSVC_X64: rl::env_k0_launch(g, blocks, s); break;
        case RLGPU_ARITH_GCC_X64: rl::env_k1_launch(g, blocks, s); break;
        default: rl::env_k2_launch(g, blocks, s); break;
    }
    RLGPU_CHECK_HIP(hipGetLastError());
}

// the arenas [first, first + count) of the set (first % kArenas == 0): every per-arena / per-player pointer
// moved to the range, the arenas' Philox streams and the penetration-solver scratch of their workgroups kept
void launch_range(rlgpu_envset* e, rl::StepArgs g, int first, int count, bool metrics_players, hipStream_t s) {
    const size_t P0 = (size_t)first * 4;
    g.arenas = e->d_arenas + (size_t)first * rl::kRec;
    g.n = count;
    g.obs = e->d_obs + P0 * RLGPU_OBS;
    g.masks = e->d_masks + P0 * RLGPU_ACTIONS;
    g.rewards = e->d_rewards + P0;
    g.terminals = e->d_terminals + first;
    g.last_rewards = e->cfg.save_rewards ? e->d_last_rewards + (size_t)first * e->plug.nr : nullptr;
    g.trunc_obs = e->d_trunc_obs + P0 * RLGPU_OBS;
    g.seed = e->cfg.seed;
    g.max_episode_steps = e->cfg.max_episode_steps;
    g.prof = nullptr;
    g.mesh = e->mesh;
    g.mesh.gjk = e->mesh.gjk ? e->mesh.gjk + (size_t)(first / rl::kArenas) * rl::kWG : nullptr;
    g.plug = e->d_plug;
    g.arith = e->cfg.arith;
    g.arena_offset = e->cfg.arena_offset + first;
    g.fuzz = e->cfg.state_setter == RLGPU_SS_FUZZED_KICKOFF;
    g.pen_slots = e->pen_slots;
    g.reward_values = g.build && e->d_reward_values ? e->d_reward_values + P0 * e->plug.nr : nullptr;
    output_only_rows(e, g);
    if (g.build && e->d_metrics) {
        g.metrics = e->d_metrics + (size_t)first * RLGPU_STEP_METRIC_SLOTS;
        g.metrics_players = metrics_players;
    }
    const unsigned blocks = rlgpu::ceil_div(count, rl::kArenas);
    switch (e->cfg.arith) {
        case RLGPU_ARITH_MSVC_X64: rl::env_k0_launch(g, blocks, s); break;
        case RLGPU_ARITH_GCC_X64: rl::env_k1_launch(g, blocks, s); break;
        default: rl::env_k2_launch(g, blocks, s); break;
    }
    RLGPU_CHECK_HIP(hipGetLastError());
}

rl::StepArgs blank() {
    rl::StepArgs g;
    std::memset(&g, 0, sizeof g);
    return g;
}
}  // namespace

extern "C" int rlgpu_arena_state_size(void) { return (int)sizeof(rlgpu_arena_state); }

extern "C" int rlgpu_envset_create(const rlgpu_envset_config* cfg, rlgpu_envset** out) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(cfg && out, "rlgpu_envset_create: null argument");
        RLGPU_REQUIRE(cfg->num_arenas > 0, "rlgpu_envset_create: num_arenas must be > 0");
        RLGPU_REQUIRE(cfg->tick_skip > 0, "tickSkip must be > 0 (EnvSet.cpp:48)");
        RLGPU_REQUIRE(cfg->action_delay >= 0 && cfg->action_delay <= cfg->tick_skip,
                      "actionDelay must be in [0, tickSkip] (EnvSet.cpp:49)");
        RLGPU_REQUIRE(cfg->mesh_tris == nullptr || cfg->mesh_ntris > 0, "mesh_ntris must be > 0 with mesh_tris");
        RLGPU_REQUIRE(cfg->arith >= 0 && cfg->arith < RLGPU_NUM_ARITH,
                      "rlgpu_envset_create: unknown arithmetic mode " + std::to_string(cfg->arith) + " (RLGPU_ARITH_*)");
        RLGPU_REQUIRE(cfg->state_setter == RLGPU_SS_KICKOFF || cfg->state_setter == RLGPU_SS_FUZZED_KICKOFF,
                      "rlgpu_envset_create: unknown state setter " + std::to_string(cfg->state_setter) + " (RLGPU_SS_*)");
        const rl::Plugins plug = plugins_from(cfg);
        ensure_const();
        if (rl::sse_api(cfg->arith)) ensure_rsqrt();
        // arena meshes (Arena::_SetupArenaCollisionShapes): triangle table + grid index in HBM
        std::vector<float> builtin;
        const float* tris = cfg->mesh_tris;
        int ntris = cfg->mesh_ntris;
        if (!tris) {
            builtin = rlgpu::builtin_mesh_bt();
            tris = builtin.data();
            ntris = (int)(builtin.size() / 9);
        }
        rlgpu::MeshGrid grid = rlgpu::build_mesh_grid(tris, ntris, cfg->mesh_tris ? cfg->mesh_object_ntris : nullptr,
                                                      cfg->mesh_tris ? cfg->mesh_objects : 1, cfg->arith);
        auto* e = new rlgpu_envset();
        if (const char* v = getenv("RLGPU_DEBUG_PEN_SAVE_SLOTS")) e->pen_slots = std::max(0, std::min(atoi(v), rl::kPenSave));
        e->cfg = *cfg;
        e->cfg.mesh_tris = nullptr;  // host pointers are not kept
        e->cfg.mesh_object_ntris = nullptr;
        e->cfg.rewards = nullptr;
        e->cfg.terminals = nullptr;
        e->plug = plug;
        RLGPU_CHECK_HIP(hipMalloc(&e->d_plug, sizeof(rl::Plugins)));
        RLGPU_CHECK_HIP(hipMemcpy(e->d_plug, &e->plug, sizeof(rl::Plugins), hipMemcpyHostToDevice));
        RLGPU_CHECK_HIP(hipMalloc(&e->d_cell_start, grid.cell_start.size() * sizeof(int)));
        RLGPU_CHECK_HIP(hipMalloc(&e->d_cell_tri, std::max<size_t>(grid.cell_tri.size(), 12) * sizeof(float)));
        RLGPU_CHECK_HIP(hipMemcpy(e->d_cell_start, grid.cell_start.data(), grid.cell_start.size() * sizeof(int),
                                  hipMemcpyHostToDevice));
        if (!grid.cell_tri.empty())
            RLGPU_CHECK_HIP(hipMemcpy(e->d_cell_tri, grid.cell_tri.data(), grid.cell_tri.size() * sizeof(float),
                                      hipMemcpyHostToDevice));
        e->mesh.cell_tri = (const float4*)e->d_cell_tri;
        e->mesh.cell_start = (const int*)e->d_cell_start;
        RLGPU_CHECK_HIP(hipMalloc(&e->d_tri, grid.tri.size() * sizeof(float)));
        RLGPU_CHECK_HIP(hipMalloc(&e->d_edge, grid.edge.size() * sizeof(float)));
        RLGPU_CHECK_HIP(hipMemcpy(e->d_tri, grid.tri.data(), grid.tri.size() * sizeof(float), hipMemcpyHostToDevice));
        RLGPU_CHECK_HIP(hipMemcpy(e->d_edge, grid.edge.data(), grid.edge.size() * sizeof(float), hipMemcpyHostToDevice));
        e->mesh.tri = (const float4*)e->d_tri;
        e->mesh.edge = (const float4*)e->d_edge;
        e->mesh.ox = grid.ox;
        e->mesh.oy = grid.oy;
        e->mesh.oz = grid.oz;
        e->mesh.inv_cell = grid.inv_cell;
        e->mesh.nx = grid.nx;
        e->mesh.ny = grid.ny;
        e->mesh.nz = grid.nz;
        e->mesh.ntris = grid.ntris;
        for (int k = 0; k < 6; k++) e->mesh.empty[k] = grid.empty[k];
        int n = cfg->num_arenas;
        {  // one GjkScratch per lane of the env kernel's grid (touched only by penetration-solver calls)
            const size_t lanes = (size_t)rlgpu::ceil_div(n, rl::kArenas) * rl::kWG;
            RLGPU_CHECK_HIP(hipMalloc(&e->d_gjk, lanes * sizeof(rl::gjk::GjkScratch)));
            e->mesh.gjk = (rl::gjk::GjkScratch*)e->d_gjk;
        }
        e->num_players = 4 * n;
        size_t P = (size_t)e->num_players;
        RLGPU_CHECK_HIP(hipMalloc(&e->d_arenas, (size_t)n * rl::kRec));
        RLGPU_CHECK_HIP(hipMalloc(&e->d_obs, P * RLGPU_OBS * sizeof(float)));
        RLGPU_CHECK_HIP(hipMalloc(&e->d_trunc_obs, P * RLGPU_OBS * sizeof(float)));
        RLGPU_CHECK_HIP(hipMalloc(&e->d_rewards, P * sizeof(float)));
        RLGPU_CHECK_HIP(hipMalloc(&e->d_last_rewards, (size_t)n * std::max(plug.nr, 1) * sizeof(float)));
        RLGPU_CHECK_HIP(hipMalloc(&e->d_masks, P * RLGPU_ACTIONS));
        RLGPU_CHECK_HIP(hipMalloc(&e->d_terminals, (size_t)n));
        RLGPU_CHECK_HIP(hipMemset(e->d_terminals, 0, (size_t)n));
        RLGPU_CHECK_HIP(hipMemset(e->d_rewards, 0, P * sizeof(float)));
        RLGPU_CHECK_HIP(hipMemset(e->d_trunc_obs, 0, P * RLGPU_OBS * sizeof(float)));
        RLGPU_CHECK_HIP(hipMemset(e->d_last_rewards, 0, (size_t)n * std::max(plug.nr, 1) * sizeof(float)));
        {  // EnvState::arenaPlayerStartIdx (EnvSet.h:35-65): 4 players per arena
            std::vector<int32_t> start(n);
            for (int i = 0; i < n; i++) start[i] = 4 * i;
            RLGPU_CHECK_HIP(hipMalloc(&e->d_player_start, (size_t)n * sizeof(int32_t)));
            RLGPU_CHECK_HIP(hipMemcpy(e->d_player_start, start.data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice));
        }
        // initial records: Arena ctor + AddCar defaults (Arena.cpp:429-562, Car.cpp:195-277)
        std::vector<char> host((size_t)n * rl::kRec, 0);
        rl::EnvConst k = rl::make_env_const();
        for (int i = 0; i < n; i++) {
            auto* s = (rlgpu_arena_state*)&host[(size_t)i * rl::kRec];
            s->ball.rot[0] = s->ball.rot[4] = s->ball.rot[8] = 1.f;
            s->ball.pos[2] = k.ball_radius;
            for (int c = 0; c < 4; c++) {
                rlgpu_car& cs = s->cars[c];
                cs.body.rot[0] = cs.body.rot[4] = cs.body.rot[8] = 1.f;
                cs.is_on_ground = 1;
                cs.boost = 100.f / 3.f;
                cs.ball_hit_tick = -1;
                cs.ball_hit_extra_tick = -1;
            }
            for (int p = 0; p < RLGPU_PADS; p++) s->pads[p].is_active = 1;
        }
        RLGPU_CHECK_HIP(hipMemcpy(e->d_arenas, host.data(), host.size(), hipMemcpyHostToDevice));
        *out = e;
        // EnvSet ctor: reset every arena (EnvSet.cpp:105-110)
        rl::StepArgs g = blank();
        g.reset_mode = 4;
        launch(e, g, nullptr);
        RLGPU_CHECK_HIP(hipDeviceSynchronize());
    });
}

extern "C" int rlgpu_envset_set_profile(rlgpu_envset* e, unsigned long long* d_counters, int64_t capacity) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e, "null envset");
        // 64 totals + 24 per workgroup of the step launch + one per arena (penetration-solver calls)
        const int64_t need = 64 + 24 * (int64_t)rlgpu::ceil_div(e->cfg.num_arenas, rl::kArenas) + e->cfg.num_arenas;
        RLGPU_REQUIRE(!d_counters || capacity >= need,
                      "rlgpu_envset_set_profile: buffer of " + std::to_string(capacity) + " counters, needs " + std::to_string(need));
        e->d_prof = d_counters;
    });
}

namespace {
const char* const kStepMetricNames[RLGPU_NUM_STEP_METRICS] = {
    "Player/In Air Ratio", "Player/Ball Touch Ratio", "Player/Demoed Ratio", "Player/Speed",
    "Player/Speed Towards Ball", "Player/Boost", "Player/Touch Height", "Game/Goal Speed"};
}

extern "C" const char* rlgpu_step_metric_name(int32_t i) {
    return i >= 0 && i < RLGPU_NUM_STEP_METRICS ? kStepMetricNames[i] : nullptr;
}

extern "C" int rlgpu_envset_enable_step_metrics(rlgpu_envset* e, int32_t enable) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e, "null envset");
        const size_t bytes = (size_t)e->cfg.num_arenas * RLGPU_STEP_METRIC_SLOTS * sizeof(double);
        if (enable && !e->d_metrics) RLGPU_CHECK_HIP(hipMalloc(&e->d_metrics, bytes));
        if (!enable && e->d_metrics) {
            RLGPU_CHECK_HIP(hipDeviceSynchronize());
            (void)hipFree(e->d_metrics);
            e->d_metrics = nullptr;
        }
        if (enable) RLGPU_CHECK_HIP(hipMemset(e->d_metrics, 0, bytes));
        e->metric_calls = 0;
    });
}

extern "C" int rlgpu_envset_step_metric_slots(rlgpu_envset* e, double* h_out, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e && h_out, "null argument");
        RLGPU_REQUIRE(e->d_metrics, "step metrics are not enabled (rlgpu_envset_enable_step_metrics)");
        hipStream_t s = rlgpu::as_stream(stream);
        RLGPU_CHECK_HIP(hipMemcpyAsync(h_out, e->d_metrics,
                                       (size_t)e->cfg.num_arenas * RLGPU_STEP_METRIC_SLOTS * sizeof(double),
                                       hipMemcpyDeviceToHost, s));
        RLGPU_CHECK_HIP(hipStreamSynchronize(s));
    });
}

extern "C" int rlgpu_envset_step_metrics(rlgpu_envset* e, double* h_total, uint64_t* h_count, int32_t reset,
                                         void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e, "null envset");
        RLGPU_REQUIRE(e->d_metrics, "step metrics are not enabled (rlgpu_envset_enable_step_metrics)");
        const int n = e->cfg.num_arenas;
        std::vector<double> slots((size_t)n * RLGPU_STEP_METRIC_SLOTS);
        hipStream_t s = rlgpu::as_stream(stream);
        RLGPU_CHECK_HIP(hipMemcpyAsync(slots.data(), e->d_metrics, slots.size() * sizeof(double), hipMemcpyDeviceToHost, s));
        RLGPU_CHECK_HIP(hipStreamSynchronize(s));
        double tot[RLGPU_NUM_STEP_METRICS] = {};
        double passes = 0, goals = 0;
        for (int a = 0; a < n; a++) {
            const double* m = &slots[(size_t)a * RLGPU_STEP_METRIC_SLOTS];
            for (int k = 0; k < RLGPU_SM_GOAL_SPEED; k++)
                for (int p = 0; p < 4; p++) tot[k] += m[k * 4 + p];
            tot[RLGPU_SM_GOAL_SPEED] += m[RLGPU_SM_SLOT_GOAL_SPEED];
            goals += m[RLGPU_SM_SLOT_GOALS];
            passes += m[RLGPU_SM_SLOT_PASSES];
        }
        if (h_total)
            for (int k = 0; k < RLGPU_NUM_STEP_METRICS; k++) h_total[k] = tot[k];
        if (h_count) {
            for (int k = 0; k < RLGPU_SM_TOUCH_HEIGHT; k++) h_count[k] = (uint64_t)(4 * passes);
            h_count[RLGPU_SM_TOUCH_HEIGHT] = (uint64_t)tot[RLGPU_SM_BALL_TOUCH];  // one AddAvg per touching player
            h_count[RLGPU_SM_GOAL_SPEED] = (uint64_t)goals;
        }
        if (reset) RLGPU_CHECK_HIP(hipMemsetAsync(e->d_metrics, 0, slots.size() * sizeof(double), s));
    });
}

extern "C" int rlgpu_envset_destroy(rlgpu_envset* e) {
    return rlgpu::guarded([&] {
        if (!e) return;
        if (e->d_metrics) (void)hipFree(e->d_metrics);
        (void)hipFree(e->d_arenas);
        (void)hipFree(e->d_obs);
        (void)hipFree(e->d_trunc_obs);
        (void)hipFree(e->d_rewards);
        (void)hipFree(e->d_last_rewards);
        (void)hipFree(e->d_masks);
        (void)hipFree(e->d_terminals);
        (void)hipFree(e->d_cell_tri);
        (void)hipFree(e->d_tri);
        (void)hipFree(e->d_edge);
        (void)hipFree(e->d_gjk);
        (void)hipFree(e->d_cell_start);
        (void)hipFree(e->d_plug);
        (void)hipFree(e->d_player_start);
        if (e->d_reward_values) (void)hipFree(e->d_reward_values);
        delete e;
    });
}

extern "C" int rlgpu_envset_enable_reward_values(rlgpu_envset* e, int32_t enable) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e, "null envset");
        RLGPU_CHECK_HIP(hipDeviceSynchronize());
        if (e->d_reward_values) (void)hipFree(e->d_reward_values);
        e->d_reward_values = nullptr;
        if (enable) {
            const size_t n = (size_t)e->num_players * std::max(e->plug.nr, 1);
            RLGPU_CHECK_HIP(hipMalloc(&e->d_reward_values, n * sizeof(float)));
            RLGPU_CHECK_HIP(hipMemset(e->d_reward_values, 0, n * sizeof(float)));
        }
    });
}

extern "C" float* rlgpu_envset_reward_values(rlgpu_envset* e) { return e ? e->d_reward_values : nullptr; }

extern "C" int rlgpu_envset_download_gamestates(rlgpu_envset* e, int32_t first, int32_t count, rlgpu_gamestate* h_out,
                                                void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e && h_out, "rlgpu_envset_download_gamestates: null argument");
        RLGPU_REQUIRE(first >= 0 && count >= 0 && first + count <= e->cfg.num_arenas, "arena range out of bounds");
        if (count == 0) return;
        RLGPU_CHECK_HIP(hipStreamSynchronize((hipStream_t)stream));
        std::vector<rlgpu_arena_state> rec((size_t)count);
        RLGPU_CHECK_HIP(hipMemcpy2D(rec.data(), sizeof(rlgpu_arena_state), e->d_arenas + (size_t)first * rl::kRec, rl::kRec,
                                    sizeof(rlgpu_arena_state), count, hipMemcpyDeviceToHost));
        rlgpu::gamestates_from_arenas(rec.data(), count, e->cfg.tick_skip, h_out);
    });
}

extern "C" int rlgpu_envset_buffers_get(rlgpu_envset* e, rlgpu_envset_buffers* out) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e && out, "rlgpu_envset_buffers_get: null argument");
        out->obs = e->d_obs;
        out->action_masks = e->d_masks;
        out->rewards = e->d_rewards;
        out->terminals = e->d_terminals;
        out->last_rewards = e->d_last_rewards;
        out->trunc_obs = e->d_trunc_obs;
        out->num_players = e->num_players;
        out->num_arenas = e->cfg.num_arenas;
        out->num_rewards = e->plug.nr;
        out->arena_player_start = e->d_player_start;
    });
}

extern "C" int rlgpu_envset_reset(rlgpu_envset* e, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e, "null envset");
        rl::StepArgs g = blank();
        g.reset_mode = 2;
        launch(e, g, rlgpu::as_stream(stream));
    });
}

extern "C" int rlgpu_envset_reset_arenas(rlgpu_envset* e, const uint8_t* d_mask, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e, "null envset");
        rl::StepArgs g = blank();
        g.reset_mode = 3;
        g.reset_mask = d_mask;
        launch(e, g, rlgpu::as_stream(stream));
    });
}

extern "C" int rlgpu_envset_step_first_half(rlgpu_envset* e, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e, "null envset");
        rl::StepArgs g = blank();
        g.ticks_first = e->cfg.action_delay;
        if (g.ticks_first == 0) {  // still snapshot prev state / clear events
            g.ticks_first = 0;
        }
        launch(e, g, rlgpu::as_stream(stream));
    });
}

extern "C" int rlgpu_envset_step_second_half(rlgpu_envset* e, const int32_t* d_actions, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e && d_actions, "rlgpu_envset_step_second_half: null argument");
        rl::StepArgs g = blank();
        g.actions = d_actions;
        g.ticks_second = e->cfg.tick_skip - e->cfg.action_delay;
        g.build = 1;
        launch(e, g, rlgpu::as_stream(stream));
    });
}

extern "C" int rlgpu_envset_step(rlgpu_envset* e, const int32_t* d_actions, int32_t reset_terminated,
                                 const rlgpu_step_outputs* out, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e && d_actions, "rlgpu_envset_step: null argument");
        RLGPU_REQUIRE(e->cfg.action_delay > 0, "fused step needs actionDelay > 0");
        rl::StepArgs g = blank();
        g.ticks_first = e->cfg.action_delay;
        g.actions = d_actions;
        g.ticks_second = e->cfg.tick_skip - e->cfg.action_delay;
        g.build = 1;
        g.reset_mode = reset_terminated ? 1 : 0;
        if (out) {
            g.out_obs = out->obs;
            g.out_masks = out->masks;
            g.out_rew = out->rewards;
            g.out_term = out->terminals;
            g.out_trunc = out->trunc_obs;
        }
        launch(e, g, rlgpu::as_stream(stream));
    });
}

extern "C" int rlgpu_envset_step_range(rlgpu_envset* e, int32_t first, int32_t count, const int32_t* d_actions,
                                       int32_t reset_terminated, const rlgpu_step_outputs* out, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e && d_actions, "rlgpu_envset_step_range: null argument");
        RLGPU_REQUIRE(e->cfg.action_delay > 0, "fused step needs actionDelay > 0");
        RLGPU_REQUIRE(first >= 0 && count > 0 && first + count <= e->cfg.num_arenas && first % rl::kArenas == 0,
                      "rlgpu_envset_step_range: the range must lie in the set and start at a multiple of 4");
        RLGPU_REQUIRE(!e->d_prof, "rlgpu_envset_step_range: not with the per-phase profile");
        rl::StepArgs g = blank();
        g.ticks_first = e->cfg.action_delay;
        g.actions = d_actions;
        g.ticks_second = e->cfg.tick_skip - e->cfg.action_delay;
        g.build = 1;
        g.reset_mode = reset_terminated ? 1 : 0;
        if (out) {
            g.out_obs = out->obs;
            g.out_masks = out->masks;
            g.out_rew = out->rewards;
            g.out_term = out->terminals;
            g.out_trunc = out->trunc_obs;
        }
        if (first == 0 && e->d_metrics) e->metric_players = (++e->metric_calls % 4) == 0;  // one StepCallback call
        launch_range(e, g, first, count, e->metric_players, rlgpu::as_stream(stream));
    });
}

extern "C" int rlgpu_envset_set_output_only(rlgpu_envset* e, int32_t enable) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e, "null envset");
        e->output_only = enable != 0;
    });
}

extern "C" int rlgpu_envset_sync(rlgpu_envset* e, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e, "null envset");
        RLGPU_CHECK_HIP(hipStreamSynchronize(rlgpu::as_stream(stream)));
    });
}

extern "C" int rlgpu_envset_build_obs(rlgpu_envset* e, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e, "null envset");
        rl::StepArgs g = blank();
        g.reset_mode = 5;
        launch(e, g, rlgpu::as_stream(stream));
    });
}

extern "C" int rlgpu_envset_get_arenas(rlgpu_envset* e, int32_t first, int32_t count, rlgpu_arena_state* h_out) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e && h_out, "null argument");
        RLGPU_REQUIRE(first >= 0 && count >= 0 && first + count <= e->cfg.num_arenas, "arena range out of bounds");
        if (count == 0) return;
        RLGPU_CHECK_HIP(hipDeviceSynchronize());
        RLGPU_CHECK_HIP(hipMemcpy2D(h_out, sizeof(rlgpu_arena_state), e->d_arenas + (size_t)first * rl::kRec, rl::kRec,
                                    sizeof(rlgpu_arena_state), count, hipMemcpyDeviceToHost));
    });
}

extern "C" int rlgpu_envset_set_arenas(rlgpu_envset* e, int32_t first, int32_t count, const rlgpu_arena_state* h_in) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(e && h_in, "null argument");
        RLGPU_REQUIRE(first >= 0 && count >= 0 && first + count <= e->cfg.num_arenas, "arena range out of bounds");
        if (count == 0) return;
        RLGPU_CHECK_HIP(hipDeviceSynchronize());
        RLGPU_CHECK_HIP(hipMemcpy2D(e->d_arenas + (size_t)first * rl::kRec, rl::kRec, h_in, sizeof(rlgpu_arena_state),
                                    sizeof(rlgpu_arena_state), count, hipMemcpyHostToDevice));
    });
}

// ------------------------------------------------------------------ box-triangle queries (tests)
namespace rl {
// lds != 0: each lane first tries a small LDS work set of its own, as the env kernel's lanes do
__global__ void __launch_bounds__(16) box_triangle_kernel(int n, const float* rot, const float* centre, const float* tri,
                                                          const float* cbt, float* out, gjk::GjkScratch* scratch,
                                                          int lds, int ar) {
    __shared__ char small[16][gjk::kSmallBytes];
    __shared__ int lock[16];
    const int i = blockIdx.x * 16 + threadIdx.x;
    lock[threadIdx.x] = 0;
    if (i >= n) return;
    const float* r = rot + 9 * (size_t)i;
    const m3 R = m3{v3{r[0], r[1], r[2]}, v3{r[3], r[4], r[5]}, v3{r[6], r[7], r[8]}};
    const v3 c = v3{centre[3 * (size_t)i], centre[3 * (size_t)i + 1], centre[3 * (size_t)i + 2]};
    const float* t = tri + 9 * (size_t)i;
    const gjk::Shape sh{C.car_impl, C.car_margin, v3{t[0], t[1], t[2]}, v3{t[3], t[4], t[5]}, v3{t[6], t[7], t[8]}, ar};
    v3 nrm, pt;
    float d = 0.f;
    gjk::Scr slow = gjk::hbm_view(scratch + i);
    gjk::Scr fast = gjk::lds_view(small[threadIdx.x]);
    const bool hit = gjk::box_triangle(R, c, sh, cbt[i], lds ? &fast : nullptr, &lock[threadIdx.x], slow, nrm, pt, d);
    float* o = out + 8 * (size_t)i;
    o[0] = hit ? 1.f : 0.f;
    o[1] = hit ? nrm.x : 0.f;
    o[2] = hit ? nrm.y : 0.f;
    o[3] = hit ? nrm.z : 0.f;
    o[4] = hit ? pt.x : 0.f;
    o[5] = hit ? pt.y : 0.f;
    o[6] = hit ? pt.z : 0.f;
    o[7] = hit ? d : 0.f;
}
// lds == 2: the env kernel's narrowphase scheme -- 64 lanes each run a query with the penetration solver
// deferred, then the whole wave runs the deferred queries one at a time with the wave-mode EPA; lds == 3:
// the same with a 6-vertex wave set, so that EPA runs overflow and rerun on the HBM set
__device__ __forceinline__ void bt_load(int i, const float* rot, const float* centre, const float* tri, int ar, m3& R, v3& c,
                                        gjk::Shape& sh) {
    const float* r = rot + 9 * (size_t)i;
    R = m3{v3{r[0], r[1], r[2]}, v3{r[3], r[4], r[5]}, v3{r[6], r[7], r[8]}};
    c = v3{centre[3 * (size_t)i], centre[3 * (size_t)i + 1], centre[3 * (size_t)i + 2]};
    const float* t = tri + 9 * (size_t)i;
    sh = gjk::Shape{C.car_impl, C.car_margin, v3{t[0], t[1], t[2]}, v3{t[3], t[4], t[5]}, v3{t[6], t[7], t[8]}, ar};
}
__device__ __forceinline__ void bt_store(float* out, int i, bool hit, v3 nrm, v3 pt, float d) {
    float* o = out + 8 * (size_t)i;
    o[0] = hit ? 1.f : 0.f;
    o[1] = hit ? nrm.x : 0.f;
    o[2] = hit ? nrm.y : 0.f;
    o[3] = hit ? nrm.z : 0.f;
    o[4] = hit ? pt.x : 0.f;
    o[5] = hit ? pt.y : 0.f;
    o[6] = hit ? pt.z : 0.f;
    o[7] = hit ? d : 0.f;
}
__global__ void __launch_bounds__(64) box_triangle_wave_kernel(int n, const float* rot, const float* centre, const float* tri,
                                                               const float* cbt, float* out, gjk::GjkScratch* scratch, int ar,
                                                               int tiny) {
    __shared__ char small[gjk::kSmallBytes];
    const int i = blockIdx.x * 64 + threadIdx.x;
    gjk::Scr slow = gjk::hbm_view(scratch + i);  // scratch holds a set for every lane of the grid
    bool deferred = false;
    gjk::PenState st{};
    if (i < n) {
        m3 R;
        v3 c, nrm, pt;
        gjk::Shape sh;
        float d = 0.f;
        bt_load(i, rot, centre, tri, ar, R, c, sh);
        const bool hit = gjk::box_triangle(R, c, sh, cbt[i], nullptr, nullptr, slow, nrm, pt, d, nullptr, gjk::kPenDefer,
                                           &deferred, &st);
        if (!deferred) bt_store(out, i, hit, nrm, pt, d);
    }
    uint64_t m = __ballot(deferred);
    while (m) {
        const int j = gjk::lowbit(m), q = blockIdx.x * 64 + j;
        m &= m - 1ull;
        m3 R;
        v3 c, nrm, pt;
        gjk::Shape sh;
        float d = 0.f;
        bt_load(q, rot, centre, tri, ar, R, c, sh);
        gjk::Scr wave = gjk::wave_view(small);
        if (tiny) wave.max_sv = 6;  // two EPA vertices, then the overflow rerun on the HBM set
        // even queries resume from the deferring lane's saved state, odd ones start over (both env paths)
        const gjk::PenState rs{gjk::rdl(st.pA, j), gjk::rdl(st.pB, j), gjk::rdl(st.nB, j), gjk::rdl(st.dist, j),
                               (int)gjk::rdl((uint32_t)st.valid, j)};
        const bool hit = gjk::box_triangle(R, c, sh, cbt[q], &wave, nullptr, slow, nrm, pt, d, nullptr, gjk::kPenWave,
                                           nullptr, nullptr, (q & 1) ? nullptr : &rs);
        if (threadIdx.x == 0) bt_store(out, q, hit, nrm, pt, d);
    }
}
}  // namespace rl

extern "C" int rlgpu_box_triangle_queries(int32_t n, const float* d_rot, const float* d_centre, const float* d_tri,
                                          const float* d_cbt, float* d_out, int32_t lds_first, int32_t arith, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(n >= 0, "rlgpu_box_triangle_queries: n must be >= 0");
        RLGPU_REQUIRE(arith >= 0 && arith < RLGPU_NUM_ARITH, "rlgpu_box_triangle_queries: unknown arithmetic mode");
        if (n == 0) return;
        RLGPU_REQUIRE(d_rot && d_centre && d_tri && d_cbt && d_out, "rlgpu_box_triangle_queries: null argument");
        ensure_const();
        if (rl::sse_api(arith)) ensure_rsqrt();
        hipStream_t s = (hipStream_t)stream;
        RLGPU_REQUIRE(lds_first >= 0 && lds_first <= 3, "rlgpu_box_triangle_queries: lds_first must be 0 .. 3");
        void* scratch = nullptr;
        const int lanes = lds_first >= 2 ? rlgpu::ceil_div(n, 64) * 64 : n;
        RLGPU_CHECK_HIP(hipMallocAsync(&scratch, (size_t)lanes * sizeof(rl::gjk::GjkScratch), s));
        if (lds_first >= 2)
            hipLaunchKernelGGL(rl::box_triangle_wave_kernel, dim3(lanes / 64), dim3(64), 0, s, n, d_rot, d_centre, d_tri,
                               d_cbt, d_out, (rl::gjk::GjkScratch*)scratch, (int)arith, (int)(lds_first == 3));
        else
            hipLaunchKernelGGL(rl::box_triangle_kernel, dim3(rlgpu::ceil_div(n, 16)), dim3(16), 0, s, n, d_rot, d_centre,
                               d_tri, d_cbt, d_out, (rl::gjk::GjkScratch*)scratch, (int)lds_first, (int)arith);
        RLGPU_CHECK_HIP(hipGetLastError());
        RLGPU_CHECK_HIP(hipFreeAsync(scratch, s));
    });
}

// ------------------------------------------------------------------ LinearMath queries (tests)
namespace rl {
// one query per lane of dmath.hpp's mode-dependent operations (rlgpu_linear_math_queries)
__global__ void __launch_bounds__(64) linear_math_kernel(int op, int ar, const float* in, int n, float* out) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const float* p = in + 24 * (size_t)i;
    float* o = out + 12 * (size_t)i;
    const m3 m = m3{v3{p[0], p[1], p[2]}, v3{p[3], p[4], p[5]}, v3{p[6], p[7], p[8]}};
    auto put9 = [&](const m3& r, float* q) {
        q[0] = r.r0.x; q[1] = r.r0.y; q[2] = r.r0.z;
        q[3] = r.r1.x; q[4] = r.r1.y; q[5] = r.r1.z;
        q[6] = r.r2.x; q[7] = r.r2.y; q[8] = r.r2.z;
    };
    if (op == 0) {
        const v3 v = bt_normalize(v3{p[0], p[1], p[2]}, ar);
        o[0] = v.x; o[1] = v.y; o[2] = v.z;
    } else if (op == 1) {
        put9(mat_from_quat(quat{p[0], p[1], p[2], p[3]}, ar), o);
    } else if (op == 2) {
        const quat q = quat_from_mat(m, ar);
        o[0] = q.x; o[1] = q.y; o[2] = q.z; o[3] = q.w;
    } else if (op == 3) {
        const quat q = qmul(quat{p[0], p[1], p[2], p[3]}, quat{p[4], p[5], p[6], p[7]}, ar);
        o[0] = q.x; o[1] = q.y; o[2] = q.z; o[3] = q.w;
    } else if (op == 4) {
        v3 np;
        m3 nr;
        integrate_transform(v3{p[9], p[10], p[11]}, m, v3{p[12], p[13], p[14]}, v3{p[15], p[16], p[17]}, kTick, np, nr, ar);
        o[0] = np.x; o[1] = np.y; o[2] = np.z;
        put9(nr, o + 3);
    } else if (op == 6) {  // rsqrtss of the first 12 floats of the row (the table lookup)
        for (int k = 0; k < 12; k++) o[k] = x86_rsqrtss(p[k]);
    } else if (op == 7) {  // the transcendentals (include/rlgpu_detmath.h)
        rs_sincosf(p[0], &o[0], &o[1]);
        o[2] = rs_atan2f(p[1], p[2]);
        o[3] = rs_asinf(p[3]);
        o[4] = rs_atanf(p[4]);
    } else {
        // a wheel ray's btSubsimplexConvexCast: R = p[0..8], from p[9..11], to p[12..14], body origin p[15..17],
        // box half extents p[18..20], sphere radius p[21] (> 0: sphere)
        float f = 0.f;
        v3 n = zero3();
        const bool hit = gjk::ray_convex_cast(v3{p[9], p[10], p[11]}, v3{p[12], p[13], p[14]}, p[21],
                                              v3{p[18], p[19], p[20]}, m, v3{p[15], p[16], p[17]}, ar, f, n);
        o[0] = hit ? 1.f : 0.f; o[1] = f; o[2] = n.x; o[3] = n.y; o[4] = n.z;
    }
}
}  // namespace rl

extern "C" int rlgpu_linear_math_queries(int32_t op, int32_t arith, const float* d_in, int32_t n, float* d_out, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(op >= 0 && op <= 7, "rlgpu_linear_math_queries: op must be in [0, 7]");
        RLGPU_REQUIRE(arith >= 0 && arith < RLGPU_NUM_ARITH, "rlgpu_linear_math_queries: unknown arithmetic mode");
        RLGPU_REQUIRE(n >= 0 && (n == 0 || (d_in && d_out)), "rlgpu_linear_math_queries: bad argument");
        if (n == 0) return;
        if (rl::sse_api(arith)) ensure_rsqrt();
        hipLaunchKernelGGL(rl::linear_math_kernel, dim3(rlgpu::ceil_div(n, 64)), dim3(64), 0, (hipStream_t)stream, (int)op,
                           (int)arith, d_in, (int)n, d_out);
        RLGPU_CHECK_HIP(hipGetLastError());
    });
}

// ------------------------------------------------------------------ box-box queries (tests)
namespace rl {
__global__ void __launch_bounds__(64) box_box_kernel(int n, const float* ra, const float* ca, const float* rb,
                                                     const float* cb, float* out) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const float* a = ra + 9 * (size_t)i;
    const float* b = rb + 9 * (size_t)i;
    const m3 Ra = m3{v3{a[0], a[1], a[2]}, v3{a[3], a[4], a[5]}, v3{a[6], a[7], a[8]}};
    const m3 Rb = m3{v3{b[0], b[1], b[2]}, v3{b[3], b[4], b[5]}, v3{b[6], b[7], b[8]}};
    const v3 pa = v3{ca[3 * (size_t)i], ca[3 * (size_t)i + 1], ca[3 * (size_t)i + 2]};
    const v3 pb = v3{cb[3 * (size_t)i], cb[3 * (size_t)i + 1], cb[3 * (size_t)i + 2]};
    float* o = out + 29 * (size_t)i;
    for (int k = 0; k < 29; k++) o[k] = 0.f;
    int cnt = 0;
    boxbox::box_box(pa, Ra, C.car_half, pb, Rb, C.car_half, [&](v3 nn, v3 p, float d) {
        float* q = o + 1 + 7 * cnt++;
        q[0] = nn.x; q[1] = nn.y; q[2] = nn.z; q[3] = p.x; q[4] = p.y; q[5] = p.z; q[6] = d;
    });
    o[0] = (float)cnt;
}
}  // namespace rl

extern "C" int rlgpu_box_box_queries(int32_t n, const float* d_rot_a, const float* d_centre_a, const float* d_rot_b,
                                     const float* d_centre_b, float* d_out, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(n >= 0, "rlgpu_box_box_queries: n must be >= 0");
        if (n == 0) return;
        RLGPU_REQUIRE(d_rot_a && d_centre_a && d_rot_b && d_centre_b && d_out, "rlgpu_box_box_queries: null argument");
        ensure_const();
        hipLaunchKernelGGL(rl::box_box_kernel, dim3(rlgpu::ceil_div(n, 64)), dim3(64), 0, (hipStream_t)stream, n, d_rot_a,
                           d_centre_a, d_rot_b, d_centre_b, d_out);
        RLGPU_CHECK_HIP(hipGetLastError());
    });
}
