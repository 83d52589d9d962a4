// env_ref.cpp -- ORACLE (test infrastructure only; never linked into the product).
//
// Restatement of the RLGymCPP environment layer on top of rsim_ref.cpp:
//   EnvSet two-half step / reset     GigaLearnCPP/RLGymCPP/src/RLGymCPP/EnvSet/EnvSet.cpp:113-354
//   GameState / Player snapshot      .../Gamestates/GameState.cpp:60-131, Player.cpp:8-25
//   AdvancedObs                      .../ObsBuilders/AdvancedObs.cpp:108-270 (+ AdvancedObs.h:10-13)
//   DefaultAction table + masks      .../ActionParsers/DefaultAction.cpp:3-118
//   rewards (ExampleMain list)       src/ExampleMain.cpp:132-177, .../Rewards/CommonRewards.h,
//                                    .../Rewards/KickoffProximityReward2v2Enhanced.h,
//                                    .../Rewards/ZeroSumReward.cpp (pass-through on the hot path)
//   terminal conditions              .../TerminalConditions/NoTouchCondition.h, src/ExampleMain.cpp:46-82
//   thread pool (CPU baseline)       .../ThreadPool.h:40-67 (contiguous chunks, one per thread)
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <limits>
#include <mutex>
#include <thread>
#include <vector>

#include "rsim_ref.hpp"

namespace orc {

// ------------------------------------------------------------------ DefaultAction (DefaultAction.cpp:3-89)
struct ActionTable {
    float a[RLGPU_ACTIONS][8];
    uint8_t ground[RLGPU_ACTIONS], air[RLGPU_ACTIONS], jump[RLGPU_ACTIONS], boost[RLGPU_ACTIONS];
    ActionTable() {
        const float RB[2] = {0, 1}, RF[3] = {-1, 0, 1};
        int n = 0;
        for (float th : RF)
            for (float st : RF)
                for (float bo : RB)
                    for (float hb : RB) {
                        if (bo == 1 && th != 1) continue;
                        float v[8] = {th, st, 0, st, 0, 0, bo, hb};
                        std::memcpy(a[n++], v, sizeof v);
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
                            std::memcpy(a[n++], v, sizeof v);
                        }
        for (int i = 0; i < n; i++) {
            const float* x = a[i];
            jump[i] = x[5] != 0;
            boost[i] = x[6] != 0;
            ground[i] = i < ng;
            air[i] = (i > ng && x[5] == 0);  // quirk: '>' drops action #24 (DefaultAction.cpp:78)
            if (i < ng && x[0] == x[6] && ((x[3] != 0) == (x[7] != 0))) air[i] = 1;
        }
    }
};
const ActionTable& actions() {
    static ActionTable t;
    return t;
}

// CommonValues::BOOST_LOCATIONS -> arena pad index (GameState.cpp:11-51)
struct PadMap {
    int map[RLGPU_PADS];
    PadMap() {
        const float loc[RLGPU_PADS][2] = {
            {0.f, -4240.0}, {-1792.0, -4184.0}, {1792.0, -4184.0}, {-3072.0, -4096.0}, {3072.0, -4096.0}, {-940.0, -3308.0},
            {940.0, -3308.0}, {0.0, -2816.0},   {-3584.0, -2484.0}, {3584.0, -2484.0}, {-1788.0, -2300.0}, {1788.0, -2300.0},
            {-2048.0, -1036.0}, {0.0, -1024.0}, {2048.0, -1036.0}, {-3584.0, 0.0},     {-1024.0, 0.0},     {1024.0, 0.0},
            {3584.0, 0.0},      {-2048.0, 1036.0}, {0.0, 1024.0},  {2048.0, 1036.0},   {-1788.0, 2300.0},  {1788.0, 2300.0},
            {-3584.0, 2484.0},  {3584.0, 2484.0},  {0.0, 2816.0},  {-940.0, 3310.0},   {940.0, 3308.0},    {-3072.0, 4096.0},
            {3072.0, 4096.0},   {-1792.0, 4184.0}, {1792.0, 4184.0}, {0.0, 4240.0}};
        const World& W = world();
        for (int i = 0; i < RLGPU_PADS; i++) {
            map[i] = -1;
            for (int j = 0; j < RLGPU_PADS; j++) {
                float dx = W.pad_pos_uu[j].x - loc[i][0], dy = W.pad_pos_uu[j].y - loc[i][1];
                if (dx * dx + dy * dy < 10) {
                    map[i] = j;
                    break;
                }
            }
        }
    }
};
const PadMap& padmap() {
    static PadMap m;
    return m;
}

// Player snapshot (uu), as the obs / reward code sees it.
struct PlayerView {
    V pos, vel, ang, fwd, right, up;
    float boost;
    bool on_ground, has_flip_or_jump, demoed, has_jumped, is_flipping, touched, orange;
    bool world_contact;
    float wc_normal_z;
};

static PlayerView view_player(const rlgpu_car& c, int i, bool touched) {
    PlayerView p;
    p.pos = ld3v(c.body.pos) * BT_TO_UU;
    p.vel = ld3v(c.body.vel) * BT_TO_UU;
    p.ang = ld3v(c.body.angvel);
    const float* r = c.body.rot;
    p.fwd = V(r[0], r[3], r[6]);
    p.right = V(r[1], r[4], r[7]);
    p.up = V(r[2], r[5], r[8]);
    p.boost = c.boost;
    p.on_ground = c.is_on_ground;
    // CarState::HasFlipOrJump (Car.cpp:279-283)
    p.has_flip_or_jump = c.is_on_ground || (!c.has_flipped && !c.has_double_jumped && c.air_time_since_jump < 1.25f);
    p.demoed = c.is_demoed;
    p.has_jumped = c.has_jumped;
    p.is_flipping = c.is_flipping;
    p.touched = touched;
    p.orange = i & 1;
    p.world_contact = c.world_contact;
    p.wc_normal_z = c.world_contact_normal[2];
    return p;
}

// ------------------------------------------------------------------ AdvancedObs
static void add_player_obs(float*& o, const PlayerView& pl, bool inv, V bpos, V bvel) {
    const float POS = 1.0f / 2300.0f, VEL = 1.0f / 2300.0f, ANG = 1.0f / 5.5f, BOOST = 0.01f;  // AdvancedObs.cpp:8-11
    auto iv = [&](V v) { return inv ? V(-v.x, -v.y, v.z) : v; };
    V pos = iv(pl.pos), vel = iv(pl.vel), ang = iv(pl.ang), f = iv(pl.fwd), r = iv(pl.right), u = iv(pl.up);
    o[0] = pos.x * POS; o[1] = pos.y * POS; o[2] = pos.z * POS;
    o[3] = f.x; o[4] = f.y; o[5] = f.z;
    o[6] = u.x; o[7] = u.y; o[8] = u.z;
    o[9] = vel.x * VEL; o[10] = vel.y * VEL; o[11] = vel.z * VEL;
    o[12] = ang.x * ANG; o[13] = ang.y * ANG; o[14] = ang.z * ANG;
    o[15] = (f.x * ang.x + f.y * ang.y + f.z * ang.z) * ANG;
    o[16] = (r.x * ang.x + r.y * ang.y + r.z * ang.z) * ANG;
    o[17] = (u.x * ang.x + u.y * ang.y + u.z * ang.z) * ANG;
    float rx = bpos.x - pos.x, ry = bpos.y - pos.y, rz = bpos.z - pos.z;
    o[18] = (f.x * rx + f.y * ry + f.z * rz) * POS;
    o[19] = (r.x * rx + r.y * ry + r.z * rz) * POS;
    o[20] = (u.x * rx + u.y * ry + u.z * rz) * POS;
    float vx = bvel.x - vel.x, vy = bvel.y - vel.y, vz = bvel.z - vel.z;
    o[21] = (f.x * vx + f.y * vy + f.z * vz) * VEL;
    o[22] = (r.x * vx + r.y * vy + r.z * vz) * VEL;
    o[23] = (u.x * vx + u.y * vy + u.z * vz) * VEL;
    o[24] = pl.boost * BOOST;
    o[25] = pl.on_ground ? 1.0f : 0.0f;
    o[26] = pl.has_flip_or_jump ? 1.0f : 0.0f;
    o[27] = pl.demoed ? 1.0f : 0.0f;
    o[28] = pl.has_jumped ? 1.0f : 0.0f;
    o += 29;
}

void build_obs_and_masks(const rlgpu_arena_state& s, const bool touched[4], float* obs_rows, uint8_t* mask_rows) {
    PlayerView P[4];
    for (int i = 0; i < 4; i++) P[i] = view_player(s.cars[i], i, touched[i]);
    V bpos = ld3v(s.ball.pos) * BT_TO_UU, bvel = ld3v(s.ball.vel) * BT_TO_UU, bang = ld3v(s.ball.angvel);
    const PadMap& pm = padmap();
    const ActionTable& at = actions();
    for (int pi = 0; pi < 4; pi++) {
        float* o = obs_rows + pi * RLGPU_OBS;
        bool inv = P[pi].orange;
        auto iv = [&](V v) { return inv ? V(-v.x, -v.y, v.z) : v; };
        V bp = iv(bpos), bv = iv(bvel), ba = iv(bang);
        const float BPOS = 1 / 5000.f, BVEL = 1 / 2300.f, BANG = 1 / 3.f;  // AdvancedObs.h:10-13 (member lookup)
        o[0] = bp.x * BPOS; o[1] = bp.y * BPOS; o[2] = bp.z * BPOS;
        o[3] = bv.x * BVEL; o[4] = bv.y * BVEL; o[5] = bv.z * BVEL;
        o[6] = ba.x * BANG; o[7] = ba.y * BANG; o[8] = ba.z * BANG;
        for (int k = 0; k < 8; k++) o[9 + k] = s.env.prev_action[pi][k];
        for (int k = 0; k < RLGPU_PADS; k++) {
            // GetBoostPads(inv) / GetBoostPadTimers(inv) -- the timers are the OTHER orientation (GameState.h:55-61)
            int act_idx = inv ? pm.map[RLGPU_PADS - k - 1] : pm.map[k];
            int tim_idx = inv ? pm.map[k] : pm.map[RLGPU_PADS - k - 1];
            bool active = s.pads[act_idx].is_active;
            float timer = s.pads[tim_idx].cooldown;
            o[17 + k] = active ? 1.0f : 1.0f / (1.0f + timer);
        }
        float* q = o + 51;
        add_player_obs(q, P[pi], inv, bp, bv);
        for (int j = 0; j < 4; j++)
            if (j != pi && P[j].orange == P[pi].orange) add_player_obs(q, P[j], inv, bp, bv);
        for (int j = 0; j < 4; j++)
            if (P[j].orange != P[pi].orange) add_player_obs(q, P[j], inv, bp, bv);
        // DefaultAction::GetActionMask (DefaultAction.cpp:91-118)
        uint8_t* m = mask_rows + pi * RLGPU_ACTIONS;
        for (int k = 0; k < RLGPU_ACTIONS; k++) {
            uint8_t r = P[pi].on_ground ? at.ground[k] : at.air[k];
            if (P[pi].boost == 0) r &= (uint8_t)~at.boost[k];
            bool turtled = P[pi].world_contact && P[pi].wc_normal_z > 0.9f;
            if (P[pi].has_flip_or_jump || turtled) r |= at.jump[k];
            m[k] = r & 1;
        }
    }
}

// ------------------------------------------------------------------ KickoffProximityReward2v2Enhanced
struct KickoffReward {
    struct Analysis {
        bool has_tm = false;
        int tm = -1;
        float tm_dist = 0, closest_opp = FLT_MAX, second_opp = FLT_MAX, avg_opp_speed = 0;
        V opp_com;
    };
    static V blue_back() { return V(0, -6000, 642.775f / 2); }
    static V orange_back() { return V(0, 6000, 642.775f / 2); }
    static float clampf(float v, float lo, float hi) { return std::min(std::max(v, lo), hi); }
    // goer = goerReward (KickoffProximityReward2v2Enhanced.h:9,135), rpw = rotationPrepWeight (:12,175)
    static float reward(int pi, const PlayerView* P, V bpos, V bvel, float goer, float rpw) {
        // IsKickoffActive
        float bspeed = rs_len(bvel);
        V b2(bpos.x, bpos.y, 0.f);
        if (!(bspeed < 2.f && bpos.z < 150.f && rs_len(b2) < 50.f)) return 0.f;
        const PlayerView& pl = P[pi];
        Analysis an;
        int nopp = 0;
        float tot_speed = 0;
        for (int j = 0; j < 4; j++) {
            const PlayerView& p = P[j];
            if (p.orange == pl.orange && j != pi) {
                an.tm = j;
                an.has_tm = true;
                an.tm_dist = rs_len(p.pos - bpos);
            } else if (p.orange != pl.orange) {
                float d = rs_len(p.pos - bpos);
                tot_speed += rs_len(p.vel);
                nopp++;
                if (d < an.closest_opp) {
                    an.second_opp = an.closest_opp;
                    an.closest_opp = d;
                } else if (d < an.second_opp) {
                    an.second_opp = d;
                }
                an.opp_com = an.opp_com + p.pos;
            }
        }
        if (nopp > 0) {
            float cf = (float)nopp;
            an.opp_com = rs_div(an.opp_com, cf);
            an.avg_opp_speed = tot_speed / cf;
        }
        if (!an.has_tm) return 0.f;
        const PlayerView& tm = P[an.tm];
        // DeterminePlayerRole
        float pdist = rs_len(pl.pos - bpos);
        float dscore = (pdist < an.tm_dist) ? 0.4f : 0.f;
        V p2b = rs_norm(bpos - pl.pos), t2b = rs_norm(bpos - tm.pos);
        float pvb = dot(pl.vel, p2b), tvb = dot(tm.vel, t2b);
        float sscore = (pvb > tvb) ? 0.3f : 0.f;
        float bscore = (pl.boost > tm.boost + 10.f) ? 0.2f : 0.f;
        float pa = rs_atan2f_at(pl.pos.y - bpos.y, pl.pos.x - bpos.x, RS_SITE_KICKOFF);
        float ta = rs_atan2f_at(tm.pos.y - bpos.y, tm.pos.x - bpos.x, RS_SITE_KICKOFF);
        float adiff = std::fabs(pa - ta);
        float spawn = (adiff > (3.14159f / 3.f)) ? 1.f : 0.f;
        float total = dscore + sscore + bscore + spawn * 0.1f;
        if (total >= 0.5f) {  // GOER
            float base = (pdist < an.closest_opp) ? goer : -goer * 0.5f;
            V to_b = rs_norm(bpos - pl.pos);
            float pvel = dot(pl.vel, to_b);
            float speed_bonus = clampf(pvel / 2300.f, -0.3f, 0.3f);
            float eff = 0.f;
            if (pl.boost > 50.f && pdist > 1000.f) eff = 0.1f;
            else if (pl.boost < 20.f && pdist > 800.f) eff = -0.15f;
            V vn = rs_norm(pl.vel);
            float approach = dot(to_b, vn);
            float angle_bonus = std::max(0.f, approach) * 0.2f;
            return clampf(base + speed_bonus + eff + angle_bonus, -1.5f, 1.5f);
        }
        // CHEATER
        V own = !pl.orange ? blue_back() : orange_back();
        V center(0.f, 0.f, 100.f);
        V cm(center.x * 1.3f, center.y * 1.3f, center.z * 1.3f);
        V base_ideal = (own + cm) * 0.5f;
        V threat = rs_norm(an.opp_com - own);
        threat = V(threat.x * 200.f, threat.y * 200.f, threat.z * 200.f);
        V tm_off(0.f, 0.f, 0.f);
        {
            float tdc = rs_len(tm.pos - center);
            if (tdc > 1500.f) {
                V dir = rs_norm(tm.pos - base_ideal);
                tm_off = V(dir.x * 300.f, dir.y * 300.f, dir.z * 300.f);
            }
        }
        V thr_adj(threat.x * 0.3f, threat.y * 0.3f, threat.z * 0.3f);
        V tm_adj(tm_off.x * 0.2f, tm_off.y * 0.2f, tm_off.z * 0.2f);
        V ideal = base_ideal + thr_adj + tm_adj;
        ideal.x = clampf(ideal.x, -3000.f, 3000.f);
        ideal.y = clampf(ideal.y, -4000.f, 4000.f);
        ideal.z = std::max(ideal.z, 17.f);
        float dti = rs_len(pl.pos - ideal);
        float posr;
        if (dti <= 600.f) posr = 0.5f * (1.f - (dti / 600.f));
        else if (dti <= 1200.f) posr = 0.5f * (1.f - (dti - 600.f) / (1200.f - 600.f)) * 0.7f;
        else if (dti <= 2000.f) posr = -0.1f * ((dti - 1200.f) / (2000.f - 1200.f));
        else posr = -0.3f;
        // strategic boost
        float best = 0.f;
        {
            const World& W = world();
            (void)W;
            static const float BL[RLGPU_PADS][3] = {
                {0.f, -4240.0, 70.0},  {-1792.0, -4184.0, 70.0}, {1792.0, -4184.0, 70.0}, {-3072.0, -4096.0, 73.0},
                {3072.0, -4096.0, 73.0}, {-940.0, -3308.0, 70.0}, {940.0, -3308.0, 70.0}, {0.0, -2816.0, 70.0},
                {-3584.0, -2484.0, 70.0}, {3584.0, -2484.0, 70.0}, {-1788.0, -2300.0, 70.0}, {1788.0, -2300.0, 70.0},
                {-2048.0, -1036.0, 70.0}, {0.0, -1024.0, 70.0}, {2048.0, -1036.0, 70.0}, {-3584.0, 0.0, 73.0},
                {-1024.0, 0.0, 70.0}, {1024.0, 0.0, 70.0}, {3584.0, 0.0, 73.0}, {-2048.0, 1036.0, 70.0},
                {0.0, 1024.0, 70.0}, {2048.0, 1036.0, 70.0}, {-1788.0, 2300.0, 70.0}, {1788.0, 2300.0, 70.0},
                {-3584.0, 2484.0, 70.0}, {3584.0, 2484.0, 70.0}, {0.0, 2816.0, 70.0}, {-940.0, 3310.0, 70.0},
                {940.0, 3308.0, 70.0}, {-3072.0, 4096.0, 73.0}, {3072.0, 4096.0, 73.0}, {-1792.0, 4184.0, 70.0},
                {1792.0, 4184.0, 70.0}, {0.0, 4240.0, 70.0}};
            for (int i = 0; i < RLGPU_PADS; i++) {
                V bp(BL[i][0], BL[i][1], BL[i][2]);
                if (bp.z > 72.0f) {
                    float dtb = rs_len(pl.pos - bp);
                    float acc = 1.f - clampf(dtb / 1500.f, 0.f, 1.f);
                    float d2b = rs_len(bp - bpos);
                    bool corner = (std::fabs(bp.x) > 2500.f && std::fabs(bp.y) > 3500.f);
                    float bv = corner ? 0.8f : 0.6f;
                    float prox = 1.f - clampf(d2b / 3000.f, 0.f, 1.f);
                    float strat = bv * (0.3f + prox * 0.7f);
                    float od = rs_len(an.opp_com - bp);
                    float deny = clampf(1.f - (od / 2000.f), 0.f, 0.3f);
                    float tv = acc * (strat + deny);
                    best = std::max(best, tv);
                }
            }
        }
        float blf = 1.f;
        if (pl.boost < 30.f) blf = 1.5f;
        else if (pl.boost > 80.f) blf = 0.5f;
        float boostr = best * blf * 0.25f;
        // rotation preparation
        float rot;
        {
            V t2g = rs_norm(own - tm.pos);
            V perp = rs_norm(V(-t2g.y, t2g.x, 0.f));
            V goff(t2g.x * 800.f, t2g.y * 800.f, t2g.z * 800.f);
            V poff(perp.x * 600.f, perp.y * 600.f, perp.z * 600.f);
            V sup = tm.pos + goff + poff;
            float dts = rs_len(pl.pos - sup);
            float ready = 1.f - clampf(dts / 1000.f, 0.f, 1.f);
            V tos = rs_norm(sup - pl.pos);
            float align = std::max(0.f, dot(rs_norm(pl.vel), tos));
            rot = (ready * 0.7f + align * 0.3f) * rpw;
        }
        float aware;
        {
            V toc = rs_norm(an.opp_com - pl.pos);
            V tob = rs_norm(bpos - pl.pos);
            float aa = dot(toc, tob);
            aware = clampf(aa * 0.5f + 0.5f, 0.f, 1.f) * 0.1f;
        }
        float camp;
        {
            float dtg = rs_len(pl.pos - own);
            float mind = 800.f;
            float bdg = rs_len(bpos - own);
            if (bdg < 2000.f) mind *= 0.7f;
            camp = 0.f;
            if (dtg < mind) camp = -0.4f * (1.f - (dtg / mind));
            camp *= 0.05f;
        }
        float tot = posr + boostr + rot + aware + camp;
        return clampf(tot, -0.8f, 0.8f);
    }
};

// ------------------------------------------------------------------ reward / terminal plugins
// The EnvCreateFn's WeightedReward list and TerminalCondition list (EnvSet.h:14-24), as the
// rlgpu_envset_config registry describes them.
struct Plugins {
    std::vector<rlgpu_reward_spec> rw;
    std::vector<rlgpu_terminal_spec> tc;
};
// src/ExampleMain.cpp:132-187
static Plugins example_main_plugins() {
    Plugins p;
    auto R = [&](int type, float w, float p0 = 0, float p1 = 0) {
        rlgpu_reward_spec r;
        std::memset(&r, 0, sizeof r);
        r.type = type;
        r.weight = w;
        r.params[0] = p0;
        r.params[1] = p1;
        p.rw.push_back(r);
    };
    R(RLGPU_RW_AIR, 0.25f);
    R(RLGPU_RW_WAVEDASH, 0.12f);
    R(RLGPU_RW_KICKOFF_PROXIMITY_2V2, 5.f);
    R(RLGPU_RW_VELOCITY_PLAYER_TO_BALL, 4.f);
    R(RLGPU_RW_STRONG_TOUCH, 60, 20, 120);
    R(RLGPU_RW_TOUCH_ACCEL, 6.f);
    R(RLGPU_RW_VELOCITY_BALL_TO_GOAL, 8.0f, 0);
    R(RLGPU_RW_PICKUP_BOOST, 0.1f);
    R(RLGPU_RW_SAVE_BOOST, 0.010f, 0.5f);
    R(RLGPU_RW_BUMP, 20);
    R(RLGPU_RW_DEMO, 80);
    R(RLGPU_RW_GOAL, 150, -1);
    R(RLGPU_RW_LOSING_PENALTY, 1.0f, 0.02f);
    p.tc.push_back(rlgpu_terminal_spec{RLGPU_TC_NO_TOUCH, 8.f});
    p.tc.push_back(rlgpu_terminal_spec{RLGPU_TC_SCORE_LIMIT, 3.f});
    return p;
}

// SaveBoostReward's powf(boost / 100, exponent): 0.5 as sqrtf (ExampleMain), else exp(b log a) on the
// deterministic kernels shared with the device (include/rlgpu_detmath.h)
static float powf_det(float a, float b) {
#ifdef RLGPU_DETMATH_LIBM
    if (RS_LIBM_AT(RS_SITE_POW)) return powf(a, b);  // the reference's call, host libm (tests/test_detmath_bound.py)
#endif
    if (b == 0.5f) return std::sqrt(a);
    if (b == 0.f) return 1.f;
    if (a == 0.f) return b > 0.f ? 0.f : std::numeric_limits<float>::infinity();
    return rs_expf(b * rs_logf(a));
}

// Reward::GetReward of one registry entry (CommonRewards.h:8-203, KickoffProximityReward2v2Enhanced.h,
// ExampleMain.cpp:84-124) for player i; CAR_MAX_SPEED 2300, BALL_MAX_SPEED 6000 (CommonValues.h)
static float reward_of(const rlgpu_reward_spec& rs, int i, const PlayerView* P, const rlgpu_env_extra& e, V bpos,
                       V bvel, V prev_bvel, bool goal) {
    const PlayerView& pl = P[i];
    const float KPH = 250.f / 9.f;  // Math::KPHToVel
    switch (rs.type) {
        case RLGPU_RW_AIR: return !pl.on_ground;
        case RLGPU_RW_WAVEDASH: return (pl.on_ground && (e.prev_is_flipping[i] && !e.prev_on_ground[i])) ? 1 : 0;
        case RLGPU_RW_KICKOFF_PROXIMITY_2V2:
            return KickoffReward::reward(i, P, bpos, bvel, rs.params[2] != 0.f ? rs.params[0] : 1.2f,
                                         rs.params[2] != 0.f ? rs.params[1] : 0.2f);
        case RLGPU_RW_VELOCITY_PLAYER_TO_BALL: {
            V dir = rs_norm(bpos - pl.pos);
            V nv = rs_div(pl.vel, 2300.f);
            return dot(dir, nv);
        }
        case RLGPU_RW_STRONG_TOUCH: {
            const float minv = rs.params[0] * KPH, maxv = rs.params[1] * KPH;
            if (!pl.touched) return 0;
            float hit = rs_len(bvel - prev_bvel);
            return hit < minv ? 0 : std::min(1.f, hit / maxv);
        }
        case RLGPU_RW_TOUCH_ACCEL: {
            const float MAXS = 110 * KPH;
            if (!pl.touched) return 0;
            float pf = std::min(1.f, rs_len(prev_bvel) / MAXS);
            float cf = std::min(1.f, rs_len(bvel) / MAXS);
            return cf > pf ? (cf - pf) : 0;
        }
        case RLGPU_RW_VELOCITY_BALL_TO_GOAL: {
            bool orange_goal = pl.orange == false;
            if (rs.params[0] != 0) orange_goal = !orange_goal;
            V tgt = orange_goal ? V(0, 6000, 642.775f / 2) : V(0, -6000, 642.775f / 2);
            V d = rs_norm(tgt - bpos);
            return dot(d, rs_div(bvel, 6000.f));
        }
        case RLGPU_RW_PICKUP_BOOST:
            return pl.boost > e.prev_boost[i] ? std::sqrt(pl.boost / 100.f) - std::sqrt(e.prev_boost[i] / 100.f) : 0;
        case RLGPU_RW_SAVE_BOOST: return std::min(std::max(powf_det(pl.boost / 100, rs.params[0]), 0.f), 1.f);
        case RLGPU_RW_BUMP: return e.ev_bump[i];
        case RLGPU_RW_DEMO: return e.ev_demo[i];
        case RLGPU_RW_BUMPED_PENALTY: return -(float)e.ev_bumped[i];
        case RLGPU_RW_DEMOED_PENALTY: return -(float)e.ev_demoed[i];
        case RLGPU_RW_GOAL: {
            if (!goal) return 0;
            bool ball_team_orange = !(bpos.y < 0);  // RS_TEAM_FROM_Y
            return (pl.orange != ball_team_orange) ? 1.f : rs.params[0];
        }
        case RLGPU_RW_LOSING_PENALTY: {
            int own = pl.orange ? e.penalty_orange : e.penalty_blue;
            int opp = pl.orange ? e.penalty_blue : e.penalty_orange;
            int deficit = opp - own;
            return deficit > 0 ? -rs.params[0] * (float)deficit : 0.f;
        }
        case RLGPU_RW_VELOCITY: return rs_len(pl.vel) / 2300.f * (float)(1 - 2 * (rs.params[0] != 0));
        case RLGPU_RW_FACE_BALL: return dot(pl.fwd, rs_norm(bpos - pl.pos));
        case RLGPU_RW_TOUCH_BALL: return pl.touched ? 1.f : 0.f;
        case RLGPU_RW_SPEED: return rs_len(pl.vel) / 2300.f;
    }
    return 0;
}

// ------------------------------------------------------------------ env step halves
struct StepOut {
    float* obs;
    uint8_t* masks;
    float* rewards;
    uint8_t* terminal;
    float* last_rewards;  // [number of rewards] of player 0 (may be null)
    int8_t* traj_term;    // [4] trajectory codes (Learner.cpp:829-861), may be null
    int max_episode_steps;
    const Plugins* plug;
};

// GameState::UpdateFromArena + terminals + rewards + obs/masks (EnvSet.cpp:157-270)
void second_half_builders(rlgpu_arena_state& s, const StepOut& out, int tick_skip_unused) {
    (void)tick_skip_unused;
    rlgpu_env_extra& e = s.env;
    int64_t cur = e.tick_count;
    int64_t tick_skip = std::max<int64_t>(cur - e.last_tick_count, 0);
    float delta_time = (int)tick_skip * (1.0f / 120.0f);
    bool touched[4];
    for (int i = 0; i < 4; i++) {
        const rlgpu_car& c = s.cars[i];
        touched[i] = c.ball_hit_valid && (uint64_t)c.ball_hit_tick >= (uint64_t)(cur - tick_skip);
    }
    V bpos = ld3v(s.ball.pos) * BT_TO_UU, bvel = ld3v(s.ball.vel) * BT_TO_UU;
    bool goal = std::fabs(s.ball.pos[1] * BT_TO_UU) > (5124.25f + 91.25f);  // Arena::IsBallScored
    PlayerView P[4];
    for (int i = 0; i < 4; i++) P[i] = view_player(s.cars[i], i, touched[i]);
    // terminal conditions of the list (EnvSet.cpp:163-181).  Every instance of NoTouchCondition
    // (NoTouchCondition.h:17-28) keeps the same timeSinceTouch and every ScoreLimitCondition
    // (ExampleMain.cpp:55-68) the same goal counts -- IsTerminal runs for all of them each step -- so
    // the arena holds one copy of each, updated every step.
    uint8_t term = 0;
    {
        bool any = touched[0] || touched[1] || touched[2] || touched[3];
        if (any) e.no_touch_time = 0;
        else e.no_touch_time += delta_time;
        if (goal) {
            if (bpos.y > 0) e.score_blue++;
            else e.score_orange++;
        }
        for (const rlgpu_terminal_spec& c : out.plug->tc) {
            bool terminal = false, truncation = false;
            switch (c.type) {
                case RLGPU_TC_NO_TOUCH:
                    terminal = !any && e.no_touch_time >= c.param;
                    truncation = true;
                    break;
                case RLGPU_TC_SCORE_LIMIT: {
                    int limit = (int)c.param;
                    terminal = (e.score_blue >= limit) || (e.score_orange >= limit);
                    break;
                }
                case RLGPU_TC_GOAL_SCORE: terminal = goal; break;  // GoalScoreCondition.h
            }
            if (!terminal) continue;
            uint8_t t = truncation ? 2 : 1;
            if (term == 0) term = t;
            else if (t == 1) term = 1;  // NORMAL dominates
        }
    }
    e.terminal = term;
    // trajectory-level code: maxEpisodeLength truncates without an arena reset (Learner.cpp:848-850)
    e.episode_steps++;
    int8_t tj = (int8_t)term;
    if (!tj && out.max_episode_steps > 0 && e.episode_steps >= out.max_episode_steps) tj = 2;
    if (tj) e.episode_steps = 0;
    if (out.traj_term)
        for (int i = 0; i < 4; i++) out.traj_term[i] = tj;
    // PreStep: LosingPenaltyReward
    if (goal) {
        if (bpos.y > 0) e.penalty_blue++;
        else e.penalty_orange++;
    }
    // rewards of the list; allRewards[i] += out[i] * weight in list order (EnvSet.cpp:183-222); lastRewards
    // holds each reward's value for the lowest car id, player 0 (:224-242; ZeroSumReward's inner rewards
    // stay empty on this path, so the value is the child's)
    float all[4] = {0, 0, 0, 0};
    V prev_bvel = ld3v(e.prev_ball_vel);
    const std::vector<rlgpu_reward_spec>& rw = out.plug->rw;
    for (size_t r = 0; r < rw.size(); r++) {
        float o[4];
        for (int i = 0; i < 4; i++) o[i] = reward_of(rw[r], i, P, e, bpos, bvel, prev_bvel, goal);
        for (int i = 0; i < 4; i++) all[i] += o[i] * rw[r].weight;
        if (out.last_rewards) out.last_rewards[r] = o[0];
    }
    for (int i = 0; i < 4; i++) out.rewards[i] = all[i];
    *out.terminal = term;
    e.last_tick_count = cur;
    build_obs_and_masks(s, touched, out.obs, out.masks);
}

// StepFirstHalf body for one arena (EnvSet.cpp:115-127)
void first_half(const World& w, rlgpu_arena_state& s, uint64_t seed, int idx, int action_delay) {
    rlgpu_env_extra& e = s.env;
    for (int i = 0; i < 3; i++) e.prev_ball_vel[i] = s.ball.vel[i] * BT_TO_UU;
    for (int i = 0; i < 4; i++) {
        e.prev_boost[i] = s.cars[i].boost;
        e.prev_is_flipping[i] = s.cars[i].is_flipping;
        e.prev_on_ground[i] = s.cars[i].is_on_ground;
        e.ev_bump[i] = e.ev_bumped[i] = e.ev_demo[i] = e.ev_demoed[i] = 0;  // ResetBeforeStep
    }
    e.has_prev = 1;
    arena_step(w, s, seed, idx, action_delay);
}

void second_half(const World& w, rlgpu_arena_state& s, uint64_t seed, int idx, int ticks, const int32_t* acts,
                 const StepOut& out) {
    const ActionTable& at = actions();
    for (int i = 0; i < 4; i++) {
        int a = std::min(std::max(acts[i], 0), RLGPU_ACTIONS - 1);
        const float* x = at.a[a];
        float* c = s.cars[i].controls;
        for (int k = 0; k < 5; k++) c[k] = x[k];
        c[5] = x[5] == 1 ? 1.f : 0.f;  // (CarControls)Action: jump/boost/handbrake == 1
        c[6] = x[6] == 1 ? 1.f : 0.f;
        c[7] = x[7] == 1 ? 1.f : 0.f;
        for (int k = 0; k < 8; k++) s.env.prev_action[i][k] = x[k];
    }
    arena_step(w, s, seed, idx, ticks);
    second_half_builders(s, out, ticks);
}

// EnvSet::ResetArena (EnvSet.cpp:275-304)
void reset_arena(rlgpu_arena_state& s, uint64_t seed, int idx, float* obs, uint8_t* masks, bool fuzz) {
    kickoff(s, seed, idx, fuzz);
    rlgpu_env_extra& e = s.env;
    e.last_tick_count = e.tick_count;  // new GameState(arena)
    e.no_touch_time = 0;
    e.score_blue = e.score_orange = 0;
    e.penalty_blue = e.penalty_orange = 0;
    e.has_prev = 0;
    e.terminal = 0;
    e.episode_steps = 0;
    std::memset(e.prev_action, 0, sizeof e.prev_action);
    for (int i = 0; i < 4; i++) e.ev_bump[i] = e.ev_bumped[i] = e.ev_demo[i] = e.ev_demoed[i] = 0;
    bool touched[4] = {false, false, false, false};  // fresh CarState: ballHitInfo invalid
    build_obs_and_masks(s, touched, obs, masks);
}

// ------------------------------------------------------------------ CPU thread pool (ThreadPool.h:40-67)
struct Pool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::function<void(int, int)> job;
    int njobs = 0, gen = 0, pending = 0;
    bool stop = false;
    explicit Pool(int n) {
        for (int t = 0; t < n; t++)
            th.emplace_back([this, t, n] {
                int seen = 0;
                for (;;) {
                    std::function<void(int, int)> j;
                    int total;
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [&] { return stop || gen != seen; });
                        if (stop) return;
                        seen = gen;
                        j = job;
                        total = njobs;
                    }
                    int per = (total + n - 1) / n, b0 = t * per, b1 = std::min(total, b0 + per);
                    if (b0 < b1) j(b0, b1);
                    {
                        std::lock_guard<std::mutex> lk(mu);
                        if (--pending == 0) done_cv.notify_all();
                    }
                }
            });
    }
    void run(int total, std::function<void(int, int)> f) {
        std::unique_lock<std::mutex> lk(mu);
        job = std::move(f);
        njobs = total;
        pending = (int)th.size();
        gen++;
        cv.notify_all();
        done_cv.wait(lk, [&] { return pending == 0; });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th) t.join();
    }
};

struct EnvSet {
    int n;
    uint64_t seed;
    int tick_skip, action_delay;
    std::vector<rlgpu_arena_state> arenas;
    std::vector<float> obs, trunc_obs, rewards, last_rewards;
    std::vector<uint8_t> masks, terminals;
    std::vector<int8_t> traj_terms;
    int max_episode_steps = 0;
    Plugins plug = example_main_plugins();
    Pool* pool = nullptr;
    int arith = RLGPU_ARITH_MSVC_X64;  // the reference build's arithmetic (oracle_env_set_arith)
    int arena_offset = 0;              // global index of arena 0 (the arenas' Philox streams)
    bool fuzz = false;                 // FuzzedKickoffState (rlgpu_envset_config.state_setter)
    World* own_world = nullptr;     // set by oracle_env_set_mesh
    std::vector<float> mesh_tris;   // its mesh, rebuilt when the arithmetic changes
    std::vector<int> mesh_obj;
    const World* w = &world(RLGPU_ARITH_MSVC_X64);
    ~EnvSet() {
        delete pool;
        delete own_world;
    }
    void par(std::function<void(int)> f) {
        if (!pool) {
            ArithScope scope(arith);
            for (int i = 0; i < n; i++) f(i);
            return;
        }
        pool->run(n, [&](int b0, int b1) {
            ArithScope scope(arith);
            for (int i = b0; i < b1; i++) f(i);
        });
    }
    void rebuild_world() {
        delete own_world;
        own_world = nullptr;
        if (mesh_tris.empty()) {
            w = &world(arith);
            return;
        }
        own_world = new World(arith);
        own_world->set_mesh(mesh_tris.data(), (int)(mesh_tris.size() / 9), mesh_obj.empty() ? nullptr : mesh_obj.data(),
                            (int)mesh_obj.size());
        w = own_world;
    }
    StepOut out(int i) {
        return {&obs[(size_t)i * 4 * RLGPU_OBS], &masks[(size_t)i * 4 * RLGPU_ACTIONS], &rewards[(size_t)i * 4], &terminals[i],
                &last_rewards[(size_t)i * RLGPU_MAX_REWARDS], &traj_terms[(size_t)i * 4], max_episode_steps, &plug};
    }
};

}  // namespace orc

using namespace orc;

extern "C" {

void* oracle_env_create(int num_arenas, uint64_t seed, int tick_skip, int action_delay, int threads, int arena_offset,
                        int state_setter) {
    EnvSet* e = new EnvSet();
    e->arena_offset = arena_offset;
    e->fuzz = state_setter == 1;
    e->n = num_arenas;
    e->seed = seed;
    e->tick_skip = tick_skip;
    e->action_delay = action_delay;
    e->arenas.resize(num_arenas);
    std::memset(e->arenas.data(), 0, sizeof(rlgpu_arena_state) * num_arenas);
    e->obs.assign((size_t)num_arenas * 4 * RLGPU_OBS, 0.f);
    e->trunc_obs.assign((size_t)num_arenas * 4 * RLGPU_OBS, 0.f);
    e->masks.assign((size_t)num_arenas * 4 * RLGPU_ACTIONS, 0);
    e->rewards.assign((size_t)num_arenas * 4, 0.f);
    e->last_rewards.assign((size_t)num_arenas * RLGPU_MAX_REWARDS, 0.f);
    e->terminals.assign(num_arenas, 0);
    e->traj_terms.assign((size_t)num_arenas * 4, 0);
    if (threads > 1) e->pool = new Pool(threads);
    for (int i = 0; i < num_arenas; i++) {
        rlgpu_arena_state& s = e->arenas[i];
        const World& W = world();
        stm(s.ball.rot, M::ident());
        s.ball.pos[2] = W.ball_radius;  // Ball::_BulletSetup start transform
        for (int c = 0; c < 4; c++) default_car(s.cars[c]);
        for (int p = 0; p < RLGPU_PADS; p++) s.pads[p].is_active = 1;
    }
    // EnvSet ctor: reset all arenas (EnvSet.cpp:105-110)
    e->par([&](int i) { reset_arena(e->arenas[i], e->seed, i + e->arena_offset, e->out(i).obs, e->out(i).masks, e->fuzz); });
    return e;
}

void oracle_env_destroy(void* h) { delete (EnvSet*)h; }

int oracle_arena_state_size(void) { return (int)sizeof(rlgpu_arena_state); }

void oracle_env_get_arenas(void* h, int first, int count, rlgpu_arena_state* out) {
    EnvSet* e = (EnvSet*)h;
    std::memcpy(out, &e->arenas[first], sizeof(rlgpu_arena_state) * count);
}

void oracle_env_set_arenas(void* h, int first, int count, const rlgpu_arena_state* in) {
    EnvSet* e = (EnvSet*)h;
    std::memcpy(&e->arenas[first], in, sizeof(rlgpu_arena_state) * count);
}

void oracle_env_step_first_half(void* h) {
    EnvSet* e = (EnvSet*)h;
    e->par([&](int i) { first_half(*e->w, e->arenas[i], e->seed, i + e->arena_offset, e->action_delay); });
}

void oracle_env_step_second_half(void* h, const int32_t* actions) {
    EnvSet* e = (EnvSet*)h;
    e->par([&](int i) {
        second_half(*e->w, e->arenas[i], e->seed, i + e->arena_offset, e->tick_skip - e->action_delay, actions + 4 * i, e->out(i));
    });
}

// EnvSet::Reset (EnvSet.cpp:306-354)
void oracle_env_reset(void* h) {
    EnvSet* e = (EnvSet*)h;
    e->par([&](int i) {
        if (e->terminals[i]) {
            e->terminals[i] = 0;
            reset_arena(e->arenas[i], e->seed, i + e->arena_offset, e->out(i).obs, e->out(i).masks, e->fuzz);
        }
    });
}

void oracle_env_reset_arenas(void* h, const uint8_t* mask) {
    EnvSet* e = (EnvSet*)h;
    e->par([&](int i) {
        if (!mask || mask[i]) reset_arena(e->arenas[i], e->seed, i + e->arena_offset, e->out(i).obs, e->out(i).masks, e->fuzz);
    });
}

// Fused step (first half + second half + optional reset); keeps terminals[] of the step.
void oracle_env_step(void* h, const int32_t* actions, int reset_terminated) {
    EnvSet* e = (EnvSet*)h;
    e->par([&](int i) {
        rlgpu_arena_state& s = e->arenas[i];
        first_half(*e->w, s, e->seed, i + e->arena_offset, e->action_delay);
        StepOut o = e->out(i);
        second_half(*e->w, s, e->seed, i + e->arena_offset, e->tick_skip - e->action_delay, actions + 4 * i, o);
        if (o.traj_term[0] == 2) std::memcpy(&e->trunc_obs[(size_t)i * 4 * RLGPU_OBS], o.obs, sizeof(float) * 4 * RLGPU_OBS);
        if (reset_terminated && *o.terminal) reset_arena(s, e->seed, i + e->arena_offset, o.obs, o.masks, e->fuzz);
    });
}

void oracle_env_build_obs(void* h) {
    EnvSet* e = (EnvSet*)h;
    e->par([&](int i) {
        bool touched[4] = {false, false, false, false};  // obs / masks do not read ballTouchedStep
        build_obs_and_masks(e->arenas[i], touched, e->out(i).obs, e->out(i).masks);
    });
}

void oracle_env_read(void* h, float* obs, uint8_t* masks, float* rewards, uint8_t* terminals, float* trunc_obs,
                     float* last_rewards) {
    EnvSet* e = (EnvSet*)h;
    if (obs) std::memcpy(obs, e->obs.data(), e->obs.size() * sizeof(float));
    if (masks) std::memcpy(masks, e->masks.data(), e->masks.size());
    if (rewards) std::memcpy(rewards, e->rewards.data(), e->rewards.size() * sizeof(float));
    if (terminals) std::memcpy(terminals, e->terminals.data(), e->terminals.size());
    if (trunc_obs) std::memcpy(trunc_obs, e->trunc_obs.data(), e->trunc_obs.size() * sizeof(float));
    if (last_rewards) std::memcpy(last_rewards, e->last_rewards.data(), e->last_rewards.size() * sizeof(float));
}

void oracle_env_set_max_episode_steps(void* h, int n) { ((EnvSet*)h)->max_episode_steps = n; }

// The reward / terminal lists (rlgpu_envset_config.rewards / terminals; NULL keeps ExampleMain's).
// last_rewards rows are RLGPU_MAX_REWARDS wide, the first n_rewards used.
void oracle_env_set_plugins(void* h, const rlgpu_reward_spec* rw, int nr, const rlgpu_terminal_spec* tc, int nt) {
    EnvSet* e = (EnvSet*)h;
    Plugins def = example_main_plugins();
    e->plug.rw = rw ? std::vector<rlgpu_reward_spec>(rw, rw + nr) : def.rw;
    e->plug.tc = tc ? std::vector<rlgpu_terminal_spec>(tc, tc + nt) : def.tc;
}

// Arena collision meshes for this set (rlgpu_envset_config.mesh_*): ntris x 9 floats (bullet
// units), object k owns the next obj_ntris[k] triangles (obj_ntris NULL: one object).
// internal-edge records of a mesh (btGenerateInternalEdgeInfo restated, edge_ref.hpp): ntris x 4 floats
// (3 angles, flags bits | 1 << 30 when the triangle has a record), the library's rlgpu_mesh_edge_info layout
void oracle_mesh_edge_info(const float* tris, int ntris, const int* obj_ntris, int nobj, int arith, float* out) {
    World wd(arith);
    wd.set_mesh(tris, ntris, obj_ntris, nobj);
    for (int t = 0; t < ntris; t++) {
        const TriInfo& ti = wd.tri_info[t];
        int flags = ti.flags | (ti.present ? (1 << 30) : 0);
        out[4 * t] = ti.e01;
        out[4 * t + 1] = ti.e12;
        out[4 * t + 2] = ti.e20;
        std::memcpy(&out[4 * t + 3], &flags, sizeof(int));
    }
}

void oracle_env_set_mesh(void* h, const float* tris, int ntris, const int* obj_ntris, int nobj) {
    EnvSet* e = (EnvSet*)h;
    e->mesh_tris.assign(tris, tris + (size_t)ntris * 9);
    if (obj_ntris) e->mesh_obj.assign(obj_ntris, obj_ntris + nobj);
    else e->mesh_obj.clear();
    e->rebuild_world();
}

// The reference build's arithmetic (RLGPU_ARITH_*, include/rlgpu_arith.h) for every later step; the set's
// edge records are rebuilt in it.
// Global index of arena 0 for the arenas' Philox streams (rlgpu_envset_config.arena_offset).
void oracle_env_set_arena_offset(void* h, int off) { ((EnvSet*)h)->arena_offset = off; }
// The state setter (RLGPU_SS_*): 1 = FuzzedKickoffState.  Resets from now on use it.
void oracle_env_set_state_setter(void* h, int ss) { ((EnvSet*)h)->fuzz = ss == 1; }

void oracle_env_set_arith(void* h, int arith) {
    EnvSet* e = (EnvSet*)h;
    e->arith = arith;
    e->rebuild_world();
}

void oracle_env_read_traj_terms(void* h, int8_t* out) {
    EnvSet* e = (EnvSet*)h;
    std::memcpy(out, e->traj_terms.data(), e->traj_terms.size());
}

// Known-answer helpers for tests.
void oracle_action_table(float* out_table, uint8_t* out_masks /* 4 x 90: ground, air, jump, boost */) {
    const ActionTable& t = actions();
    std::memcpy(out_table, t.a, sizeof t.a);
    std::memcpy(out_masks, t.ground, RLGPU_ACTIONS);
    std::memcpy(out_masks + RLGPU_ACTIONS, t.air, RLGPU_ACTIONS);
    std::memcpy(out_masks + 2 * RLGPU_ACTIONS, t.jump, RLGPU_ACTIONS);
    std::memcpy(out_masks + 3 * RLGPU_ACTIONS, t.boost, RLGPU_ACTIONS);
}

void oracle_pad_map(int* out) { std::memcpy(out, padmap().map, sizeof(int) * RLGPU_PADS); }

uint32_t oracle_philox(uint64_t key, uint32_t c0, uint32_t c1) {
    uint32_t o[4];
    philox(key, c0, c1, o);
    return o[0];
}

}  // extern "C"
