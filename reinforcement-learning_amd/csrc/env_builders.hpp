// env_builders.hpp -- the RLGymCPP layer of the env kernel: GameState snapshot, terminal
// conditions, the ExampleMain reward list, AdvancedObs and DefaultAction masks, kickoff reset.
#pragma once
#include "env_contacts.hpp"

namespace rl {

struct PView {
    v3 pos, vel, ang, fwd, right, up;
    float boost;
    bool on_ground, hfj, demoed, has_jumped, is_flipping, orange, world_contact;
    float wc_z;
};

DEV PView view_player(ArenaLDS* A, int i) {
    const rlgpu_car& c = A->s.cars[i];
    PView p;
    p.pos = ld3(c.body.pos) * kBT2UU;
    p.vel = ld3(c.body.vel) * kBT2UU;
    p.ang = ld3(c.body.angvel);
    const float* r = c.body.rot;
    p.fwd = v3{r[0], r[3], r[6]};
    p.right = v3{r[1], r[4], r[7]};
    p.up = v3{r[2], r[5], r[8]};
    p.boost = c.boost;
    p.on_ground = c.is_on_ground;
    p.hfj = c.is_on_ground || (!c.has_flipped && !c.has_double_jumped && c.air_time_since_jump < 1.25f);  // Car.cpp:279-283
    p.demoed = c.is_demoed;
    p.has_jumped = c.has_jumped;
    p.is_flipping = c.is_flipping;
    p.orange = i & 1;
    p.world_contact = c.world_contact;
    p.wc_z = c.world_contact_normal[2];
    return p;
}

DEV v3 inv_if(v3 v, bool inv) { return inv ? v3{-v.x, -v.y, v.z} : v; }

// AdvancedObs::AddPlayerToObsFast (AdvancedObs.cpp:108-172)
DEV void add_player_obs(float* o, const PView& pl, bool inv, v3 bp, v3 bv) {
    const float POS = 1.0f / 2300.0f, VEL = 1.0f / 2300.0f, ANG = 1.0f / 5.5f, BOOST = 0.01f;
    v3 pos = inv_if(pl.pos, inv), vel = inv_if(pl.vel, inv), ang = inv_if(pl.ang, inv);
    v3 f = inv_if(pl.fwd, inv), r = inv_if(pl.right, inv), u = inv_if(pl.up, inv);
    o[0] = pos.x * POS; o[1] = pos.y * POS; o[2] = pos.z * POS;
    o[3] = f.x; o[4] = f.y; o[5] = f.z;
    o[6] = u.x; o[7] = u.y; o[8] = u.z;
    o[9] = vel.x * VEL; o[10] = vel.y * VEL; o[11] = vel.z * VEL;
    o[12] = ang.x * ANG; o[13] = ang.y * ANG; o[14] = ang.z * ANG;
    o[15] = (f.x * ang.x + f.y * ang.y + f.z * ang.z) * ANG;
    o[16] = (r.x * ang.x + r.y * ang.y + r.z * ang.z) * ANG;
    o[17] = (u.x * ang.x + u.y * ang.y + u.z * ang.z) * ANG;
    float rx = bp.x - pos.x, ry = bp.y - pos.y, rz = bp.z - pos.z;
    o[18] = (f.x * rx + f.y * ry + f.z * rz) * POS;
    o[19] = (r.x * rx + r.y * ry + r.z * rz) * POS;
    o[20] = (u.x * rx + u.y * ry + u.z * rz) * POS;
    float vx = bv.x - vel.x, vy = bv.y - vel.y, vz = bv.z - vel.z;
    o[21] = (f.x * vx + f.y * vy + f.z * vz) * VEL;
    o[22] = (r.x * vx + r.y * vy + r.z * vz) * VEL;
    o[23] = (u.x * vx + u.y * vy + u.z * vz) * VEL;
    o[24] = pl.boost * BOOST;
    o[25] = pl.on_ground ? 1.0f : 0.0f;
    o[26] = pl.hfj ? 1.0f : 0.0f;
    o[27] = pl.demoed ? 1.0f : 0.0f;
    o[28] = pl.has_jumped ? 1.0f : 0.0f;
}

// AdvancedObs::BuildObs + DefaultAction::GetActionMask of the arena's 4 players into LDS rows, on its 16 lanes with
// one code path (AdvancedObs.cpp, DefaultAction masks): the 29-float player blocks of every row on lanes 4 j + pi
// (j: self, teammate, first opponent, second opponent), then the ball / previous-action, boost-pad and mask
// elements dealt over the lanes.  Every element is the same expression as in a per-player build; only the lane
// that writes it differs.
DEV void build_obs_rows(ArenaLDS* A, int l) {
    {
        const int pi = l & 3, j = l >> 2;
        const bool inv = pi & 1;  // the player's team (orange = index & 1)
        const v3 bp = inv_if(ld3(A->s.ball.pos) * kBT2UU, inv), bv = inv_if(ld3(A->s.ball.vel) * kBT2UU, inv);
        const int opp = (pi & 1) ^ 1;  // the first opponent: the other team's lower index
        const int who = j == 0 ? pi : (j == 1 ? pi ^ 2 : (j == 2 ? opp : opp + 2));
        add_player_obs(A->u.out.obs[pi] + 51 + 29 * j, view_player(A, who), inv, bp, bv);
    }
    // ball (AdvancedObs.h:10-13 scales) and previous action: 4 x 17 elements
    for (int e = l; e < 4 * 17; e += kTeam) {
        const int p = e / 17, k = e - 17 * (e / 17);
        float* o = A->u.out.obs[p];
        if (k < 9) {
            const int w = k / 3, c = k - 3 * (k / 3);  // w: position, velocity, angular velocity
            const float* src = w == 0 ? A->s.ball.pos : (w == 1 ? A->s.ball.vel : A->s.ball.angvel);
            float x = w < 2 ? src[c] * kBT2UU : src[c];
            if ((p & 1) && c < 2) x = -x;  // inv_if
            const float sc = w == 0 ? 1 / 5000.f : (w == 1 ? 1 / 2300.f : 1 / 3.f);
            o[k] = x * sc;
        } else {
            o[k] = A->s.env.prev_action[p][k - 9];
        }
    }
    // boost pads: 4 x 34 elements
    for (int e = l; e < 4 * RLGPU_PADS; e += kTeam) {
        const int p = e / RLGPU_PADS, k = e - RLGPU_PADS * (e / RLGPU_PADS);
        const bool inv = p & 1;
        const int fwd = C.pad_map[k], rev = C.pad_map[RLGPU_PADS - k - 1];
        const int act_idx = inv ? rev : fwd;
        const int tim_idx = inv ? fwd : rev;  // GameState.h:60 quirk
        const bool active = A->s.pads[act_idx].is_active;
        const float timer = A->s.pads[tim_idx].cooldown;
        A->u.out.obs[p][17 + k] = active ? 1.0f : 1.0f / (1.0f + timer);
    }
    // action masks: 4 x 90 bytes; the players' flags packed 3 bits each (no run-time register index)
    uint32_t fl = 0;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const rlgpu_car& c = A->s.cars[p];
        const bool hfj = c.is_on_ground || (!c.has_flipped && !c.has_double_jumped && c.air_time_since_jump < 1.25f);
        const bool turtled = c.world_contact && c.world_contact_normal[2] > 0.9f;
        fl |= (uint32_t)((c.is_on_ground ? 1 : 0) | (c.boost == 0 ? 2 : 0) | ((hfj || turtled) ? 4 : 0)) << (3 * p);
    }
    for (int e = l; e < 4 * RLGPU_ACTIONS; e += kTeam) {
        const int p = e / RLGPU_ACTIONS, k = e - RLGPU_ACTIONS * (e / RLGPU_ACTIONS);
        const uint32_t f = fl >> (3 * p), bits = C.mask_bits[k];
        uint32_t r = (f & 1) ? (bits & 1) : ((bits >> 1) & 1);  // ground / air table
        if (f & 2) r &= ~(bits >> 3);                           // no boost: the boost actions off
        if (f & 4) r |= (bits >> 2) & 1;                         // can jump (or turtled): the jump actions on
        A->u.out.masks[p][k] = (uint8_t)(r & 1);
    }
}

// KickoffProximityReward2v2Enhanced (KickoffProximityReward2v2Enhanced.h:14-366).  goer = goerReward (:9, used at
// :135), rpw = rotationPrepWeight (:12, used at :175); cheaterReward / dynamicWeight are never read by GetReward.
DEV float kickoff_reward(ArenaLDS* A, int pi, const PView& pl, v3 bpos, v3 bvel, float goer, float rpw) {
    float bspeed = rs_len(bvel);
    v3 b2 = v3{bpos.x, bpos.y, 0.f};
    if (!(bspeed < 2.f && bpos.z < 150.f && rs_len(b2) < 50.f)) return 0.f;
    bool has_tm = false;
    int tm_i = -1;
    float tm_dist = 0, closest = 3.402823466e+38f, second = 3.402823466e+38f;
    v3 opp_com = zero3();
    int nopp = 0;
    float tot_speed = 0;
    for (int j = 0; j < 4; j++) {
        const PView p = view_player(A, j);
        if (p.orange == pl.orange && j != pi) {
            tm_i = j;
            has_tm = true;
            tm_dist = rs_len(p.pos - bpos);
        } else if (p.orange != pl.orange) {
            float d = rs_len(p.pos - bpos);
            tot_speed += rs_len(p.vel);
            nopp++;
            if (d < closest) {
                second = closest;
                closest = d;
            } else if (d < second) {
                second = d;
            }
            opp_com = opp_com + p.pos;
        }
    }
    if (nopp > 0) opp_com = rs_div(opp_com, (float)nopp);
    if (!has_tm) return 0.f;
    const PView tm = view_player(A, tm_i);
    float pdist = rs_len(pl.pos - bpos);
    float dscore = (pdist < tm_dist) ? 0.4f : 0.f;
    v3 p2b = rs_norm(bpos - pl.pos), t2b = rs_norm(bpos - tm.pos);
    float pvb = dot(pl.vel, p2b), tvb = dot(tm.vel, t2b);
    float sscore = (pvb > tvb) ? 0.3f : 0.f;
    float bscore = (pl.boost > tm.boost + 10.f) ? 0.2f : 0.f;
    float pa = rs_atan2f(pl.pos.y - bpos.y, pl.pos.x - bpos.x);
    float ta = rs_atan2f(tm.pos.y - bpos.y, tm.pos.x - bpos.x);
    float adiff = fabsf(pa - ta);
    float spawn = (adiff > (3.14159f / 3.f)) ? 1.f : 0.f;
    float total = dscore + sscore + bscore + spawn * 0.1f;
    if (total >= 0.5f) {
        float base = (pdist < closest) ? goer : -goer * 0.5f;
        v3 to_b = rs_norm(bpos - pl.pos);
        float pvel = dot(pl.vel, to_b);
        float speed_bonus = clampf(pvel / 2300.f, -0.3f, 0.3f);
        float eff = 0.f;
        if (pl.boost > 50.f && pdist > 1000.f) eff = 0.1f;
        else if (pl.boost < 20.f && pdist > 800.f) eff = -0.15f;
        v3 vn = rs_norm(pl.vel);
        float approach = dot(to_b, vn);
        float angle_bonus = stdmax(0.f, approach) * 0.2f;
        return clampf(base + speed_bonus + eff + angle_bonus, -1.5f, 1.5f);
    }
    v3 own = !pl.orange ? v3{0, -6000, 642.775f / 2} : v3{0, 6000, 642.775f / 2};
    v3 center = v3{0.f, 0.f, 100.f};
    v3 cm = v3{center.x * 1.3f, center.y * 1.3f, center.z * 1.3f};
    v3 base_ideal = (own + cm) * 0.5f;
    v3 threat = rs_norm(opp_com - own);
    threat = v3{threat.x * 200.f, threat.y * 200.f, threat.z * 200.f};
    v3 tm_off = zero3();
    {
        float tdc = rs_len(tm.pos - center);
        if (tdc > 1500.f) {
            v3 dir = rs_norm(tm.pos - base_ideal);
            tm_off = v3{dir.x * 300.f, dir.y * 300.f, dir.z * 300.f};
        }
    }
    v3 thr_adj = v3{threat.x * 0.3f, threat.y * 0.3f, threat.z * 0.3f};
    v3 tm_adj = v3{tm_off.x * 0.2f, tm_off.y * 0.2f, tm_off.z * 0.2f};
    v3 ideal = base_ideal + thr_adj + tm_adj;
    ideal.x = clampf(ideal.x, -3000.f, 3000.f);
    ideal.y = clampf(ideal.y, -4000.f, 4000.f);
    ideal.z = stdmax(ideal.z, 17.f);
    float dti = rs_len(pl.pos - ideal);
    float posr;
    if (dti <= 600.f) posr = 0.5f * (1.f - (dti / 600.f));
    else if (dti <= 1200.f) posr = 0.5f * (1.f - (dti - 600.f) / (1200.f - 600.f)) * 0.7f;
    else if (dti <= 2000.f) posr = -0.1f * ((dti - 1200.f) / (2000.f - 1200.f));
    else posr = -0.3f;
    float best = 0.f;
    for (int i = 0; i < RLGPU_PADS; i++) {
        v3 bl = C.boost_loc[i];
        if (bl.z > 72.0f) {
            float dtb = rs_len(pl.pos - bl);
            float acc = 1.f - clampf(dtb / 1500.f, 0.f, 1.f);
            float d2b = rs_len(bl - bpos);
            bool corner = (fabsf(bl.x) > 2500.f && fabsf(bl.y) > 3500.f);
            float bvv = corner ? 0.8f : 0.6f;
            float prox = 1.f - clampf(d2b / 3000.f, 0.f, 1.f);
            float strat = bvv * (0.3f + prox * 0.7f);
            float od = rs_len(opp_com - bl);
            float deny = clampf(1.f - (od / 2000.f), 0.f, 0.3f);
            float tv = acc * (strat + deny);
            best = stdmax(best, tv);
        }
    }
    float blf = 1.f;
    if (pl.boost < 30.f) blf = 1.5f;
    else if (pl.boost > 80.f) blf = 0.5f;
    float boostr = best * blf * 0.25f;
    float rot;
    {
        v3 t2g = rs_norm(own - tm.pos);
        v3 perp = rs_norm(v3{-t2g.y, t2g.x, 0.f});
        v3 goff = v3{t2g.x * 800.f, t2g.y * 800.f, t2g.z * 800.f};
        v3 poff = v3{perp.x * 600.f, perp.y * 600.f, perp.z * 600.f};
        v3 sup = tm.pos + goff + poff;
        float dts = rs_len(pl.pos - sup);
        float ready = 1.f - clampf(dts / 1000.f, 0.f, 1.f);
        v3 tos = rs_norm(sup - pl.pos);
        float align = stdmax(0.f, dot(rs_norm(pl.vel), tos));
        rot = (ready * 0.7f + align * 0.3f) * rpw;
    }
    float aware;
    {
        v3 toc = rs_norm(opp_com - pl.pos);
        v3 tob = rs_norm(bpos - pl.pos);
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

// a^b for SaveBoostReward's powf (CommonRewards.h:136-145): b = 0.5 as sqrtf (correctly rounded on
// both sides, the ExampleMain case), otherwise exp(b log a) on the shared deterministic kernels
DEV float reward_powf(float a, float b) {
    if (b == 0.5f) return sqrtf(a);
    if (b == 0.f) return 1.f;
    if (a == 0.f) return b > 0.f ? 0.f : __int_as_float(0x7f800000);
    return rs_expf(b * rs_logf(a));
}

// one weighted reward of the registry for player i (CommonRewards.h:8-203,
// KickoffProximityReward2v2Enhanced.h, src/ExampleMain.cpp:84-124); CommonValues CAR_MAX_SPEED 2300,
// BALL_MAX_SPEED 6000, goal backs (0, +-6000, 642.775 / 2) (CommonValues.h)
DEV float reward_value(ArenaLDS* A, const rlgpu_reward_spec& rs, int i, const PView& pl, v3 bpos, v3 bvel, v3 prev_bvel,
                       bool goal) {
    const rlgpu_env_extra& e = A->s.env;
    const float KPH = 250.f / 9.f;  // Math::KPHToVel (RG/Math.h:12-14)
    bool touched = A->a.touched[i] != 0;
    switch (rs.type) {
        case RLGPU_RW_AIR: return !pl.on_ground;
        case RLGPU_RW_WAVEDASH: return (pl.on_ground && (e.prev_is_flipping[i] && !e.prev_on_ground[i])) ? 1.f : 0.f;
        case RLGPU_RW_KICKOFF_PROXIMITY_2V2:  // params[2] != 0: params[0..1] hold the tunables, else the defaults
            return kickoff_reward(A, i, pl, bpos, bvel, rs.params[2] != 0.f ? rs.params[0] : 1.2f,
                                  rs.params[2] != 0.f ? rs.params[1] : 0.2f);
        case RLGPU_RW_VELOCITY_PLAYER_TO_BALL: {
            v3 dir = rs_norm(bpos - pl.pos);
            v3 nv = rs_div(pl.vel, 2300.f);
            return dot(dir, nv);
        }
        case RLGPU_RW_STRONG_TOUCH: {
            float minv = rs.params[0] * KPH, maxv = rs.params[1] * KPH;
            if (!touched) return 0.f;
            float hit = rs_len(bvel - prev_bvel);
            return hit < minv ? 0.f : stdmin(1.f, hit / maxv);
        }
        case RLGPU_RW_TOUCH_ACCEL: {
            const float MAXS = 110 * KPH;
            if (!touched) return 0.f;
            float pf = stdmin(1.f, rs_len(prev_bvel) / MAXS);
            float cf = stdmin(1.f, rs_len(bvel) / MAXS);
            return cf > pf ? (cf - pf) : 0.f;
        }
        case RLGPU_RW_VELOCITY_BALL_TO_GOAL: {
            bool target_orange = !pl.orange;
            if (rs.params[0] != 0.f) target_orange = !target_orange;  // ownGoal
            v3 tgt = target_orange ? v3{0, 6000, 642.775f / 2} : v3{0, -6000, 642.775f / 2};
            v3 d = rs_norm(tgt - bpos);
            return dot(d, rs_div(bvel, 6000.f));
        }
        case RLGPU_RW_PICKUP_BOOST:
            return pl.boost > e.prev_boost[i] ? sqrtf(pl.boost / 100.f) - sqrtf(e.prev_boost[i] / 100.f) : 0.f;
        case RLGPU_RW_SAVE_BOOST: {
            float x = reward_powf(pl.boost / 100, rs.params[0]);
            return stdmin(stdmax(x, 0.f), 1.f);  // RS_CLAMP
        }
        case RLGPU_RW_BUMP: return e.ev_bump[i];
        case RLGPU_RW_DEMO: return e.ev_demo[i];
        case RLGPU_RW_BUMPED_PENALTY: return -(float)e.ev_bumped[i];
        case RLGPU_RW_DEMOED_PENALTY: return -(float)e.ev_demoed[i];
        case RLGPU_RW_GOAL: {
            if (!goal) return 0.f;
            bool team_from_y_orange = !(bpos.y < 0);  // RS_TEAM_FROM_Y
            return (pl.orange != team_from_y_orange) ? 1.f : rs.params[0];  // concedeScale
        }
        case RLGPU_RW_LOSING_PENALTY: {
            int own = pl.orange ? e.penalty_orange : e.penalty_blue;
            int opp = pl.orange ? e.penalty_blue : e.penalty_orange;
            int deficit = opp - own;
            return deficit > 0 ? -rs.params[0] * (float)deficit : 0.f;
        }
        case RLGPU_RW_VELOCITY: return rs_len(pl.vel) / 2300.f * (float)(1 - 2 * (rs.params[0] != 0.f));
        case RLGPU_RW_FACE_BALL: return dot(pl.fwd, rs_norm(bpos - pl.pos));
        case RLGPU_RW_TOUCH_BALL: return touched ? 1.f : 0.f;
        case RLGPU_RW_SPEED: return rs_len(pl.vel) / 2300.f;
    }
    return 0.f;
}

// Arena::ResetToRandomKickoff (Arena.cpp:112-216) + EnvSet::ResetArena state (EnvSet.cpp:275-304), one lane
DEV void kickoff_reset(ArenaLDS* A, uint64_t seed, int arena, bool fuzz) {
    int order[5] = {0, 1, 2, 3, 4};
    for (int i = 4; i > 0; i--) {
        int j = (int)(rng_next(A, seed, arena) % (uint32_t)(i + 1));
        int t = order[i];
        order[i] = order[j];
        order[j] = t;
    }
    for (int i = 0; i < 2; i++) {
        int k = order[i];
        for (int team = 0; team < 2; team++) {
            int ci = 2 * i + team;
            v3 pos = v3{C.kick_x[k], C.kick_y[k], 17.f};
            if (team == 1) pos = pos * v3{-1, -1, 1};
            set_car_state(A, ci, pos, C.kick_rot[team][k], 100.f / 3.f, true);
        }
    }
    if (fuzz) {  // FuzzedKickoffState::ResetArena: GetState, pos += RandFloat(-0.1, 0.1) uu, SetState
        for (int ci = 0; ci < 4; ci++) {
            rlgpu_body& b = A->s.cars[ci].body;
            for (int k = 0; k < 3; k++) {
                const float r = -0.1f + rng_uniform(A, seed, arena) * (0.1f - -0.1f);
                b.pos[k] = (b.pos[k] * kBT2UU + r) * kUU2BT;
                b.vel[k] = (b.vel[k] * kBT2UU) * kUU2BT;
            }
        }
    }
    st3(A->s.ball.pos, v3{0, 0, 93.15f} * kUU2BT);
    stm(A->s.ball.rot, ident3());
    st3(A->s.ball.vel, zero3());
    st3(A->s.ball.angvel, zero3());
    st3(A->s.ball_vel_impulse_cache, zero3());
    for (int p = 0; p < RLGPU_PADS; p++) {
        A->s.pads[p].is_active = 1;
        A->s.pads[p].cooldown = 0;
        A->s.pads[p].prev_locked_car_id = 0;
    }
    rlgpu_env_extra& e = A->s.env;
    e.last_tick_count = e.tick_count;
    e.no_touch_time = 0;
    e.score_blue = e.score_orange = 0;
    e.penalty_blue = e.penalty_orange = 0;
    e.has_prev = 0;
    e.terminal = 0;
    e.episode_steps = 0;
    for (int p = 0; p < 4; p++) {
        for (int k = 0; k < 8; k++) e.prev_action[p][k] = 0.f;
        e.ev_bump[p] = e.ev_bumped[p] = e.ev_demo[p] = e.ev_demoed[p] = 0;
    }
}

}  // namespace rl
