// env_step.hpp -- the env kernel (one launch = every arena of the set: StepFirstHalf / StepSecondHalf /
// resets / builders, env_kernel.hpp) and its launch arguments.
//
// Every translation unit that defines RLGPU_ENV_KERNEL (the kernel's name) and RLGPU_ENV_ARITH (an
// RLGPU_ARITH_* mode, include/rlgpu_arith.h) gets the kernel specialised for that arithmetic: arith(A) is
// then a constant (env_device.hpp), so the other builds' LinearMath and solver-row branches fold away and
// do not hold registers (env_k0.hip, env_k1.hip, env_k2.hip).  Without RLGPU_ENV_KERNEL only StepArgs is
// declared (env.hip's host code).
#pragma once
#include "env_builders.hpp"

namespace rl {

struct StepArgs {
    char* arenas;
    int n;
    int ticks_first;        // StepFirstHalf ticks (actionDelay), 0 = skip
    const int32_t* actions; // StepSecondHalf actions (null = skip second half)
    int ticks_second;       // tickSkip - actionDelay
    int build;              // run GameState / terminal / reward / obs builders
    int reset_mode;         // 0 none, 1 reset terminated (fused), 2 EnvSet::Reset, 3 mask, 4 all, 5 obs only
    const uint8_t* reset_mask;
    float* obs;
    uint8_t* masks;
    float* rewards;
    uint8_t* terminals;
    float* last_rewards;
    float* trunc_obs;
    float* out_obs;        // experience append (rlgpu_step_outputs), each may be null
    uint8_t* out_masks;
    float* out_rew;
    int8_t* out_term;
    float* out_trunc;
    int max_episode_steps;
    uint64_t seed;
    unsigned long long* prof;  // [32] phase cycle counters or null
    MeshView mesh;
    double* metrics;           // [n][RLGPU_STEP_METRIC_SLOTS] StepCallback sums (build steps) or null
    int metrics_players;       // this call is one of ExampleMain's every-4th "expensive" calls
    const Plugins* plug;       // the set's reward / terminal registry (device)
    int arith;                 // RLGPU_ARITH_* (rlgpu_envset_config.arith): copied into Aux::arith at launch
    int arena_offset;          // global index of arena 0 (the arenas' Philox streams)
    float* reward_values;      // [players][nr] each reward's value before its weight, or null
    int fuzz;                  // FuzzedKickoffState (rlgpu_envset_config.state_setter)
    int pen_slots;             // deferred penetration queries whose GJK state is saved (kPenSave; tests: fewer)
};

#ifdef RLGPU_ENV_KERNEL

// ExampleMain's StepCallback (src/ExampleMain.cpp:233-283) on this arena's GameState as the
// builders left it (after UpdateFromArena, before any reset), Report::AddAvg's fp64 totals kept per
// arena and player: slot RLGPU_SM_* x 4 + player.  Lane l = player l; lane 0 adds the per-state
// goal speed and the arena's count of player passes.  Vec::Length / Normalized / Dot / RS_MAX are
// restated in float (MathTypes.h:31-93, Framework.h:47); the totals are fp64 as Report::Avg.
DEV void step_metrics(ArenaLDS* A, int l, double* m, bool players) {
    if (players) {
        const rlgpu_car& c = A->s.cars[l];
        const v3 pos = ld3(c.body.pos) * kBT2UU, vel = ld3(c.body.vel) * kBT2UU;
        const v3 bp = ld3(A->s.ball.pos) * kBT2UU;
        const bool touched = A->a.touched[l] != 0;
        const v3 dir = rs_norm(bp - pos);
        const float toward = vel.x * dir.x + vel.y * dir.y + vel.z * dir.z;
        m[RLGPU_SM_IN_AIR * 4 + l] += c.is_on_ground ? 0.0 : 1.0;
        m[RLGPU_SM_BALL_TOUCH * 4 + l] += touched ? 1.0 : 0.0;
        m[RLGPU_SM_DEMOED * 4 + l] += c.is_demoed ? 1.0 : 0.0;
        m[RLGPU_SM_SPEED * 4 + l] += (double)rs_len(vel);
        m[RLGPU_SM_SPEED_TO_BALL * 4 + l] += (double)(0.f > toward ? 0.f : toward);
        m[RLGPU_SM_BOOST * 4 + l] += (double)c.boost;
        if (touched) m[RLGPU_SM_TOUCH_HEIGHT * 4 + l] += (double)bp.z;
    }
    if (l == 0) {
        if (players) m[RLGPU_SM_SLOT_PASSES] += 1.0;
        if (A->a.goal) {
            m[RLGPU_SM_SLOT_GOAL_SPEED] += (double)rs_len(ld3(A->s.ball.vel) * kBT2UU);
            m[RLGPU_SM_SLOT_GOALS] += 1.0;
        }
    }
}


// The boost-pad constants a lane tests every tick (pads l, l + 16, l + 32), held in registers for
// the whole launch instead of re-read from the constant buffer with lane-varying addresses in every
// tick's pad-collision phase.
constexpr int kPadsPerLane = (RLGPU_PADS + kTeam - 1) / kTeam;
struct PadRegs {
    int px[kPadsPerLane], py[kPadsPerLane];
    v3 pos[kPadsPerLane], bmin[kPadsPerLane], bmax[kPadsPerLane];
    float rad[kPadsPerLane];
};
DEV void load_pad_regs(PadRegs& R, int l) {
#pragma unroll
    for (int k = 0; k < kPadsPerLane; k++) {
        const int p = l + k * kTeam < RLGPU_PADS ? l + k * kTeam : 0;
        R.px[k] = C.pad_cell_x[p];
        R.py[k] = C.pad_cell_y[p];
        R.pos[k] = C.pad_pos_bt[p];
        R.bmin[k] = C.pad_box_min[p];
        R.bmax[k] = C.pad_box_max[p];
        R.rad[k] = (C.pad_big[p] ? 208.f : 144.f) * kUU2BT;
    }
}

// ------------------------------------------------------------------ one tick (Arena::Step body)
// Inlined into the tick loop.  Inlined, the compiler hoists the launch-invariant
// constant-buffer values of all phases out of the loop (408 VGPR + AGPR, one wave per SIMD);
// called (__noinline__) the kernel needs 248 VGPRs and could run two waves per SIMD, but measured
// slower: 870 -> 938 us per launch at 4 arenas per wave, and 2 arenas per wave (two waves per
// SIMD) 1.7x slower per arena.
DEV void tick(ArenaLDS* A, const MeshView& M, int l, bool valid, uint64_t seed, int arena, Prof& P, const PadRegs& R,
                          int nvalid) {
    if (valid) {  // per body / car on lanes 0-4: independent fields, read before the respawns below write
        rlgpu_arena_state& s = A->s;
        if (l == 0) {
            A->u.wc.njob = 0;  // this tick's wheel-ray cast jobs
            bool sleep = len2(ld3(s.ball.vel)) == 0 && len2(ld3(s.ball.angvel)) == 0;  // Arena.cpp:722-727
            s.ball_sleeping = sleep;
            A->a.ball_sleep = sleep;
            A->a.active[0] = 1;
        } else if (l < 5) {
            const int c = l - 1;
            A->a.active[c + 1] = !s.cars[c].is_demoed;
            float* ctl = s.cars[c].controls;  // CarControls::ClampFix
            for (int k = 0; k < 5; k++) ctl[k] = stdclamp(ctl[k], -1.f, 1.f);
        }
        if (l < 5) {
            A->a.snap_vel[l] = bvel(A, l);
            A->a.snap_ang[l] = bang(A, l);
        }
    }
    sync();
    if (valid && l == 0) {
        rlgpu_arena_state& s = A->s;
        // demo timer / respawn (Car.cpp:66-84), RNG draws in car order
        for (int c = 0; c < 4; c++) {
            rlgpu_car& cs = s.cars[c];
            if (cs.is_demoed) {
                cs.demo_respawn_timer = stdmax(cs.demo_respawn_timer - kTick, 0.f);
                if (cs.demo_respawn_timer == 0.f) {
                    int idx = (int)(rng_next(A, seed, arena) % 4u);
                    bool orange = c & 1;
                    v3 pos = v3{C.respawn_x[idx], C.respawn_y[idx] * (orange ? -1.f : 1.f), 36.f};
                    set_car_state(A, c, pos, C.respawn_rot[orange][idx], 100.f / 3.f, false);
                }
            }
        }
    }
    sync();
    P.mark(0);
    if (valid && !A->s.cars[l >> 2].is_demoed) wheel_phase(A, M, l >> 2, l & 3);
    sync();
    P.mark(1);
    wheel_casts(A - (threadIdx.x >> 4), nvalid);
    sync();
    P.mark(30);
    if (valid && !A->s.cars[l >> 2].is_demoed) wheel_phase_b(A, l >> 2, l & 3);
    sync();
    P.mark(31);
    if (valid && l < 4) car_phase_a(A, l);
    sync();
    P.mark(33);
    // Car::_UpdateWheels' per-wheel friction: lane 4 car + wheel
    if (valid && !A->s.cars[l >> 2].is_demoed) wheel_friction(A, l >> 2, l & 3);
    sync();
    P.mark(34);
    if (valid) {
        if (l < 4) {
            car_phase(A, l);
        } else {
            for (int p = l - 4; p < RLGPU_PADS; p += 12) {  // BoostPad::_PreTickUpdate
                rlgpu_pad& pd = A->s.pads[p];
                if (pd.cooldown > 0) pd.cooldown = stdmax(pd.cooldown - kTick, 0.f);
                pd.is_active = pd.cooldown == 0;
            }
        }
    }
    sync();
    P.mark(2);
    if (valid && l < 5) {  // applyGravity + predictUnconstraintMotion
        add_force(A, l, C.gravity * (l == 0 ? kBallMass : kCarMass));
        if (l == 0) {
            rlgpu_body* b = body(A, 0);
            st3(b->vel, ld3(b->vel) * C.ball_damp);
            st3(b->angvel, ld3(b->angvel) * 1.f);
            A->a.pred_pos[0] = bpos(A, 0) + bvel(A, 0) * kTick;
            A->a.pred_rot[0] = brot(A, 0);
        } else {
            integrate_transform(bpos(A, l), brot(A, l), bvel(A, l), bang(A, l), kTick, A->a.pred_pos[l], A->a.pred_rot[l],
                                arith(A));
        }
    }
    sync();
    P.mark(3);
    if (valid && l < 5) {  // updateAabbs: the broadphase AABB and home cell of body l (one lane per body)
        v3 mn, mx;
        broad_aabb(A, l, mn, mx);
        A->u.bp.mn[l] = mn;
        A->u.bp.mx[l] = mx;
        A->u.bp.cell[l] = bp_home(mn) + 1;
    }
    sync();
    if (valid && l == 0) {
        bp_update(A);  // btRSBroadphase::setAabb in body order
        bool awake = !A->a.ball_sleep;
        if (!awake) {
            const v3 m0 = A->u.bp.mn[0], m1 = A->u.bp.mx[0];
            for (int ci = 1; ci <= 4; ci++) {
                if (!A->a.active[ci]) continue;
                if (aabb_overlap(m0, m1, A->u.bp.mn[ci], A->u.bp.mx[ci])) awake = true;
            }
        }
        A->a.ball_awake = awake;
        A->a.ncand = 0;
        A->a.nq = 0;
    }
    if (threadIdx.x == 0) g_pen_save.n = 0;
    sync();
    P.mark(4);
    if (valid)
        // work items: the 5 body-vs-mesh pairs split into kMeshChunks parts each (the heavy items,
        // spread over distinct lanes first), then the 30 light pairs
        for (int item = l; item < 5 * kMeshChunks + 30; item += kTeam) {
            if (item < 5 * kMeshChunks) {
                narrow_pair(A, M, (item / kMeshChunks) * 5, item % kMeshChunks, kMeshChunks);
            } else {
                int j = item - 5 * kMeshChunks;  // 0..29 -> the plane and dynamic ranks
                narrow_pair(A, M, j < 20 ? (j / 4) * 5 + 1 + (j % 4) : 25 + (j - 20));
            }
        }
    sync();
    P.mark(22);
    narrow_queue(A - (threadIdx.x >> 4), nvalid, M);
    sync();
    P.mark(5);
    narrow_deferred(A - (threadIdx.x >> 4), nvalid, M);
    sync();
    P.mark(18);
    if (valid) sort_candidates(A, l);
    sync();
    if (valid && l == 0) {
        commit_contacts(A, M, &P);
        if (threadIdx.x == 0) P.mark(16);
    }
    sync();
    solve_lanes(A, l, valid, &P);
    sync();
    P.mark(6);
    if (valid && l < 5) {  // integrateTransforms (btDiscreteDynamicsWorld.cpp:889-985)
        bool act = l == 0 ? A->a.ball_awake != 0 : A->a.active[l] != 0;
        if (act) {
            rlgpu_body* b = body(A, l);
            if (l == 0) {
                st3(b->pos, ld3(b->pos) + ld3(b->vel) * kTick);
            } else {
                v3 np;
                m3 nr;
                integrate_transform(ld3(b->pos), ldm(b->rot), ld3(b->vel), ld3(b->angvel), kTick, np, nr, arith(A));
                st3(b->pos, np);
                stm(b->rot, nr);
            }
            update_inertia(A, l);
        }
        A->a.force[l] = zero3();
        A->a.torque[l] = zero3();
    }
    sync();
    P.mark(7);
    if (valid && l < 4) {  // Car::_PostTickUpdate + _FinishPhysicsTick (Car.cpp:133-193)
        rlgpu_car& cs = A->s.cars[l];
        if (!cs.is_demoed) {
            rlgpu_body* b = &cs.body;
            float sp2 = len2(ld3(b->vel) * kBT2UU);
            if (cs.is_supersonic && cs.supersonic_time < 1.f)
                cs.is_supersonic = sp2 >= 2100.f * 2100.f;
            else
                cs.is_supersonic = sp2 >= 2200.f * 2200.f;
            if (cs.is_supersonic)
                cs.supersonic_time += kTick;
            else
                cs.supersonic_time = 0;
            if (cs.car_contact_cooldown > 0) cs.car_contact_cooldown = stdmax(cs.car_contact_cooldown - kTick, 0.f);
            for (int k = 0; k < 8; k++) cs.last_controls[k] = cs.controls[k];
            v3 cache = ld3(cs.vel_impulse_cache);
            v3 v = ld3(b->vel), w = ld3(b->angvel);
            if (!is_zero(cache)) {
                v += cache;
                st3(cs.vel_impulse_cache, zero3());
            }
            const float maxv = 2300.f * kUU2BT;
            if (len2(v) > maxv * maxv) v = bt_normalize(v, arith(A)) * maxv;  // vel.normalized() (Car.cpp:183-186)
            if (len2(w) > 5.5f * 5.5f) w = bt_normalize(w, arith(A)) * 5.5f;
            st3(b->vel, v);
            st3(b->angvel, w);
        }
    }
    sync();
    P.mark(8);
    if (valid) {  // BoostPadGrid::CheckCollision per pad (BoostPadGrid.cpp:5-25, BoostPad.cpp:61-86)
        // per-car eligibility and 3x3 grid-cell window, computed once (not per pad)
        int cx0[4], cx1[4], cy0[4], cy1[4];
        v3 cp[4];
#pragma unroll
        for (int ci = 0; ci < 4; ci++) {
            const rlgpu_car& cs = A->s.cars[ci];
            v3 cpos = ld3(cs.body.pos);
            v3 pos_uu = cpos * kBT2UU;
            cp[ci] = cpos;
            bool ok = !(cs.is_demoed || cs.boost >= 100) && !(pos_uu.z > 95.f + 250.f);
            int ix = (int)(pos_uu.x / 1024 + 4), iy = (int)(pos_uu.y / 1024 + 5);
            cx0[ci] = ok ? (ix - 1 > 0 ? ix - 1 : 0) : 1 << 20;  // empty window when not eligible
            cx1[ci] = ix + 1 < 7 ? ix + 1 : 7;
            cy0[ci] = iy - 1 > 0 ? iy - 1 : 0;
            cy1[ci] = iy + 1 < 9 ? iy + 1 : 9;
        }
#pragma unroll
        for (int k = 0; k < kPadsPerLane; k++) {
            const int p = l + k * kTeam;
            if (p >= RLGPU_PADS) break;
            const int px = R.px[k], py = R.py[k];
            const v3 ppos = R.pos[k];
            const float rad = R.rad[k];
            const uint32_t prev_locked = A->s.pads[p].prev_locked_car_id;
            int locked = -1;
#pragma unroll
            for (int ci = 0; ci < 4; ci++) {
                if (px < cx0[ci] || px > cx1[ci] || py < cy0[ci] || py > cy1[ci]) continue;
                v3 cpos = cp[ci];
                bool col = false;
                if (prev_locked == (uint32_t)(ci + 1)) {
                    v3 mn, mx;
                    body_aabb(ci + 1, cpos, ldm(A->s.cars[ci].body.rot), mn, mx);
                    const v3 bmin = R.bmin[k], bmax = R.bmax[k];
                    col = (bmax.x > mn.x && bmax.y > mn.y && bmax.z > mn.z) && (bmin.x < mx.x && bmin.y < mx.y && bmin.z < mx.z);
                } else {
                    float dx = cpos.x - ppos.x, dy = cpos.y - ppos.y;
                    if (dx * dx + dy * dy < rad * rad) col = fabsf(cpos.z - ppos.z) < (95.f * kUU2BT);
                }
                if (col) locked = ci;
            }
            A->a.locked[p] = locked;
        }
    }
    sync();
    P.mark(9);
    // BoostPad::_PostTickUpdate (BoostPad.cpp:88-105): each pad's own state on the lane that tested it (pads
    // l, l + 16, l + 32), then the pickups' boost in pad order on the arena's lane 0 (a car may pick two pads)
    uint64_t picked[kPadsPerLane];
#pragma unroll
    for (int k = 0; k < kPadsPerLane; k++) {
        const int p = l + k * kTeam;
        bool pick = false;
        if (valid && p < RLGPU_PADS) {
            rlgpu_pad& pd = A->s.pads[p];
            const int lk = A->a.locked[p];
            if (lk >= 0 && pd.is_active) {
                pick = true;
                pd.is_active = 0;
                pd.cooldown = R.rad[k] > 144.f * kUU2BT ? 10.f : 4.f;  // a big pad (pad_big: radius 208)
            }
            pd.prev_locked_car_id = lk >= 0 ? (uint32_t)(lk + 1) : 0u;
        }
        picked[k] = __ballot(pick);
    }
    if (valid && l == 0) {
        const int team = (int)(threadIdx.x >> 4);
#pragma unroll
        for (int k = 0; k < kPadsPerLane; k++)
            for (uint32_t bits = (uint32_t)(picked[k] >> (16 * team)) & 0xffffu; bits; bits &= bits - 1u) {
                const int p = __ffs(bits) - 1 + k * kTeam;
                rlgpu_car& cs = A->s.cars[A->a.locked[p]];
                cs.boost = stdmin(cs.boost + (C.pad_big[p] ? 100.f : 12.f), 100.f);
            }
        rlgpu_body* b = &A->s.ball;  // Ball::_FinishPhysicsTick (Ball.cpp:112-138)
        v3 v = ld3(b->vel), w = ld3(b->angvel);
        v3 cache = ld3(A->s.ball_vel_impulse_cache);
        if (!is_zero(cache)) {
            v += cache;
            st3(A->s.ball_vel_impulse_cache, zero3());
        }
        const float maxv = 6000.f * kUU2BT;
        if (len2(v) > maxv * maxv) v = bt_normalize(v, arith(A)) * maxv;  // vel.normalized() (Ball.cpp:128-131)
        if (len2(w) > 6.f * 6.f) w = bt_normalize(w, arith(A)) * 6.f;
        st3(b->vel, v);
        st3(b->angvel, w);
        A->s.env.tick_count++;
    }
    sync();
    P.mark(10);
}

// copy the 4 obs rows (and mask rows) of this arena from LDS to [players x OBS] outputs
DEV void copy_rows(ArenaLDS* A, int l, int arena, float* obs, uint8_t* masks) {
    if (obs) {
        const float* src = &A->u.out.obs[0][0];
        float* dst = obs + (size_t)arena * 4 * RLGPU_OBS;
        for (int k = l; k < 4 * RLGPU_OBS; k += kTeam) dst[k] = src[k];
    }
    if (masks) {
        const uint8_t* msrc = &A->u.out.masks[0][0];
        uint8_t* mdst = masks + (size_t)arena * 4 * RLGPU_ACTIONS;
        for (int k = l; k < 4 * RLGPU_ACTIONS; k += kTeam) mdst[k] = msrc[k];
    }
}

__global__ void __launch_bounds__(kWG) RLGPU_ENV_KERNEL(StepArgs g) {
    __shared__ ArenaLDS lds[kArenas];
    const int team = threadIdx.x >> 4, l = threadIdx.x & 15;
    const int arena = blockIdx.x * kArenas + team;
    const bool valid = arena < g.n;
    ArenaLDS* A = &lds[team];
    Prof P{g.prof, g.prof ? (long long)clock64() : 0};
    // ---- stage the 4 arena records into LDS (contiguous 16-byte loads)
    {
        int first = blockIdx.x * kArenas;
        int cnt = g.n - first < kArenas ? g.n - first : kArenas;
        const int chunks = kRec / 16;
        for (int k = threadIdx.x; k < cnt * chunks; k += kWG) {
            int a = k / chunks, c = k % chunks;
            const uint4* src = (const uint4*)(g.arenas + (size_t)(first + a) * kRec) + c;
            uint4* dst = (uint4*)&lds[a] + c;
            *dst = *src;
        }
    }
    sync(); P.mark(11);
    if (valid && l < 5) {
        A->a.force[l] = zero3();
        A->a.torque[l] = zero3();
        update_inertia(A, l);
    }
    if (l == 0) {
        A->a.epa_lock = A->a.npen = 0;
        A->a.arith = g.arith;
    }
    if (threadIdx.x == 0) g_pen_save.cap = g.pen_slots;
    sync(); P.mark(11);
    // ---- StepFirstHalf (EnvSet.cpp:113-130) prelude
    if (g.ticks_first > 0) {
        if (valid && l == 0) {
            rlgpu_env_extra& e = A->s.env;
            for (int i = 0; i < 3; i++) e.prev_ball_vel[i] = A->s.ball.vel[i] * kBT2UU;
            for (int i = 0; i < 4; i++) {
                e.prev_boost[i] = A->s.cars[i].boost;
                e.prev_is_flipping[i] = A->s.cars[i].is_flipping;
                e.prev_on_ground[i] = A->s.cars[i].is_on_ground;
                e.ev_bump[i] = e.ev_bumped[i] = e.ev_demo[i] = e.ev_demoed[i] = 0;
            }
            e.has_prev = 1;
        }
        sync(); P.mark(11);
    }
    // ---- the ticks of both halves in ONE loop (a single inlined copy of the tick body keeps the
    // kernel's hot code small enough for the instruction cache); StepSecondHalf's action parse
    // (EnvSet.cpp:132-156) runs when the first half's actionDelay ticks are done
    {
        PadRegs pregs;
        load_pad_regs(pregs, l);
        const int t1 = g.ticks_first, t2 = g.actions ? g.ticks_second : 0;
        for (int t = 0;; t++) {
            if (g.actions && t == t1) {
                if (valid && l < 4) {
                    int a = g.actions[arena * 4 + l];
                    a = a < 0 ? 0 : (a > RLGPU_ACTIONS - 1 ? RLGPU_ACTIONS - 1 : a);
                    const float* x = C.action[a];
                    float* c = A->s.cars[l].controls;
                    for (int k = 0; k < 5; k++) c[k] = x[k];
                    c[5] = x[5] == 1 ? 1.f : 0.f;
                    c[6] = x[6] == 1 ? 1.f : 0.f;
                    c[7] = x[7] == 1 ? 1.f : 0.f;
                    for (int k = 0; k < 8; k++) A->s.env.prev_action[l][k] = x[k];
                }
                sync(); P.mark(11);
            }
            if (t >= t1 + t2) break;
            tick(A, g.mesh, l, valid, g.seed, arena + g.arena_offset, P, pregs, stdmin(kArenas, g.n - (int)blockIdx.x * kArenas));
        }
    }
    // ---- builders: GameState::UpdateFromArena, terminals, rewards, obs, masks
    uint8_t term = 0;
    if (g.build) {
        if (valid && l == 0) {
            rlgpu_env_extra& e = A->s.env;
            int64_t cur = e.tick_count;
            int64_t tick_skip = cur - e.last_tick_count > 0 ? cur - e.last_tick_count : 0;
            float delta_time = (int)tick_skip * (1.0f / 120.0f);
            bool any = false;
            for (int i = 0; i < 4; i++) {
                const rlgpu_car& c = A->s.cars[i];
                bool t = c.ball_hit_valid && (uint64_t)c.ball_hit_tick >= (uint64_t)(cur - tick_skip);
                A->a.touched[i] = t;
                any |= t;
            }
            float by = A->s.ball.pos[1] * kBT2UU;
            bool goal = fabsf(by) > (5124.25f + 91.25f);
            A->a.goal = goal;
            // the conditions' state: NoTouchCondition::timeSinceTouch and ScoreLimitCondition's goal
            // counts evolve identically in every instance (each IsTerminal is called every step), so one
            // copy serves any number of instances with different limits
            if (any) e.no_touch_time = 0;
            else e.no_touch_time += delta_time;
            if (goal) {
                if (by > 0) e.score_blue++;
                else e.score_orange++;
            }
            // terminal merge over the registry's list (EnvSet.cpp:167-180): NORMAL dominates
            uint8_t tt = 0;
            for (int k = 0; k < g.plug->nt; k++) {
                const rlgpu_terminal_spec& tc = g.plug->tc[k];
                bool hit = false, trunc = false;
                if (tc.type == RLGPU_TC_NO_TOUCH) {
                    hit = !any && e.no_touch_time >= tc.param;
                    trunc = true;
                } else if (tc.type == RLGPU_TC_SCORE_LIMIT) {
                    const int lim = (int)tc.param;
                    hit = (e.score_blue >= lim) || (e.score_orange >= lim);
                } else if (tc.type == RLGPU_TC_GOAL_SCORE) {
                    hit = goal;
                }
                if (hit) {
                    const uint8_t cur = trunc ? 2 : 1;
                    if (tt == 0 || cur == 1) tt = cur;
                }
            }
            e.terminal = tt;
            if (goal) {
                if (by > 0) e.penalty_blue++;
                else e.penalty_orange++;
            }
            // trajectory-level code (Learner.cpp:829-861): max episode length truncates the
            // trajectory without resetting the arena
            e.episode_steps++;
            uint8_t tj = tt;
            if (!tj && g.max_episode_steps > 0 && e.episode_steps >= g.max_episode_steps) tj = 2;
            if (tj) e.episode_steps = 0;
            A->a.traj_term = tj;
        }
        sync(); P.mark(12);
        if (valid) {
            // the arena's 16 lanes: lane l evaluates player l & 3's rewards r = l >> 2, + 4, + 8, ... (each reward is a
            // pure function of the snapshot); then the player's lane sums them in list order, allRewards[i] +=
            // out[i] * weight (EnvSet.cpp:199-222), fetching each value from the lane that computed it
            const int pi = l & 3, q = l >> 2;
            const PView me = view_player(A, pi);  // the other players' views are read where used
            v3 bp = ld3(A->s.ball.pos) * kBT2UU, bv = ld3(A->s.ball.vel) * kBT2UU, pbv = ld3(A->s.env.prev_ball_vel);
            const int nr = g.plug->nr;
            constexpr int kPer = (RLGPU_MAX_REWARDS + 3) / 4;
            float ov[kPer];
#pragma unroll
            for (int k = 0; k < kPer; k++) ov[k] = 0.f;
#pragma unroll 1
            for (int k = 0; q + 4 * k < nr; k++) {
                const int r = q + 4 * k;
                const float o = reward_value(A, g.plug->rw[r], pi, me, bp, bv, pbv, A->a.goal != 0);
#pragma unroll
                for (int j = 0; j < kPer; j++) ov[j] = j == k ? o : ov[j];  // no run-time register index
                if (pi == 0 && g.last_rewards) g.last_rewards[(size_t)arena * nr + r] = o;
                if (g.reward_values) g.reward_values[((size_t)arena * 4 + pi) * nr + r] = o;
            }
            float all = 0.f;
            const int base = (int)(threadIdx.x & ~15u) + pi;
#pragma unroll
            for (int r = 0; r < RLGPU_MAX_REWARDS; r++) {
                if (r >= nr) break;
                const float o = __shfl(ov[r >> 2], base + 4 * (r & 3));
                all += o * g.plug->rw[r].weight;
            }
            if (l < 4) A->a.all_rewards[l] = all;
        }
        sync(); P.mark(12);
        if (valid && l < 4) {
            float r = A->a.all_rewards[l];
            g.rewards[arena * 4 + l] = r;
            if (g.out_rew) g.out_rew[arena * 4 + l] = r;
            if (g.out_term) g.out_term[arena * 4 + l] = (int8_t)A->a.traj_term;
        }
        if (g.metrics && valid && l < 4) step_metrics(A, l, g.metrics + (size_t)arena * RLGPU_STEP_METRIC_SLOTS,
                                                      g.metrics_players != 0);
        uint8_t tj = 0;
        if (valid) {
            term = A->s.env.terminal;
            tj = (uint8_t)A->a.traj_term;
        }
        sync(); P.mark(12);
        if (valid && l == 0) {
            g.terminals[arena] = term;
            A->s.env.last_tick_count = A->s.env.tick_count;
        }
        const bool fused_reset = g.reset_mode == 1 && valid && term != 0;
        if (valid) build_obs_rows(A, l);
        sync(); P.mark(13);
        if (valid) {
            copy_rows(A, l, arena, g.obs, g.masks);
            if (!fused_reset) copy_rows(A, l, arena, g.out_obs, g.out_masks);
            if (tj == 2) {
                copy_rows(A, l, arena, g.trunc_obs, nullptr);
                copy_rows(A, l, arena, g.out_trunc, nullptr);
            }
        }
        sync(); P.mark(13);
        if (g.reset_mode == 1) {
            if (fused_reset && l == 0) kickoff_reset(A, g.seed, arena + g.arena_offset, g.fuzz != 0);
            sync(); P.mark(14);
            if (fused_reset) build_obs_rows(A, l);
            sync(); P.mark(14);
            if (fused_reset) {
                copy_rows(A, l, arena, g.obs, g.masks);
                copy_rows(A, l, arena, g.out_obs, g.out_masks);
            }
            sync(); P.mark(14);
        }
    }
    // ---- EnvSet::Reset / ResetArena / obs rebuild
    if (g.reset_mode >= 2) {
        bool do_reset = false;
        if (valid) {
            if (g.reset_mode == 2) do_reset = g.terminals[arena] != 0;
            else if (g.reset_mode == 3) do_reset = g.reset_mask ? g.reset_mask[arena] != 0 : true;
            else if (g.reset_mode == 4) do_reset = true;
        }
        sync(); P.mark(14);
        if (do_reset && l == 0) {
            kickoff_reset(A, g.seed, arena + g.arena_offset, g.fuzz != 0);
            if (g.reset_mode == 2) g.terminals[arena] = 0;
        }
        sync(); P.mark(14);
        bool rebuild = do_reset || (valid && g.reset_mode == 5);
        if (rebuild) build_obs_rows(A, l);
        sync(); P.mark(14);
        if (rebuild) copy_rows(A, l, arena, g.obs, g.masks);
        sync(); P.mark(14);
    }
    // ---- write the records back
    {
        int first = blockIdx.x * kArenas;
        int cnt = g.n - first < kArenas ? g.n - first : kArenas;
        const int chunks = kRec / 16;
        for (int k = threadIdx.x; k < cnt * chunks; k += kWG) {
            int a = k / chunks, c = k % chunks;
            uint4* dst = (uint4*)(g.arenas + (size_t)(first + a) * kRec) + c;
            const uint4* src = (const uint4*)&lds[a] + c;
            *dst = *src;
        }
    }
    P.mark(15);
    if (g.prof && valid && l == 0 && A->a.npen) {  // penetration-solver calls: total and this workgroup's
        atomicAdd(&g.prof[28], (unsigned long long)A->a.npen);
        atomicAdd(&g.prof[kProfWG + (size_t)blockIdx.x * kProfPhases + 23], (unsigned long long)A->a.npen);
        atomicAdd(&g.prof[kProfWG + (size_t)gridDim.x * kProfPhases + arena], (unsigned long long)A->a.npen);
    }
}
#endif  // RLGPU_ENV_KERNEL

}  // namespace rl
