// EnvSetGPU.hpp -- RLGC::EnvSet's interface over the device env set, for a caller that keeps the reference's
// EnvCreateFn (RG/EnvSet/EnvSet.h:14-34, src/ExampleMain.cpp:128-226) and its Learner loop
// (GigaLearnCPP Learner.cpp:603-861: StepFirstHalf / StepSecondHalf / Reset / ResetArena, state.*).
//
// * The EnvCreateFn's plugin objects are translated into the device registry (rlgpu_reward_spec /
//   rlgpu_terminal_spec, include/rlgpu_env.h) by exact dynamic type: every registry class with the
//   constructor fields the reference declares (StrongTouchReward's speeds, GoalReward's concedeScale,
//   ZeroSumReward's wrapper over a registry child, NoTouchCondition's maxTime, ...).
// * A Reward or TerminalCondition of any other type -- a user's own plugin -- runs on the host through its own
//   virtuals, in StepSecondHalf, as EnvSet::StepSecondHalf calls them (EnvSet.cpp:163-250): the step's
//   GameStates come down (rlgpu_envset_download_gamestates), the host conditions merge into the device's
//   terminal (NORMAL dominating TRUNCATED), every host reward gets PreStep then GetAllRewardsInPlace(gs,
//   isFinal = terminal != 0, out), and the weighted sum is rebuilt in list order from the device's per-reward
//   values (rlgpu_envset_reward_values) and the host values, then written back to state.rewards /
//   state.terminals.  The fallback is counted (fallbackStats) and announced once on stderr; with no host
//   plugin nothing crosses the bus.
// * obs / masks stay on the device (AdvancedObs and DefaultAction are the kernels'); ResetArena re-runs the
//   host plugins' Reset(initialState) on the arena's new GameState (EnvSet.cpp:275-303).
//
// Builds against this repository's RLGC.hpp or, with RLGPU_FACADE_RLGC_HEADER naming a header that pulls in
// the reference's RLGymCPP types, inside the reference tree.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <typeinfo>
#include <vector>

#include "../../include/rlgpu_core.h"
#include "../../include/rlgpu_env.h"
#include "../../include/rlgpu_gamestate.h"
#ifdef RLGPU_FACADE_RLGC_HEADER
#include RLGPU_FACADE_RLGC_HEADER
#else
#include "RLGC.hpp"
#endif

namespace RLGC {

inline void RlgpuCheck(int st, const char* what) {
    if (st != RLGPU_OK) throw std::runtime_error(std::string(what) + ": " + rlgpu_last_error());
}
inline void RlgpuCheckHip(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// ---------------------------------------------------------------------------------------------------------
// Translation: EnvCreateResult -> device registry + host plugin list
// ---------------------------------------------------------------------------------------------------------
struct PluginPlan {
    std::vector<rlgpu_reward_spec> deviceRewards;      // the registry entries, in list order
    std::vector<rlgpu_terminal_spec> deviceTerminals;
    std::vector<int> rewardSlot;                        // per EnvCreateResult::rewards entry: device index, -1 = host
    std::vector<int> hostTerminals;                     // indices into terminalConditions that run on the host
    std::vector<std::string> hostNames;                 // host plugins' type names (the log line)
    int32_t stateSetter = RLGPU_SS_KICKOFF;             // KickoffState / FuzzedKickoffState
    int NumHostRewards() const {
        int n = 0;
        for (int s : rewardSlot) n += s < 0;
        return n;
    }
    bool HasHost() const { return NumHostRewards() > 0 || !hostTerminals.empty(); }
};

namespace detail {
template <class T>
inline bool Is(const void* p, const std::type_info& t) {
    return p && t == typeid(T);
}

// StrongTouchReward stores KPHToVel(kph); the registry takes the kph and multiplies by the same 250/9 on the
// device, so find the float whose product reproduces the stored speed exactly -- the shortest decimal first
// (the constructor argument as written, e.g. 20 rather than its neighbour 20.000002)
inline float KphFromVel(float vel, const char* what) {
    const float c = 250.f / 9.f;
    float k = vel / c;
    for (int d = 0; d <= 7; d++) {
        const double s = std::pow(10.0, d);
        const float r = (float)(std::round((double)k * s) / s);
        if (r * c == vel) return r;
    }
    if (k * c == vel) return k;
    float up = k, dn = k;
    for (int i = 0; i < 8; i++) {
        up = std::nextafter(up, INFINITY);
        dn = std::nextafter(dn, -INFINITY);
        if (up * c == vel) return up;
        if (dn * c == vel) return dn;
    }
    throw std::invalid_argument(std::string("StrongTouchReward: ") + what + " is not KPHToVel of any float");
}

// the registry entry of one reward object, or false when the device has no code for its exact type
inline bool RegistryReward(Reward* r, rlgpu_reward_spec& s) {
    const std::type_info& t = typeid(*r);
    s.params[0] = s.params[1] = s.params[2] = 0;
    if (Is<ZeroSumReward>(r, t)) {
        auto* z = static_cast<ZeroSumReward*>(r);
        if (!z->child || !RegistryReward(z->child, s) || s.zero_sum) return false;
        s.zero_sum = 1;
        s.zero_sum_team_spirit = z->teamSpirit;
        s.zero_sum_opponent_scale = z->opponentScale;
        return true;
    }
    s.zero_sum = 0;
    s.zero_sum_team_spirit = s.zero_sum_opponent_scale = 0;
    if (Is<AirReward>(r, t)) s.type = RLGPU_RW_AIR;
    else if (Is<WavedashReward>(r, t)) s.type = RLGPU_RW_WAVEDASH;
    else if (Is<KickoffProximityReward2v2Enhanced>(r, t)) {
        auto* k = static_cast<KickoffProximityReward2v2Enhanced*>(r);
        // the tunables GetReward reads (KickoffProximityReward2v2Enhanced.h:9,12,135,175); cheaterReward and
        // dynamicWeight are declared but never read by it
        s.type = RLGPU_RW_KICKOFF_PROXIMITY_2V2;
        if (k->goerReward != 1.2f || k->rotationPrepWeight != 0.2f) {  // defaults stay the registry's zero params
            s.params[0] = k->goerReward;
            s.params[1] = k->rotationPrepWeight;
            s.params[2] = 1.f;
        }
    } else if (Is<VelocityPlayerToBallReward>(r, t)) s.type = RLGPU_RW_VELOCITY_PLAYER_TO_BALL;
    else if (Is<StrongTouchReward>(r, t)) {
        auto* st = static_cast<StrongTouchReward*>(r);
        s.type = RLGPU_RW_STRONG_TOUCH;
        s.params[0] = KphFromVel(st->minRewardedVel, "minRewardedVel");
        s.params[1] = KphFromVel(st->maxRewardedVel, "maxRewardedVel");
    } else if (Is<TouchAccelReward>(r, t)) s.type = RLGPU_RW_TOUCH_ACCEL;
    else if (Is<VelocityBallToGoalReward>(r, t)) {
        s.type = RLGPU_RW_VELOCITY_BALL_TO_GOAL;
        s.params[0] = static_cast<VelocityBallToGoalReward*>(r)->ownGoal ? 1.f : 0.f;
    } else if (Is<PickupBoostReward>(r, t)) s.type = RLGPU_RW_PICKUP_BOOST;
    else if (Is<SaveBoostReward>(r, t)) {
        s.type = RLGPU_RW_SAVE_BOOST;
        s.params[0] = static_cast<SaveBoostReward*>(r)->exponent;
    } else if (Is<BumpReward>(r, t)) s.type = RLGPU_RW_BUMP;
    else if (Is<DemoReward>(r, t)) s.type = RLGPU_RW_DEMO;
    else if (Is<GoalReward>(r, t)) {
        s.type = RLGPU_RW_GOAL;
        s.params[0] = static_cast<GoalReward*>(r)->concedeScale;
#ifndef RLGPU_FACADE_USER_EXAMPLEMAIN_CLASSES  // else ExampleMain's own class: a host plugin
    } else if (Is<LosingPenaltyReward>(r, t)) {
        s.type = RLGPU_RW_LOSING_PENALTY;
        s.params[0] = static_cast<LosingPenaltyReward*>(r)->penaltyScale;
#endif
    } else if (Is<BumpedPenalty>(r, t)) s.type = RLGPU_RW_BUMPED_PENALTY;
    else if (Is<DemoedPenalty>(r, t)) s.type = RLGPU_RW_DEMOED_PENALTY;
    else if (Is<VelocityReward>(r, t)) {
        s.type = RLGPU_RW_VELOCITY;
        s.params[0] = static_cast<VelocityReward*>(r)->isNegative ? 1.f : 0.f;
    } else if (Is<FaceBallReward>(r, t)) s.type = RLGPU_RW_FACE_BALL;
    else if (Is<TouchBallReward>(r, t)) s.type = RLGPU_RW_TOUCH_BALL;
    else if (Is<SpeedReward>(r, t)) s.type = RLGPU_RW_SPEED;
    else return false;
    return true;
}

inline bool RegistryTerminal(TerminalCondition* c, rlgpu_terminal_spec& s) {
    const std::type_info& t = typeid(*c);
    s.param = 0;
    if (Is<NoTouchCondition>(c, t)) {
        s.type = RLGPU_TC_NO_TOUCH;
        s.param = static_cast<NoTouchCondition*>(c)->maxTime;
#ifndef RLGPU_FACADE_USER_EXAMPLEMAIN_CLASSES
    } else if (Is<ScoreLimitCondition>(c, t)) {
        s.type = RLGPU_TC_SCORE_LIMIT;
        s.param = (float)static_cast<ScoreLimitCondition*>(c)->limit;
#endif
    } else if (Is<GoalScoreCondition>(c, t)) s.type = RLGPU_TC_GOAL_SCORE;
    else return false;
    return true;
}

inline bool SameSpec(const rlgpu_reward_spec& a, const rlgpu_reward_spec& b) {
    return a.type == b.type && a.weight == b.weight && a.params[0] == b.params[0] && a.params[1] == b.params[1] &&
           a.params[2] == b.params[2] && a.zero_sum == b.zero_sum && a.zero_sum_team_spirit == b.zero_sum_team_spirit &&
           a.zero_sum_opponent_scale == b.zero_sum_opponent_scale;
}
}  // namespace detail

// One arena's EnvCreateResult.  Throws std::invalid_argument for what neither side can run: a builder other
// than AdvancedObs / DefaultAction / KickoffState / FuzzedKickoffState (the kernels' own), a registry class with a field the
// registry cannot hold, or lists longer than RLGPU_MAX_REWARDS / RLGPU_MAX_TERMINALS.
inline PluginPlan TranslatePlugins(const EnvCreateResult& r) {
    if (r.obsBuilder && typeid(*r.obsBuilder) != typeid(AdvancedObs))
        throw std::invalid_argument(std::string("EnvCreateResult: obs builder ") + typeid(*r.obsBuilder).name() +
                                    " (the kernels build AdvancedObs)");
    if (r.actionParser && typeid(*r.actionParser) != typeid(DefaultAction))
        throw std::invalid_argument(std::string("EnvCreateResult: action parser ") + typeid(*r.actionParser).name() +
                                    " (the kernels parse DefaultAction)");
    if (r.stateSetter && typeid(*r.stateSetter) != typeid(KickoffState) && typeid(*r.stateSetter) != typeid(FuzzedKickoffState))
        throw std::invalid_argument(std::string("EnvCreateResult: state setter ") + typeid(*r.stateSetter).name() +
                                    " (the kernels reset to KickoffState or FuzzedKickoffState)");
    PluginPlan p;
    if (r.stateSetter && typeid(*r.stateSetter) == typeid(FuzzedKickoffState)) p.stateSetter = RLGPU_SS_FUZZED_KICKOFF;
    for (const WeightedReward& w : r.rewards) {
        if (!w.reward) throw std::invalid_argument("EnvCreateResult: null reward");
        rlgpu_reward_spec s{};
        if (detail::RegistryReward(w.reward, s)) {
            s.weight = w.weight;
            p.rewardSlot.push_back((int)p.deviceRewards.size());
            p.deviceRewards.push_back(s);
        } else {
            p.rewardSlot.push_back(-1);
            p.hostNames.push_back(w.reward->GetName());
        }
    }
    for (size_t i = 0; i < r.terminalConditions.size(); i++) {
        TerminalCondition* c = r.terminalConditions[i];
        if (!c) throw std::invalid_argument("EnvCreateResult: null terminal condition");
        rlgpu_terminal_spec s{};
        if (detail::RegistryTerminal(c, s)) {
            p.deviceTerminals.push_back(s);
        } else {
            p.hostTerminals.push_back((int)i);
            p.hostNames.push_back(typeid(*c).name());
        }
    }
    if (p.deviceRewards.size() > RLGPU_MAX_REWARDS || p.deviceTerminals.size() > RLGPU_MAX_TERMINALS)
        throw std::invalid_argument("EnvCreateResult: more registry plugins than RLGPU_MAX_REWARDS / RLGPU_MAX_TERMINALS");
    return p;
}

// The arenas share one registry list: EnvCreateFn must give every arena the same classes and fields in the
// same order (the host plugin objects themselves stay per arena).
inline void RequireSamePlan(const PluginPlan& a, const PluginPlan& b, int index) {
    bool same = a.rewardSlot == b.rewardSlot && a.hostTerminals == b.hostTerminals && a.stateSetter == b.stateSetter &&
                a.deviceRewards.size() == b.deviceRewards.size() && a.deviceTerminals.size() == b.deviceTerminals.size();
    for (size_t i = 0; same && i < a.deviceRewards.size(); i++) same = detail::SameSpec(a.deviceRewards[i], b.deviceRewards[i]);
    for (size_t i = 0; same && i < a.deviceTerminals.size(); i++)
        same = a.deviceTerminals[i].type == b.deviceTerminals[i].type && a.deviceTerminals[i].param == b.deviceTerminals[i].param;
    if (!same)
        throw std::invalid_argument("EnvCreateFn(" + std::to_string(index) +
                                    ") returned plugins that differ from arena 0's (one device registry per env set)");
}

// ---------------------------------------------------------------------------------------------------------
// GameState from a device record (include/rlgpu_gamestate.h)
// ---------------------------------------------------------------------------------------------------------
namespace detail {
inline Vec V(const float* f) { return Vec(f[0], f[1], f[2]); }
inline RotMat R(const float* m) {
    RotMat r;
    r.forward = V(m);
    r.right = V(m + 3);
    r.up = V(m + 6);
    return r;
}
}  // namespace detail

// GameState::UpdateFromArena (GameState.cpp:60-131) on a record: prev links as the reference sets them
// (this->prev = prev, prev->prev = NULL, players[i].prev = &prev->players[i]), lastTouchCarID carried over
// unless a player touched the ball this step.  fresh: the GameState(arena) of ResetArena, whose first
// UpdateFromArena counts the ticks since tick 0 (deltaTime = tickCount / 120, every valid hit in the window).
inline void FillGameState(GameState& gs, const rlgpu_gamestate& g, GameState* prev, bool fresh) {
    gs.prev = prev;
    if (prev) prev->prev = nullptr;
    if (fresh) {
        gs.lastTouchCarID = -1;
        gs.deltaTime = (int)g.last_tick_count * (1.0f / 120.0f);
    } else {
        gs.deltaTime = g.delta_time;
    }
    gs.goalScored = g.goal_scored != 0;
    gs.lastTickCount = g.last_tick_count;
    gs.ball.pos = detail::V(g.ball.pos);
    gs.ball.rotMat = detail::R(g.ball.rot);
    gs.ball.vel = detail::V(g.ball.vel);
    gs.ball.angVel = detail::V(g.ball.ang_vel);
    gs.players.resize(RLGPU_CARS);
    for (int i = 0; i < RLGPU_CARS; i++) {
        const rlgpu_player_state& s = g.players[i];
        const rlgpu_car_state& c = s.car;
        Player& p = gs.players[i];
        p.pos = detail::V(c.pos);
        p.rotMat = detail::R(c.rot);
        p.vel = detail::V(c.vel);
        p.angVel = detail::V(c.ang_vel);
        p.isOnGround = c.is_on_ground;
        for (int w = 0; w < 4; w++) p.wheelsWithContact[w] = c.wheels_with_contact[w];
        p.hasJumped = c.has_jumped;
        p.hasDoubleJumped = c.has_double_jumped;
        p.hasFlipped = c.has_flipped;
        p.flipRelTorque = detail::V(c.flip_rel_torque);
        p.jumpTime = c.jump_time;
        p.flipTime = c.flip_time;
        p.isFlipping = c.is_flipping;
        p.isJumping = c.is_jumping;
        p.airTime = c.air_time;
        p.airTimeSinceJump = c.air_time_since_jump;
        p.boost = c.boost;
        p.timeSpentBoosting = c.time_spent_boosting;
        p.isSupersonic = c.is_supersonic;
        p.supersonicTime = c.supersonic_time;
        p.handbrakeVal = c.handbrake_val;
        p.isAutoFlipping = c.is_auto_flipping;
        p.autoFlipTimer = c.auto_flip_timer;
        p.autoFlipTorqueScale = c.auto_flip_torque_scale;
        p.worldContact.hasContact = c.world_contact_has_contact;
        p.worldContact.contactNormal = detail::V(c.world_contact_normal);
        p.carContact.otherCarID = c.car_contact_other_car_id;
        p.carContact.cooldownTimer = c.car_contact_cooldown_timer;
        p.isDemoed = c.is_demoed;
        p.demoRespawnTimer = c.demo_respawn_timer;
        p.ballHitInfo.isValid = c.ball_hit_is_valid;
        p.ballHitInfo.relativePosOnBall = detail::V(c.ball_hit_relative_pos_on_ball);
        p.ballHitInfo.ballPos = detail::V(c.ball_hit_ball_pos);
        p.ballHitInfo.extraHitVel = detail::V(c.ball_hit_extra_hit_vel);
        p.ballHitInfo.tickCountWhenHit = (uint64_t)c.ball_hit_tick_count_when_hit;
        p.ballHitInfo.tickCountWhenExtraImpulseApplied = (uint64_t)c.ball_hit_tick_count_when_extra_impulse_applied;
        p.lastControls.throttle = c.last_controls[0];
        p.lastControls.steer = c.last_controls[1];
        p.lastControls.pitch = c.last_controls[2];
        p.lastControls.yaw = c.last_controls[3];
        p.lastControls.roll = c.last_controls[4];
        p.lastControls.jump = c.last_controls[5] != 0;
        p.lastControls.boost = c.last_controls[6] != 0;
        p.lastControls.handbrake = c.last_controls[7] != 0;
        p.prev = prev && (int)prev->players.size() > i ? &prev->players[i] : nullptr;
        if (p.prev) p.prev->prev = nullptr;
        p.index = s.index;
        p.carId = s.car_id;
        p.team = (Team)s.team;
        p.eventState = PlayerEventState{};
        p.eventState.bump = s.events[5];
        p.eventState.bumped = s.events[6];
        p.eventState.demo = s.events[7];
        p.eventState.demoed = s.events[8];
        if (fresh) {  // Player.cpp:17-22 with tickSkip = tickCount (lastTickCount 0)
            p.ballTouchedStep = c.ball_hit_is_valid != 0;
            p.ballTouchedTick = c.ball_hit_is_valid && (uint64_t)c.ball_hit_tick_count_when_hit == g.last_tick_count - 1;
        } else {
            p.ballTouchedStep = s.ball_touched_step;
            p.ballTouchedTick = s.ball_touched_tick;
        }
        if (p.ballTouchedStep) gs.lastTouchCarID = (int)p.carId;
        const float* pa = s.prev_action;
        p.prevAction.throttle = pa[0];
        p.prevAction.steer = pa[1];
        p.prevAction.pitch = pa[2];
        p.prevAction.yaw = pa[3];
        p.prevAction.roll = pa[4];
        p.prevAction.jump = pa[5];
        p.prevAction.boost = pa[6];
        p.prevAction.handbrake = pa[7];
    }
    gs.boostPads.assign(g.boost_pads, g.boost_pads + RLGPU_PADS);
    gs.boostPadsInv.assign(g.boost_pads_inv, g.boost_pads_inv + RLGPU_PADS);
    gs.boostPadTimers.assign(g.boost_pad_timers, g.boost_pad_timers + RLGPU_PADS);
    gs.boostPadTimersInv.assign(g.boost_pad_timers_inv, g.boost_pad_timers_inv + RLGPU_PADS);
}

// ---------------------------------------------------------------------------------------------------------
// EnvSetGPU
// ---------------------------------------------------------------------------------------------------------
struct EnvSetGPUOptions {
    uint64_t seed = 0;
    int32_t arith = RLGPU_ARITH_MSVC_X64;
    int32_t maxEpisodeSteps = 0;
    int32_t arenaOffset = 0;
    const float* meshTris = nullptr;  // null: the built-in synthetic arena (rlgpu_envset_config)
    int32_t meshNtris = 0, meshObjects = 0;
    const int32_t* meshObjectNtris = nullptr;
};

struct FallbackStats {
    int hostRewards = 0, hostTerminals = 0;  // plugins per arena that run on the host
    uint64_t steps = 0;                       // StepSecondHalf calls that ran them
    uint64_t rewardCalls = 0, terminalCalls = 0, resetCalls = 0;  // host plugin invocations (all arenas)
};

class EnvSetGPU {
  public:
    EnvSetConfig config;
    rlgpu_envset* h = nullptr;
    rlgpu_envset_buffers state{};  // device views of EnvState (EnvSet.h:35-60)
    hipStream_t stream = nullptr;
    std::vector<EnvCreateResult> results;  // the EnvCreateFn's per-arena plugin objects (owned)
    PluginPlan plan;
    FallbackStats fallbackStats;
    // host mirrors of EnvState::gameStates / prevGameStates: kept every step while host plugins run,
    // refreshed by GetGameStates() otherwise
    std::vector<GameState> gameStates, prevGameStates;
    std::vector<std::vector<float>> lastRewards;  // [arena][list entry] (saveRewards with host rewards)
    int obsSize = RLGPU_OBS, numActions = RLGPU_ACTIONS;

    EnvSetGPU(const EnvSetConfig& c, const EnvSetGPUOptions& o = {}, hipStream_t s = nullptr) : config(c), stream(s) {
        plan = CreateEnvs(c, results);
        rlgpu_envset_config cfg{};
        cfg.num_arenas = c.numArenas;
        cfg.tick_skip = c.tickSkip;
        cfg.action_delay = c.actionDelay;
        cfg.seed = o.seed;
        cfg.save_rewards = c.saveRewards;
        cfg.max_episode_steps = o.maxEpisodeSteps;
        cfg.mesh_tris = o.meshTris;
        cfg.mesh_ntris = o.meshNtris;
        cfg.mesh_objects = o.meshObjects;
        cfg.mesh_object_ntris = o.meshObjectNtris;
        cfg.rewards = plan.deviceRewards.data();
        cfg.n_rewards = (int32_t)plan.deviceRewards.size();
        cfg.terminals = plan.deviceTerminals.data();
        cfg.n_terminals = (int32_t)plan.deviceTerminals.size();
        // an empty list is a list (no rewards), not the NULL that selects ExampleMain's
        static const rlgpu_reward_spec kNoRewards{};
        static const rlgpu_terminal_spec kNoTerminals{};
        if (!cfg.rewards) cfg.rewards = &kNoRewards;
        if (!cfg.terminals) cfg.terminals = &kNoTerminals;
        cfg.arith = o.arith;
        cfg.arena_offset = o.arenaOffset;
        cfg.state_setter = plan.stateSetter;
        RlgpuCheck(rlgpu_envset_create(&cfg, &h), "EnvSet");
        RlgpuCheck(rlgpu_envset_buffers_get(h, &state), "EnvSet buffers");
        InitHost();
    }
    // Attached to a device env set made by someone else from this plan's registry lists (the trainer facade: the
    // C++ Learner owns the env set, the plugin objects and the host fallback live here).  Not destroyed here.
    EnvSetGPU(const EnvSetConfig& c, std::vector<EnvCreateResult>&& res, const PluginPlan& p, rlgpu_envset* attached,
              hipStream_t s)
        : config(c), h(attached), stream(s), results(std::move(res)), plan(p), owns(false) {
        if (!h) throw std::invalid_argument("EnvSetGPU: null env set to attach to");
        RlgpuCheck(rlgpu_envset_buffers_get(h, &state), "EnvSet buffers");
        if (state.num_arenas != c.numArenas) throw std::invalid_argument("EnvSetGPU: attached env set has another arena count");
        InitHost();
    }

    // EnvSet ctor (EnvSet.cpp:46-111): one EnvCreateFn call per arena, each result's arena checked against the
    // device's and its plugins translated; every arena must give the same plan.  Returns it.
    static PluginPlan CreateEnvs(const EnvSetConfig& c, std::vector<EnvCreateResult>& results) {
        if (!c.envCreateFn) throw std::invalid_argument("EnvSetConfig: no envCreateFn");
        if (c.numArenas <= 0) throw std::invalid_argument("EnvSetConfig: numArenas must be positive");
        PluginPlan plan;
        results.reserve(c.numArenas);
        for (int i = 0; i < c.numArenas; i++) {
            results.push_back(c.envCreateFn(i));
            RequireDeviceArena(results.back().arena, i);
            PluginPlan p = TranslatePlugins(results.back());
            if (i == 0) plan = p;
            else RequireSamePlan(plan, p, i);
        }
        return plan;
    }

  private:
    void InitHost() {
        const EnvSetConfig& c = config;
        fallbackStats.hostRewards = plan.NumHostRewards();
        fallbackStats.hostTerminals = (int)plan.hostTerminals.size();
        if (plan.HasHost()) {
            std::string names;
            for (auto& n : plan.hostNames) names += (names.empty() ? "" : ", ") + n;
            std::fprintf(stderr, "EnvSetGPU: %d reward(s) and %d terminal condition(s) without device code run on the host "
                                 "every step (%s)\n", fallbackStats.hostRewards, fallbackStats.hostTerminals, names.c_str());
            if (plan.NumHostRewards() > 0) RlgpuCheck(rlgpu_envset_enable_reward_values(h, 1), "EnvSet reward values");
            hostTerms.assign(c.numArenas, 0);
            hostRewards.assign((size_t)state.num_players, 0.f);
            if (c.saveRewards) lastRewards.assign(c.numArenas, std::vector<float>(results[0].rewards.size(), 0.f));
            // the initial ResetArena of every arena (EnvSet.cpp:105-110): plugins' Reset on the new states
            std::vector<int> all(c.numArenas);
            for (int i = 0; i < c.numArenas; i++) all[i] = i;
            HostReset(all);
        }
    }

  public:
    EnvSetGPU(const EnvSetGPU&) = delete;
    EnvSetGPU& operator=(const EnvSetGPU&) = delete;
    ~EnvSetGPU() {
        if (owns) rlgpu_envset_destroy(h);
        if (dMask) (void)hipFree(dMask);
        if (dActions) (void)hipFree(dActions);
        for (auto& r : results) {
            delete r.arena;  // EnvSet owns its arenas (EnvSet.h:67-124)
            for (auto& w : r.rewards) delete w.reward;
            for (auto* t : r.terminalConditions) delete t;
            delete r.obsBuilder;
            delete r.actionParser;
            delete r.stateSetter;
        }
    }

    void StepFirstHalf(bool async) {
        if (plan.HasHost())
            for (int a = 0; a < config.numArenas; a++) prevGameStates[a] = gameStates[a];  // EnvSet.cpp:119-120
        RlgpuCheck(rlgpu_envset_step_first_half(h, stream), "StepFirstHalf");
        if (!async) Sync();
    }

    void StepSecondHalf(const int32_t* dActions, bool async) {
        RlgpuCheck(rlgpu_envset_step_second_half(h, dActions, stream), "StepSecondHalf");
        if (plan.HasHost()) HostStep();
        if (!async) Sync();
    }

    // EnvSet::StepSecondHalf(const IList& actionIndices, bool async) (EnvSet.h:106): host action indices, one per
    // player, uploaded to the device
    void StepSecondHalf(const IList& actions, bool async) {
        if ((int)actions.size() != state.num_players)
            throw std::invalid_argument("StepSecondHalf: " + std::to_string(actions.size()) + " actions for " +
                                        std::to_string(state.num_players) + " players");
        if (!dActions) RlgpuCheckHip(hipMalloc(&dActions, (size_t)state.num_players * sizeof(int32_t)), "actions");
        static_assert(sizeof(int) == sizeof(int32_t), "IList holds int32 action indices");
        RlgpuCheckHip(hipMemcpyAsync(dActions, actions.data(), actions.size() * sizeof(int32_t), hipMemcpyHostToDevice, stream),
                      "actions");
        StepSecondHalf(dActions, async);
    }

    void Sync() { RlgpuCheck(rlgpu_envset_sync(h, stream), "Sync"); }

    // The trainer facade's step hook (rlgpu_learner_set_step_hook) on an attached set: after the device step, the
    // host plugins as StepSecondHalf runs them (the previous states kept as StepFirstHalf does); after the reset,
    // the plugins' Reset on the arenas whose merged terminal reset them.
    void HostAfterStep() {
        if (!plan.HasHost()) return;
        for (int a = 0; a < config.numArenas; a++) prevGameStates[a] = gameStates[a];
        HostStep();
    }
    void HostAfterReset() {
        if (!plan.HasHost()) return;
        std::vector<int> reset;
        for (int a = 0; a < config.numArenas; a++)
            if (hostTerms[a]) reset.push_back(a);
        if (!reset.empty()) HostReset(reset);
    }

    // EnvSet::Reset: every arena whose terminal is set (the merged host + device terminal)
    void Reset() {
        std::vector<int> reset;
        if (plan.HasHost()) {
            Sync();
            for (int a = 0; a < config.numArenas; a++)
                if (hostTerms[a]) reset.push_back(a);
        }
        RlgpuCheck(rlgpu_envset_reset(h, stream), "Reset");
        if (!reset.empty()) HostReset(reset);
    }

    void ResetArena(int i) {
        if (i < 0 || i >= config.numArenas) throw std::out_of_range("ResetArena: arena index");
        if (!dMask) RlgpuCheckHip(hipMalloc(&dMask, config.numArenas), "ResetArena mask");
        RlgpuCheckHip(hipMemsetAsync(dMask, 0, config.numArenas, stream), "ResetArena mask");
        RlgpuCheckHip(hipMemsetAsync(dMask + i, 1, 1, stream), "ResetArena mask");
        RlgpuCheck(rlgpu_envset_reset_arenas(h, dMask, stream), "ResetArena");
        if (plan.HasHost()) HostReset({i});
    }

    // EnvState::gameStates for a StepCallbackFn (Learner.cpp:796-797): with host plugins these are the states
    // the plugins saw; otherwise one download of every arena
    const std::vector<GameState>& GetGameStates() {
        if (!plan.HasHost()) {
            Download(0, config.numArenas);
            gameStates.resize(config.numArenas);
            for (int a = 0; a < config.numArenas; a++) FillGameState(gameStates[a], recs[a], nullptr, false);
        }
        return gameStates;
    }

  private:
    bool owns = true;
    uint8_t* dMask = nullptr;
    int32_t* dActions = nullptr;
    std::vector<rlgpu_gamestate> recs;
    std::vector<uint8_t> hostTerms;
    std::vector<float> hostRewards, rewardValues;

    void Download(int first, int count) {
        recs.resize((size_t)config.numArenas);
        RlgpuCheck(rlgpu_envset_download_gamestates(h, first, count, recs.data() + first, stream), "download GameStates");
    }

    void HostReset(const std::vector<int>& arenas) {
        Sync();
        recs.resize((size_t)config.numArenas);
        gameStates.resize(config.numArenas);
        prevGameStates.resize(config.numArenas);
        for (int a : arenas) {
            RlgpuCheck(rlgpu_envset_download_gamestates(h, a, 1, recs.data() + a, stream), "download GameStates");
            GameState& gs = gameStates[a];
            FillGameState(gs, recs[a], nullptr, true);
            gs.userInfo = results[a].userInfo;
            for (int t : plan.hostTerminals) results[a].terminalConditions[t]->Reset(gs);
            for (size_t k = 0; k < plan.rewardSlot.size(); k++)
                if (plan.rewardSlot[k] < 0) results[a].rewards[k].reward->Reset(gs);
            fallbackStats.resetCalls++;
            prevGameStates[a].MakeEmpty();
            hostTerms[a] = 0;
        }
    }

    // EnvSet::StepSecondHalf's plugin part (EnvSet.cpp:163-255) for the host plugins
    void HostStep() {
        const int A = config.numArenas, P = state.num_players;
        const int ndev = (int)plan.deviceRewards.size(), nlist = (int)plan.rewardSlot.size();
        const bool hostRew = plan.NumHostRewards() > 0;
        Download(0, A);  // synchronises the stream first
        RlgpuCheckHip(hipMemcpy(hostTerms.data(), state.terminals, A, hipMemcpyDeviceToHost), "terminals");
        if (hostRew && ndev > 0) {
            rewardValues.resize((size_t)P * ndev);
            RlgpuCheckHip(hipMemcpy(rewardValues.data(), rlgpu_envset_reward_values(h), rewardValues.size() * sizeof(float),
                                    hipMemcpyDeviceToHost), "reward values");
        }
        std::vector<float> out(RLGPU_CARS), all(RLGPU_CARS);
        for (int a = 0; a < A; a++) {
            GameState* prev = prevGameStates[a].IsEmpty() ? nullptr : &prevGameStates[a];
            GameState& gs = gameStates[a];
            FillGameState(gs, recs[a], prev, false);
            gs.userInfo = results[a].userInfo;
            uint8_t term = hostTerms[a];
            for (int t : plan.hostTerminals) {
                TerminalCondition* c = results[a].terminalConditions[t];
                fallbackStats.terminalCalls++;
                if (c->IsTerminal(gs)) {
                    uint8_t cur = c->IsTruncation() ? TRUNCATED : NORMAL;
                    if (term == NOT_TERMINAL || cur == NORMAL) term = cur;
                }
            }
            hostTerms[a] = term;
            if (!hostRew) continue;
            for (int k = 0; k < nlist; k++)
                if (plan.rewardSlot[k] < 0) results[a].rewards[k].reward->PreStep(gs);
            std::fill(all.begin(), all.end(), 0.f);
            for (int k = 0; k < nlist; k++) {
                const WeightedReward& w = results[a].rewards[k];
                const int slot = plan.rewardSlot[k];
                if (slot >= 0) {
                    for (int i = 0; i < RLGPU_CARS; i++) out[i] = rewardValues[((size_t)a * RLGPU_CARS + i) * ndev + slot];
                } else {
                    w.reward->GetAllRewardsInPlace(gs, term != NOT_TERMINAL, out.data());
                    fallbackStats.rewardCalls++;
                }
                for (int i = 0; i < RLGPU_CARS; i++) all[i] += out[i] * w.weight;
                if (config.saveRewards) {  // the device's sample: player 0 (rlgpu_envset_buffers.last_rewards)
                    float v = out[0];
                    const std::vector<float>* inner = w.reward->GetInnerRewards();
                    if (slot < 0 && inner && !inner->empty()) v = (*inner)[0];
                    lastRewards[a][k] = v;
                }
            }
            for (int i = 0; i < RLGPU_CARS; i++) hostRewards[(size_t)a * RLGPU_CARS + i] = all[i];
        }
        RlgpuCheckHip(hipMemcpyAsync(state.terminals, hostTerms.data(), A, hipMemcpyHostToDevice, stream), "terminals");
        if (hostRew)
            RlgpuCheckHip(hipMemcpyAsync(state.rewards, hostRewards.data(), (size_t)P * sizeof(float), hipMemcpyHostToDevice,
                                         stream), "rewards");
        RlgpuCheckHip(hipStreamSynchronize(stream), "host plugin upload");  // the host buffers are reused next step
        fallbackStats.steps++;
    }
};

}  // namespace RLGC
