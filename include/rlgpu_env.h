/*
 * rlgpu_env.h -- C ABI of the vectorised RLGymCPP/RocketSim arena set on MI355X.
 *
 * Replaces the env side of the reference's hot path:
 *   RLGC::EnvSet            GigaLearnCPP/RLGymCPP/src/RLGymCPP/EnvSet/EnvSet.h:14-110
 *     EnvSet(const EnvSetConfig&)          EnvSet.cpp:46-111   -> rlgpu_envset_create
 *     StepFirstHalf(bool async)            EnvSet.cpp:113-130  -> rlgpu_envset_step_first_half
 *     StepSecondHalf(actions, bool async)  EnvSet.cpp:132-273  -> rlgpu_envset_step_second_half
 *     Sync()                               EnvSet.h:107        -> rlgpu_envset_sync
 *     ResetArena(int) / Reset()            EnvSet.cpp:275-354  -> rlgpu_envset_reset_arena / _reset
 *     state.{obs,actionMasks,rewards,terminals,arenaPlayerStartIdx}
 *                                          EnvSet.h:35-65      -> rlgpu_envset_buffers
 * The EnvCreateFn's plugin set (EnvCreateResult, EnvSet.h:14-24) is AdvancedObs, DefaultAction and
 * KickoffState, plus a device registry of weighted rewards and terminal conditions
 * (rlgpu_reward_spec / rlgpu_terminal_spec lists in rlgpu_envset_config; NULL lists = src/ExampleMain.cpp:
 * 128-226: the 13 weighted rewards and NoTouchCondition(8) + ScoreLimitCondition(3)).
 *
 * Arena state lives on the device as one 2,312-byte record per arena (array of structs: a
 * workgroup stages whole records into LDS with coalesced 16-byte loads, runs the step there and
 * writes them back once, so the record is read and written exactly once per step whatever the
 * access pattern inside -- DESIGN.md section 3); one env step is ONE kernel launch
 * (7 ticks with the previous controls, action parse, 1 tick, builders, reset-if-terminal)
 * when rlgpu_envset_step() is used, or two launches through the two-half API.
 *
 * All "d_" pointers are device pointers; "h_" pointers are host memory owned by the caller.
 */
#ifndef RLGPU_ENV_H
#define RLGPU_ENV_H

#include <stdint.h>
#include "rlgpu_arith.h"
#include "rlgpu_core.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RLGPU_CARS 4          /* 2v2 (src/ExampleMain.cpp:200-208) */
#define RLGPU_PADS 34         /* RLConst::BoostPads 6 big + 28 small (RLConst.h:212-214) */
#define RLGPU_MANIFOLDS 12    /* contact-manifold slots per arena per tick (build limit, overflow counted) */
#define RLGPU_MAX_SOLVER_ROWS 14 /* contact rows per arena per tick (build limit, overflow counted) */
#define RLGPU_MAX_MESH_OBJECTS 32 /* static collision meshes per arena (SOCCAR loads 16, HOOPS 12) */
#define RLGPU_OBS 167         /* AdvancedObs 9+8+34+29*4 (AdvancedObs.cpp:193-270) */
#define RLGPU_ACTIONS 90      /* DefaultAction table (DefaultAction.cpp:3-89) */
#define RLGPU_REWARDS 13      /* ExampleMain reward list (src/ExampleMain.cpp:132-177) */
#define RLGPU_MAX_REWARDS 32  /* weighted rewards per env set (device registry) */
#define RLGPU_MAX_TERMINALS 8 /* terminal conditions per env set */
#define RLGPU_SS_KICKOFF 0        /* KickoffState */
#define RLGPU_SS_FUZZED_KICKOFF 1 /* FuzzedKickoffState */

/* Reward plugins of the device registry: RLGymCPP's CommonRewards (RG/Rewards/CommonRewards.h),
 * KickoffProximityReward2v2Enhanced (RG/Rewards/KickoffProximityReward2v2Enhanced.h) and ExampleMain's
 * LosingPenaltyReward (src/ExampleMain.cpp:84-124).  params[] are the constructor arguments, 0 meaning
 * the reference default where noted.  The first 13 ids are ExampleMain's list in its order. */
enum {
    RLGPU_RW_AIR = 0,                     /* AirReward */
    RLGPU_RW_WAVEDASH = 1,                /* WavedashReward */
    RLGPU_RW_KICKOFF_PROXIMITY_2V2 = 2,   /* KickoffProximityReward2v2Enhanced: params[2] != 0 -> params[0] goerReward,
                                             params[1] rotationPrepWeight (else the class defaults 1.2 / 0.2;
                                             cheaterReward / dynamicWeight are never read by its GetReward) */
    RLGPU_RW_VELOCITY_PLAYER_TO_BALL = 3, /* VelocityPlayerToBallReward */
    RLGPU_RW_STRONG_TOUCH = 4,            /* StrongTouchReward(params[0] minSpeedKPH, params[1] maxSpeedKPH) */
    RLGPU_RW_TOUCH_ACCEL = 5,             /* TouchAccelReward */
    RLGPU_RW_VELOCITY_BALL_TO_GOAL = 6,   /* VelocityBallToGoalReward(params[0] ownGoal != 0) */
    RLGPU_RW_PICKUP_BOOST = 7,            /* PickupBoostReward */
    RLGPU_RW_SAVE_BOOST = 8,              /* SaveBoostReward(params[0] exponent) */
    RLGPU_RW_BUMP = 9,                    /* BumpReward (PlayerDataEventReward<bump>) */
    RLGPU_RW_DEMO = 10,                   /* DemoReward */
    RLGPU_RW_GOAL = 11,                   /* GoalReward(params[0] concedeScale) */
    RLGPU_RW_LOSING_PENALTY = 12,         /* LosingPenaltyReward(params[0] penaltyPerGoalBehind) */
    RLGPU_RW_BUMPED_PENALTY = 13,         /* BumpedPenalty */
    RLGPU_RW_DEMOED_PENALTY = 14,         /* DemoedPenalty */
    RLGPU_RW_VELOCITY = 15,               /* VelocityReward(params[0] isNegative != 0) */
    RLGPU_RW_FACE_BALL = 16,              /* FaceBallReward */
    RLGPU_RW_TOUCH_BALL = 17,             /* TouchBallReward */
    RLGPU_RW_SPEED = 18,                  /* SpeedReward */
    RLGPU_NUM_REWARD_TYPES = 19
};
/* One WeightedReward {Reward*, weight} (EnvSet.h:14-18).  zero_sum != 0: the reward is wrapped in
 * ZeroSumReward(child, zero_sum_team_spirit, zero_sum_opponent_scale) -- accepted for the API, and a
 * pass-through exactly as in the reference: ZeroSumReward overrides only GetAllRewards, while the hot
 * path calls GetAllRewardsInPlace, which runs the child's GetReward (ZeroSumReward.cpp:3-48,
 * Reward.h:43-48). */
typedef struct {
    int32_t type;      /* RLGPU_RW_* */
    float weight;
    float params[3];
    int32_t zero_sum;
    float zero_sum_team_spirit, zero_sum_opponent_scale;
} rlgpu_reward_spec;

/* Terminal conditions (RG/TerminalConditions/NoTouchCondition.h, GoalScoreCondition.h, src/ExampleMain.cpp:46-82).  The list is merged as
 * EnvSet::StepSecondHalf does: any condition sets the arena's terminal, NORMAL dominating TRUNCATED
 * (EnvSet.cpp:167-180). */
enum {
    RLGPU_TC_NO_TOUCH = 0,     /* NoTouchCondition(param maxTime s): truncation */
    RLGPU_TC_SCORE_LIMIT = 1,  /* ScoreLimitCondition(param goals): normal */
    RLGPU_TC_GOAL_SCORE = 2,   /* GoalScoreCondition: normal */
    RLGPU_NUM_TERMINAL_TYPES = 3
};
typedef struct {
    int32_t type;  /* RLGPU_TC_* */
    float param;
} rlgpu_terminal_spec;

/* One contact point (btManifoldPoint subset, bullet units). */
typedef struct {
    float localA[3], localB[3]; /* in body-A / body-B frames */
    float normalB[3];           /* normal on B, world space, pointing towards A */
    float dist;                 /* signed distance (negative = penetration) */
    float applied;              /* m_appliedImpulse (warm start; 0 for a fresh point) */
    float friction, restitution;
    int32_t special;            /* m_isSpecial: ball-world contact (Arena.cpp:265-273) */
} rlgpu_contact;

/* Contact manifold of one body pair, rebuilt every tick: RocketSim's broadphase removes every
 * overlapping pair at the start of each collision pass and re-adds the ones that still overlap
 * (btRSBroadphase.cpp:392-465), which destroys the pair's algorithm and its manifold
 * (btOverlappingPairCache.cpp:36-46, btConvexConvexAlgorithm.cpp:198-205,
 * btConvexConcaveCollisionAlgorithm.cpp:60-64).  So manifolds never outlive a tick and are not
 * part of the arena record; the kernels keep them in LDS scratch.  Key encoding: see
 * env_kernel.hpp / rsim_ref.cpp (pair_key). */
typedef struct {
    int32_t key;
    int32_t count;
    rlgpu_contact pts[4];
} rlgpu_manifold;

/* Rigid body, bullet units (1 = 50 uu); rot is btMatrix3x3 row-major, columns = forward,right,up. */
typedef struct {
    float pos[3];
    float rot[9];
    float vel[3];
    float angvel[3];
} rlgpu_body;

/* Car (RocketSim CarState, Car.h:17-100, plus the btVehicleRL wheel values that persist
 * across ticks, btVehicleRL.h:9-30, and CarControls). */
typedef struct {
    rlgpu_body body;
    float controls[8];      /* throttle, steer, pitch, yaw, roll, jump, boost, handbrake */
    float last_controls[8];
    float boost, jump_time, flip_time, air_time, air_time_since_jump, time_spent_boosting;
    float supersonic_time, handbrake_val, auto_flip_timer, auto_flip_torque_scale;
    float demo_respawn_timer, car_contact_cooldown;
    float flip_rel_torque[3];
    float world_contact_normal[3];
    float vel_impulse_cache[3];
    float ball_hit_rel_pos[3], ball_hit_ball_pos[3], ball_hit_extra_vel[3];
    int64_t ball_hit_tick;        /* -1 == never (~0ULL in the reference) */
    int64_t ball_hit_extra_tick;  /* -1 == never */
    uint32_t car_contact_other_id;
    uint8_t is_on_ground, has_jumped, has_double_jumped, has_flipped;
    uint8_t is_flipping, is_jumping, is_supersonic, is_auto_flipping;
    uint8_t world_contact, is_demoed, ball_hit_valid, pad0;
    uint8_t wheel_contact[4];
    /* btWheelInfoRL values read one tick after they are written */
    float wheel_steer[4], wheel_engine_force[4], wheel_brake[4];
    float wheel_lat_friction[4], wheel_long_friction[4], wheel_extra_pushback[4];
} rlgpu_car;

typedef struct {
    float cooldown;
    uint8_t is_active;
    uint8_t pad[3];
    uint32_t prev_locked_car_id;
} rlgpu_pad;

/* Per-arena env bookkeeping (GameState + plugin state). */
typedef struct {
    int64_t tick_count;          /* Arena::tickCount */
    int64_t last_tick_count;     /* GameState::lastTickCount */
    float prev_ball_vel[3];      /* GameState::prev->ball.vel (uu/s) */
    float prev_boost[RLGPU_CARS];
    uint8_t prev_is_flipping[RLGPU_CARS];
    uint8_t prev_on_ground[RLGPU_CARS];
    uint8_t has_prev;            /* prevGameStates[i] non-empty */
    uint8_t terminal;            /* last terminal type (0/1/2) */
    uint8_t pad[2];
    float prev_action[RLGPU_CARS][8];
    float no_touch_time;         /* NoTouchCondition::timeSinceTouch */
    int32_t score_blue, score_orange;     /* ScoreLimitCondition */
    int32_t penalty_blue, penalty_orange; /* LosingPenaltyReward */
    uint8_t ev_bump[RLGPU_CARS], ev_bumped[RLGPU_CARS], ev_demo[RLGPU_CARS], ev_demoed[RLGPU_CARS];
    uint32_t rng_counter;        /* Philox counter for this arena's draws */
    uint32_t manifold_overflow;  /* contacts dropped by a build limit (manifolds, candidates, rows) */
    int32_t episode_steps;       /* steps in the current trajectory (Learner maxEpisodeLength) */
    /* btRSBroadphase cell-list history (btRSBroadphase.cpp:160-176,284-320), per dynamic body (ball, cars
     * 1-4): its home cell + 1 (0 = not placed yet) and its rank in the order the bodies last entered their
     * cells, which is every cell's dynamic-list order (all 0 = creation order, as a fresh arena has) */
    uint16_t bp_cell[RLGPU_CARS + 1];
    uint8_t bp_rank[RLGPU_CARS + 1];
    uint8_t pad1;
} rlgpu_env_extra;

/* Complete serialised arena (the wire format of rlgpu_envset_get/set_arenas). */
typedef struct {
    rlgpu_body ball;
    float ball_vel_impulse_cache[3];
    int32_t ball_sleeping;
    rlgpu_car cars[RLGPU_CARS];
    rlgpu_pad pads[RLGPU_PADS];
    rlgpu_env_extra env;
} rlgpu_arena_state;

typedef struct {
    int32_t num_arenas;
    int32_t tick_skip;       /* LearnerConfig::tickSkip (ExampleMain.cpp:356) */
    int32_t action_delay;    /* LearnerConfig::actionDelay = tickSkip-1 (ExampleMain.cpp:358) */
    uint64_t seed;           /* Philox key: kickoff shuffles and demo respawns */
    int32_t save_rewards;    /* keep per-reward values of player 0 (EnvSetConfig::saveRewards) */
    int32_t max_episode_steps; /* trajectory truncation (Learner.cpp:550,848): 0 = off; ExampleMain
                                  maxEpisodeDuration 300 s -> 300*120/tickSkip = 4500 */
    /* Arena collision meshes (RocketSim::GetArenaCollisionShapes -> Arena::_SetupArenaCollisionShapes,
     * RocketSim.cpp:100-170, Arena.cpp:1015-1058).  mesh_tris == NULL selects the built-in
     * synthetic mesh (include/rlgpu_arena_mesh.h).  Otherwise mesh_ntris triangles of 9 floats
     * (v0, v1, v2 in bullet units, i.e. the .cmf vertices as stored -- see rlgpu_cmf_parse),
     * grouped by collision object in load order: object k owns the next mesh_object_ntris[k]
     * triangles (mesh_object_ntris == NULL: one object).  Host memory, copied at create. */
    const float* mesh_tris;
    int32_t mesh_ntris;
    int32_t mesh_objects;
    const int32_t* mesh_object_ntris;
    /* The EnvCreateFn's rewards and terminal conditions (EnvCreateResult, EnvSet.h:14-24), host
     * memory copied at create.  rewards == NULL: ExampleMain's 13 weighted rewards
     * (src/ExampleMain.cpp:132-177); terminals == NULL: NoTouchCondition(8) + ScoreLimitCondition(3)
     * (:181-187).  An unknown type, a list longer than the RLGPU_MAX_* limits or a bad parameter is
     * rejected by rlgpu_envset_create with RLGPU_ERR_UNSUPPORTED / RLGPU_ERR_INVALID_ARG and a
     * message naming it (rlgpu_last_error) -- a user's own C++ plugin class has no device code here. */
    const rlgpu_reward_spec* rewards;
    int32_t n_rewards;
    const rlgpu_terminal_spec* terminals;
    int32_t n_terminals;
    /* The reference build whose Bullet arithmetic the step follows (RLGPU_ARITH_*, include/rlgpu_arith.h):
     * 0 = RLGPU_ARITH_MSVC_X64, the reference's own build (build.ps1); RLGPU_ARITH_GCC_X64; RLGPU_ARITH_SCALAR.
     * The x86 modes read this host's rsqrtss table at create (RLGPU_ERR_UNSUPPORTED on a host without one). */
    int32_t arith;
    /* global index of arena 0 for the arenas' Philox streams (key seed, counter (arena, draw)): rank r of a
     * data-parallel job passes r x num_arenas, so its arenas are the ones a single device holding every
     * arena would step (0 for one device) */
    int32_t arena_offset;
    /* EnvCreateResult::stateSetter (RLGPU_SS_*): KickoffState (RG/StateSetters/KickoffState.h), or
     * FuzzedKickoffState (FuzzedKickoffState.h:7-26: the kickoff, then every car's position moved by
     * RandFloat(-0.1, 0.1) uu per axis through CarState, RS/Sim/Car/Car.cpp:23-36) -- the skill tracker's
     * (PolicyVersionManager.cpp:24-31).  The fuzz draws are the arena's Philox stream after the kickoff's. */
    int32_t state_setter;
} rlgpu_envset_config;

/* Experience-append destinations of the fused step (Learner.cpp:823-861); any may be NULL. */
typedef struct {
    float* obs;          /* [players][OBS] obs after the step (post-reset): rollout row t+1 */
    uint8_t* masks;      /* [players][ACTIONS] masks after the step (post-reset) */
    float* rewards;      /* [players] */
    int8_t* terminals;   /* [players] trajectory codes 0 / 1 NORMAL / 2 TRUNCATED (incl. max length) */
    float* trunc_obs;    /* [players][OBS] obs before the reset, written where the code is 2 */
} rlgpu_step_outputs;

typedef struct rlgpu_envset rlgpu_envset;

/* Device views of EnvState (EnvSet.h:35-65).  Valid until rlgpu_envset_destroy. */
typedef struct {
    float* obs;              /* [num_players][RLGPU_OBS] */
    uint8_t* action_masks;   /* [num_players][RLGPU_ACTIONS] */
    float* rewards;          /* [num_players] */
    uint8_t* terminals;      /* [num_arenas]: 0, 1 NORMAL, 2 TRUNCATED */
    float* last_rewards;     /* [num_arenas][num_rewards]: each reward's value for player 0 (if save_rewards;
                                EnvState::lastRewards, EnvSet.cpp:224-242) */
    float* trunc_obs;        /* [num_players][RLGPU_OBS] pre-reset obs of truncated arenas */
    int32_t num_players;
    int32_t num_arenas;
    int32_t num_rewards;     /* length of the reward list */
    int32_t* arena_player_start; /* [num_arenas] EnvState::arenaPlayerStartIdx (4 * arena, 2v2) */
} rlgpu_envset_buffers;

/* Creates the set, resets every arena to a random kickoff (EnvSet.cpp:105-110). */
int rlgpu_envset_create(const rlgpu_envset_config* cfg, rlgpu_envset** out);
int rlgpu_envset_destroy(rlgpu_envset* env);
int rlgpu_envset_buffers_get(rlgpu_envset* env, rlgpu_envset_buffers* out);

/* EnvSet::Reset(): reset arenas whose terminal flag is set, rebuild their obs/masks. */
int rlgpu_envset_reset(rlgpu_envset* env, void* stream);
/* EnvSet::ResetArena(i) for every i with d_mask[i] != 0 (d_mask == NULL: all arenas). */
int rlgpu_envset_reset_arenas(rlgpu_envset* env, const uint8_t* d_mask, void* stream);

/* Two-half step with the reference's action delay. */
int rlgpu_envset_step_first_half(rlgpu_envset* env, void* stream);
int rlgpu_envset_step_second_half(rlgpu_envset* env, const int32_t* d_actions, void* stream);
/* Fused: first half + second half + (optional) reset of terminated arenas in one launch, plus
 * the experience append into `out` (may be NULL).  buffers.trunc_obs also receives the
 * pre-reset rows of trajectories ending TRUNCATED.  Requires action_delay > 0. */
int rlgpu_envset_step(rlgpu_envset* env, const int32_t* d_actions, int32_t reset_terminated,
                      const rlgpu_step_outputs* out, void* stream);
/* The fused step of the arenas [first, first + count) only (first a multiple of 4): d_actions holds those
 * arenas' players' actions and `out` those players' rows.  Ranges of one set with disjoint arenas may run
 * concurrently on different streams -- the C++ Learner's collection runs arena groups on their own streams,
 * so one group's launch tail (a launch lasts as long as its slowest workgroup) overlaps the other groups'
 * work.  Every arena's results are the full-set step's bit for bit.  ExampleMain's StepCallback cadence
 * (every 4th step for the player metrics) advances at the range that starts at arena 0.  Not with the
 * per-phase profile (rlgpu_envset_set_profile). */
int rlgpu_envset_step_range(rlgpu_envset* env, int32_t first, int32_t count, const int32_t* d_actions,
                            int32_t reset_terminated, const rlgpu_step_outputs* out, void* stream);
int rlgpu_envset_sync(rlgpu_envset* env, void* stream);
/* Output-only rows (default off): a fused step given `out` rows for obs / masks / truncation obs writes those
 * rows only there, not also into the set's own buffers (rlgpu_envset_buffers obs / masks / trunc_obs), which
 * then keep the last step that had no such output.  One copy of the 3 KB of rows per env step instead of two
 * (obs 2,672 B + masks 360 B per arena); the C++ Learner turns it on for its own set, whose rollout rows are the
 * only ones it reads.  A step without `out` (or with a NULL row pointer) writes the set's buffers as always. */
int rlgpu_envset_set_output_only(rlgpu_envset* env, int32_t enable);

/* Wire-format state transfer (host <-> device), for GameState snapshots, tests and replay. */
int rlgpu_envset_get_arenas(rlgpu_envset* env, int32_t first, int32_t count, rlgpu_arena_state* h_out);
int rlgpu_envset_set_arenas(rlgpu_envset* env, int32_t first, int32_t count, const rlgpu_arena_state* h_in);
/* Rebuild obs/masks of all arenas from the current state (no physics). */
int rlgpu_envset_build_obs(rlgpu_envset* env, void* stream);

/* Diagnostics: when d_counters (uint64, device, 64 + 24 x workgroups + arenas) is non-NULL, every launch
 * adds the shader cycles thread 0 of each workgroup spends per phase (0-10 tick phases, 11 load/halves
 * prelude, 12 builders, 13 obs rows, 14 resets, 15 store, 16-22 solver sub-phases, 18 the deferred
 * penetration queries) to d_counters[phase] (all workgroups) and to d_counters[64 + 24 * workgroup + phase];
 * slot 23 of a workgroup and d_counters[64 + 24 * workgroups + arena] count penetration-solver calls.
 * NULL disables (the default).  capacity: entries of d_counters (>= 64 + 24 * workgroups + arenas, else
 * RLGPU_ERR_INVALID_ARG). */
int rlgpu_envset_set_profile(rlgpu_envset* env, unsigned long long* d_counters, int64_t capacity);

/* ExampleMain's StepCallback metrics on the device.  Replaces the StepCallbackFn that
 * Learner::Start calls after every StepSecondHalf (GL/public/GigaLearnCPP/Learner.h:11,
 * Learner.cpp:796-797) with the callback src/ExampleMain.cpp:233-283 registers: on every 4th call
 * (its stepCounter) each player of each GameState adds "Player/In Air Ratio", "Ball Touch Ratio",
 * "Demoed Ratio", "Speed", "Speed Towards Ball", "Boost" and, when it touched the ball this step,
 * "Touch Height"; on every call each state that scored adds "Game/Goal Speed" -- Report::AddAvg's
 * (total, count) in fp64 (Report.h:11-45).  When enabled, every launch that runs the builders (fused
 * step, second half) is one callback call: the kernel adds the pre-reset GameState's values to
 * per-arena fp64 slots (RLGPU_STEP_METRIC_SLOTS per arena: metric x 4 + player for the 7 player
 * metrics, then goal-speed total, goal count, player-pass count). */
enum {
    RLGPU_SM_IN_AIR = 0,
    RLGPU_SM_BALL_TOUCH = 1,
    RLGPU_SM_DEMOED = 2,
    RLGPU_SM_SPEED = 3,
    RLGPU_SM_SPEED_TO_BALL = 4,
    RLGPU_SM_BOOST = 5,
    RLGPU_SM_TOUCH_HEIGHT = 6,
    RLGPU_SM_GOAL_SPEED = 7,
    RLGPU_NUM_STEP_METRICS = 8,
    RLGPU_SM_SLOT_GOAL_SPEED = 28, /* per-arena slots after the 7 x 4 player slots */
    RLGPU_SM_SLOT_GOALS = 29,
    RLGPU_SM_SLOT_PASSES = 30,
    RLGPU_STEP_METRIC_SLOTS = 32
};
/* Report key of metric i ("Player/In Air Ratio", ...), NULL when out of range. */
const char* rlgpu_step_metric_name(int32_t i);
/* enable != 0: allocate and zero the per-arena slots and the call counter; 0: free them. */
int rlgpu_envset_enable_step_metrics(rlgpu_envset* env, int32_t enable);
/* Report::Avg totals and counts of the RLGPU_NUM_STEP_METRICS metrics since the last reset: the
 * per-arena slots summed in fp64 in arena order (host), after synchronising `stream`.  reset != 0
 * zeroes the slots afterwards (Report cleared at each metrics report).  Either output may be NULL. */
int rlgpu_envset_step_metrics(rlgpu_envset* env, double* h_total, uint64_t* h_count, int32_t reset, void* stream);
/* The raw per-arena slots [num_arenas][RLGPU_STEP_METRIC_SLOTS] (tests, custom reductions). */
int rlgpu_envset_step_metric_slots(rlgpu_envset* env, double* h_out, void* stream);

/* The registry lists ExampleMain's EnvCreateFn builds (src/ExampleMain.cpp:132-187), the defaults of
 * NULL config lists: writes up to RLGPU_MAX_REWARDS / RLGPU_MAX_TERMINALS entries (any output may be
 * NULL). */
int rlgpu_envset_default_plugins(rlgpu_reward_spec* rewards, int32_t* n_rewards, rlgpu_terminal_spec* terminals,
                                 int32_t* n_terminals);

/* Static sizes for binding checks. */
int rlgpu_arena_state_size(void);

#ifdef __cplusplus
}
#endif
#endif
