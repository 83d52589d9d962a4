/*
 * rlgpu_gamestate.h -- host RLGC::GameState records of an env set's arenas, for everything the reference
 * runs on GameStates outside the device registry: a StepCallbackFn (GigaLearnCPP Learner.h:11, called with
 * the states after every StepSecondHalf, Learner.cpp:796-797), render / metrics senders, and user reward /
 * terminal plugins the device has no code for (the host fallback of host/rlgc_env.hpp).
 *
 * One record restates GameState::UpdateFromArena (RG/Gamestates/GameState.cpp:60-131) and
 * Player::UpdateFromCar (RG/Gamestates/Player.cpp:8-25) on the arena record: RocketSim's GetState units
 * (uu, uu/s, rad/s; bullet values x 50 where RocketSim converts), players in car creation order (ids 1-4,
 * blue / orange alternating), ballTouchedStep = the hit tick >= tickCount - tickSkip, the boost pads through
 * CommonValues::BOOST_LOCATIONS' index map with the inverted arrays (GameState.cpp:98-126; the reference's
 * GetBoostPadTimers(inverted) returns the opposite array, GameState.h:60 -- the C++ facade keeps that).
 * lastTouchCarID here is this step's (-1 when nobody touched the ball); the facade carries it over steps as
 * the reference's GameState member does.
 */
#ifndef RLGPU_GAMESTATE_H
#define RLGPU_GAMESTATE_H

#include <stdint.h>
#include "rlgpu_env.h"

#ifdef __cplusplus
extern "C" {
#endif

/* RocketSim CarState (RS/Sim/Car/Car.h:17-100) */
typedef struct {
    float pos[3];           /* uu */
    float rot[9];           /* RotMat rows as RocketSim stores them: forward, right, up (columns of the basis) */
    float vel[3];           /* uu/s */
    float ang_vel[3];       /* rad/s */
    uint8_t is_on_ground, has_jumped, has_double_jumped, has_flipped;
    uint8_t is_flipping, is_jumping, is_supersonic, is_auto_flipping;
    uint8_t is_demoed, world_contact_has_contact, ball_hit_is_valid, pad0;
    uint8_t wheels_with_contact[4]; /* front left, front right, back left, back right */
    float flip_rel_torque[3];
    float jump_time, flip_time, air_time, air_time_since_jump, boost, time_spent_boosting, supersonic_time;
    float handbrake_val, auto_flip_timer, auto_flip_torque_scale, demo_respawn_timer;
    float world_contact_normal[3];
    uint32_t car_contact_other_car_id;
    float car_contact_cooldown_timer;
    float ball_hit_relative_pos_on_ball[3], ball_hit_ball_pos[3], ball_hit_extra_hit_vel[3];
    int64_t ball_hit_tick_count_when_hit, ball_hit_tick_count_when_extra_impulse_applied;
    float last_controls[8];  /* throttle, steer, pitch, yaw, roll, jump, boost, handbrake */
} rlgpu_car_state;

/* RLGC::Player (RG/Gamestates/Player.h) */
typedef struct {
    rlgpu_car_state car;
    int32_t index;    /* in the GameState's players */
    uint32_t car_id;  /* Car::id */
    int32_t team;     /* 0 blue, 1 orange */
    /* PlayerEventState: goal, save, assist, shot, shotPass, bump, bumped, demo, demoed (the arena's event
     * tracker sets bump / bumped / demo / demoed, EnvSet.cpp:31-42) */
    uint8_t events[9];
    uint8_t ball_touched_step, ball_touched_tick, pad0;
    float prev_action[8];
} rlgpu_player_state;

/* RLGC::GameState (RG/Gamestates/GameState.h) */
typedef struct {
    float delta_time;
    int32_t goal_scored;
    int32_t last_touch_car_id;  /* this step's (see above) */
    uint64_t last_tick_count;
    struct {
        float pos[3], rot[9], vel[3], ang_vel[3];
    } ball;                     /* BallState, uu */
    rlgpu_player_state players[RLGPU_CARS];
    uint8_t boost_pads[RLGPU_PADS], boost_pads_inv[RLGPU_PADS];
    float boost_pad_timers[RLGPU_PADS], boost_pad_timers_inv[RLGPU_PADS];
} rlgpu_gamestate;

/* The GameStates of arenas [first, first + count) as they are now (after the last step's builders: the
 * state the reference hands its StepCallback and its reward plugins), after synchronising `stream`; the
 * set's tick_skip is ballTouchedStep's window. */
int rlgpu_envset_download_gamestates(rlgpu_envset* env, int32_t first, int32_t count, rlgpu_gamestate* h_out,
                                     void* stream);

/* The same restatement on arena records the caller holds (rlgpu_envset_get_arenas, the wire format). */
int rlgpu_gamestates_from_arenas(const rlgpu_arena_state* h_arenas, int32_t count, int32_t tick_skip,
                                 rlgpu_gamestate* h_out);

/* Per-player, per-reward values of the last builders launch (the values the weighted sum adds, before the
 * weights): enable != 0 makes every later step write them ([num_players][num_rewards] floats, device);
 * rlgpu_envset_reward_values returns the buffer (NULL while disabled).  The host fallback of unknown reward
 * plugins reads them to rebuild the reference's weighted sum in list order. */
int rlgpu_envset_enable_reward_values(rlgpu_envset* env, int32_t enable);
float* rlgpu_envset_reward_values(rlgpu_envset* env);

/* sizeof(rlgpu_gamestate), for binding checks */
int rlgpu_gamestate_size(void);

#ifdef __cplusplus
}
#endif
#endif
