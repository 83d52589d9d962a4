// gamestate.cpp -- RLGC::GameState records from arena records (include/rlgpu_gamestate.h).  Host code (g++).
//
// GameState::UpdateFromArena (RG/Gamestates/GameState.cpp:60-131) and Player::UpdateFromCar
// (RG/Gamestates/Player.cpp:8-25) over the wire-format record (include/rlgpu_env.h): Ball::GetState /
// Car::GetState convert Bullet units back to uu (x 50, BulletLink.h:11-15; angular velocity unchanged,
// RS/Sim/Car/Car.cpp:10-36, RS/Sim/Ball/Ball.cpp:12-40); the rotation matrix is RocketSim's RotMat (forward,
// right, up = the basis columns).  The kernels' builders read the same fields (env_builders.hpp view_player).
#include <cstring>

#include "../../include/rlgpu_gamestate.h"
#include "../csrc/common.hpp"
#include "../csrc/mesh.hpp"

namespace rlgpu {
namespace {
constexpr float kBT2UU = 50.f;

void rot_mat(const float* b, float* out) {  // btMatrix3x3 rows -> RotMat (forward, right, up) = columns
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) out[3 * c + r] = b[3 * r + c];
}
}  // namespace

void gamestates_from_arenas(const rlgpu_arena_state* rec, int count, int tick_skip, rlgpu_gamestate* out) {
    int map[RLGPU_PADS];
    boost_pad_index_map(map);
    for (int a = 0; a < count; a++) {
        const rlgpu_arena_state& s = rec[a];
        rlgpu_gamestate& g = out[a];
        std::memset(&g, 0, sizeof g);
        const uint64_t tick = (uint64_t)s.env.tick_count;
        // deltaTime = ticks since the previous update / 120 (GameState.cpp:71-74): after a step's builders
        // lastTickCount == tickCount, so the step's own span is the set's tickSkip
        g.delta_time = (float)tick_skip * (1.0f / 120.0f);
        g.last_tick_count = tick;
        for (int i = 0; i < 3; i++) {
            g.ball.pos[i] = s.ball.pos[i] * kBT2UU;
            g.ball.vel[i] = s.ball.vel[i] * kBT2UU;
            g.ball.ang_vel[i] = s.ball.angvel[i];
        }
        rot_mat(s.ball.rot, g.ball.rot);
        g.last_touch_car_id = -1;
        for (int i = 0; i < RLGPU_CARS; i++) {
            const rlgpu_car& c = s.cars[i];
            rlgpu_player_state& p = g.players[i];
            rlgpu_car_state& cs = p.car;
            for (int k = 0; k < 3; k++) {
                cs.pos[k] = c.body.pos[k] * kBT2UU;
                cs.vel[k] = c.body.vel[k] * kBT2UU;
                cs.ang_vel[k] = c.body.angvel[k];
                cs.flip_rel_torque[k] = c.flip_rel_torque[k];
                cs.world_contact_normal[k] = c.world_contact_normal[k];
                cs.ball_hit_relative_pos_on_ball[k] = c.ball_hit_rel_pos[k];
                cs.ball_hit_ball_pos[k] = c.ball_hit_ball_pos[k];
                cs.ball_hit_extra_hit_vel[k] = c.ball_hit_extra_vel[k];
            }
            rot_mat(c.body.rot, cs.rot);
            cs.is_on_ground = c.is_on_ground;
            cs.has_jumped = c.has_jumped;
            cs.has_double_jumped = c.has_double_jumped;
            cs.has_flipped = c.has_flipped;
            cs.is_flipping = c.is_flipping;
            cs.is_jumping = c.is_jumping;
            cs.is_supersonic = c.is_supersonic;
            cs.is_auto_flipping = c.is_auto_flipping;
            cs.is_demoed = c.is_demoed;
            cs.world_contact_has_contact = c.world_contact;
            cs.ball_hit_is_valid = c.ball_hit_valid;
            std::memcpy(cs.wheels_with_contact, c.wheel_contact, sizeof cs.wheels_with_contact);
            cs.jump_time = c.jump_time;
            cs.flip_time = c.flip_time;
            cs.air_time = c.air_time;
            cs.air_time_since_jump = c.air_time_since_jump;
            cs.boost = c.boost;
            cs.time_spent_boosting = c.time_spent_boosting;
            cs.supersonic_time = c.supersonic_time;
            cs.handbrake_val = c.handbrake_val;
            cs.auto_flip_timer = c.auto_flip_timer;
            cs.auto_flip_torque_scale = c.auto_flip_torque_scale;
            cs.demo_respawn_timer = c.demo_respawn_timer;
            cs.car_contact_other_car_id = c.car_contact_other_id;
            cs.car_contact_cooldown_timer = c.car_contact_cooldown;
            cs.ball_hit_tick_count_when_hit = c.ball_hit_tick;
            cs.ball_hit_tick_count_when_extra_impulse_applied = c.ball_hit_extra_tick;
            std::memcpy(cs.last_controls, c.last_controls, sizeof cs.last_controls);
            p.index = i;
            p.car_id = (uint32_t)(i + 1);  // Arena::AddCar ids from 1, cars in creation order
            p.team = i & 1;
            p.events[5] = s.env.ev_bump[i];  // PlayerEventState: bump, bumped, demo, demoed
            p.events[6] = s.env.ev_bumped[i];
            p.events[7] = s.env.ev_demo[i];
            p.events[8] = s.env.ev_demoed[i];
            if (c.ball_hit_valid) {  // Player.cpp:17-22
                p.ball_touched_step = (uint64_t)c.ball_hit_tick >= tick - (uint64_t)tick_skip;
                p.ball_touched_tick = (uint64_t)c.ball_hit_tick == tick - 1;
            }
            if (p.ball_touched_step) g.last_touch_car_id = (int32_t)p.car_id;
            std::memcpy(p.prev_action, s.env.prev_action[i], sizeof p.prev_action);
        }
        for (int i = 0; i < RLGPU_PADS; i++) {  // GameState.cpp:109-126
            const rlgpu_pad& pd = s.pads[map[i]];
            const rlgpu_pad& pi = s.pads[map[RLGPU_PADS - i - 1]];
            g.boost_pads[i] = pd.is_active;
            g.boost_pads_inv[i] = pi.is_active;
            g.boost_pad_timers[i] = pd.cooldown;
            g.boost_pad_timers_inv[i] = pi.cooldown;
        }
        // Arena::IsBallScored (SOCCAR): |ball y| beyond the goal line plus the ball radius
        g.goal_scored = (s.ball.pos[1] * kBT2UU > 5124.25f + 91.25f) || (s.ball.pos[1] * kBT2UU < -(5124.25f + 91.25f));
    }
}

}  // namespace rlgpu

extern "C" int rlgpu_gamestates_from_arenas(const rlgpu_arena_state* h_arenas, int32_t count, int32_t tick_skip,
                                            rlgpu_gamestate* h_out) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE((h_arenas && h_out) || count == 0, "rlgpu_gamestates_from_arenas: null argument");
        RLGPU_REQUIRE(count >= 0 && tick_skip > 0, "rlgpu_gamestates_from_arenas: bad count or tick_skip");
        rlgpu::gamestates_from_arenas(h_arenas, count, tick_skip, h_out);
    });
}

extern "C" int rlgpu_gamestate_size(void) { return (int)sizeof(rlgpu_gamestate); }
