// arena_wire.cpp -- RocketSim's arena byte stream (include/rlgpu_arena_wire.h) for the arena records
// of include/rlgpu_env.h.  Host code (g++).
//
// One visitor per section walks the reference's field list in order; the writer (Out) emits each
// field and the reader (In) parses it back into the record, so the two directions share one list.
// Field lists (RS/ = GigaLearnCPP/RLGymCPP/RocketSim/src/):
//   stream primitives   RS/DataStream/DataStreamOut.h:15-44, DataStreamIn.h:49-84
//   Arena               RS/Sim/Arena/Arena.cpp:572-599 (write), :601-671 and :703-714 (read)
//   ArenaConfig         RS/Sim/Arena/ArenaConfig/ArenaConfig.cpp:5-35, ArenaConfig.h:18-53
//   Car                 RS/Sim/Car/Car.cpp:299-328, Car.h:117-123, CarControls.h:7-38,
//                       CarConfig/CarConfig.h:18-38, CarConfig.cpp:20-81 (Octane)
//   BallHitInfo         RS/Sim/BallHitInfo/BallHitInfo.cpp:5-17, BallHitInfo.h:9-30
//   BoostPadState       RS/Sim/BoostPad/BoostPad.cpp:21-31, BoostPad.h:23-34
//   BallState           RS/Sim/Ball/Ball.cpp:19-49, Ball.h:17-46
//   MutatorConfig       RS/Sim/MutatorConfig/MutatorConfig.cpp:5-49, MutatorConfig.h:16-83, RLConst.h
#include <cstring>
#include <string>

#include "../../include/rlgpu_arena_wire.h"
#include "../csrc/common.hpp"

namespace {

using rlgpu::Error;

constexpr float kBtToUu = 50.f, kUuToBt = 1.f / 50.f;  // RS/BulletLink.h:12-15
constexpr float kBoostMax = 100.f, kCarMassBt = 180.f;  // RLConst.h:22,47

struct V3 {
    float x, y, z;
};

// ------------------------------------------------------------------ writer
struct Out {
    uint8_t* p;  // null: count the bytes only
    uint64_t cap;
    uint64_t n = 0;

    void bytes(const void* src, uint64_t k) {
        if (p && n + k <= cap) std::memcpy(p + n, src, k);
        n += k;
    }
    template <class T>
    void raw(T v) {
        bytes(&v, sizeof v);
    }
    void vec4(float x, float y, float z) {
        const float q[4] = {x, y, z, 0.f};  // Vec's 4th lane (MathTypes.h:7-16)
        bytes(q, sizeof q);
    }
    void count(uint32_t k) { raw(k); }
    void count16(uint16_t k) { raw(k); }
    void fixed_u8(uint8_t v, const char*) { raw(v); }
    void fixed_u32(uint32_t v, const char*) { raw(v); }
    void fixed_f32(float v, const char*) { raw(v); }
    void fixed_vec(V3 v, const char*) { vec4(v.x, v.y, v.z); }
    void skip_u32(uint32_t v) { raw(v); }
    void skip_f32(float v) { raw(v); }
    void f(const float& v) { raw(v); }
    void b(const uint8_t& v) { raw<uint8_t>(v != 0); }
    void button(const float& v) { raw<uint8_t>(v != 0.f); }
    void u32(const uint32_t& v) { raw(v); }
    void tick(const int64_t& v) { raw((uint64_t)v); }
    void vec(const float* v) { vec4(v[0], v[1], v[2]); }
    void vec_uu(const float* v) { vec4(v[0] * kBtToUu, v[1] * kBtToUu, v[2] * kBtToUu); }  // GetState
    void rot(const float* r) {  // RotMat forward, right, up: the columns of the row-major basis
        for (int c = 0; c < 3; c++) vec4(r[c], r[3 + c], r[6 + c]);
    }
    void controls(const float* c) {  // a CarControls struct: 5 floats, jump, boost, handbrake, 1 pad byte
        for (int k = 0; k < 5; k++) raw(c[k]);
        for (int k = 5; k < 8; k++) raw<uint8_t>(c[k] != 0.f);
        raw<uint8_t>(0);
    }
    int car(int k) {  // team and id of the k-th car: ids 1..4 in creation order (Arena.cpp:65)
        raw<uint8_t>(k & 1);
        raw<uint32_t>(k + 1);
        return k;
    }
    bool hit(const uint8_t& valid) {
        b(valid);
        return valid != 0;
    }
};

// ------------------------------------------------------------------ reader
struct In {
    const uint8_t* p;
    uint64_t n;
    uint64_t i = 0;
    unsigned seen = 0;

    void bytes(void* dst, uint64_t k) {
        if (k > n - i)
            throw Error(RLGPU_ERR_INVALID_ARG, "arena stream truncated: " + std::to_string(k) + " bytes wanted at byte " +
                                                   std::to_string(i) + " of " + std::to_string(n));
        std::memcpy(dst, p + i, k);
        i += k;
    }
    template <class T>
    T raw() {
        T v;
        bytes(&v, sizeof v);
        return v;
    }
    [[noreturn]] void unsupported(const char* what) {
        throw Error(RLGPU_ERR_UNSUPPORTED, std::string("arena stream: ") + what +
                                               " differs from what this engine simulates (SOCCAR, 120 Hz, 2v2 "
                                               "Octanes, default ArenaConfig / MutatorConfig)");
    }
    void vec4(float* q) { bytes(q, 4 * sizeof(float)); }
    // DataStreamIn::ReadMultipleFromList: a field-count mismatch fails the read (DataStreamIn.h:73-77)
    void count(uint32_t k) {
        const uint32_t got = raw<uint32_t>();
        if (got != k)
            throw Error(RLGPU_ERR_INVALID_ARG, "arena stream: prop count mismatch at byte " + std::to_string(i - 4) +
                                                   ", expected " + std::to_string(k) + " but have " + std::to_string(got));
    }
    void count16(uint16_t k) {  // MutatorConfig's field count (MutatorConfig.cpp:41-46)
        const uint16_t got = raw<uint16_t>();
        if (got != k)
            throw Error(RLGPU_ERR_INVALID_ARG, "arena stream: MutatorConfig of " + std::to_string(got) +
                                                   " fields, expected " + std::to_string(k) +
                                                   " (another RocketSim version)");
    }
    void fixed_u8(uint8_t v, const char* w) {
        if (raw<uint8_t>() != v) unsupported(w);
    }
    void fixed_u32(uint32_t v, const char* w) {
        if (raw<uint32_t>() != v) unsupported(w);
    }
    void fixed_f32(float v, const char* w) {
        if (raw<float>() != v) unsupported(w);
    }
    void fixed_vec(V3 v, const char* w) {
        float q[4];
        vec4(q);
        if (q[0] != v.x || q[1] != v.y || q[2] != v.z) unsupported(w);
    }
    void skip_u32(uint32_t) { raw<uint32_t>(); }
    void skip_f32(float) { raw<float>(); }
    void f(float& v) { v = raw<float>(); }
    void b(uint8_t& v) { v = raw<uint8_t>() != 0; }
    void button(float& v) { v = raw<uint8_t>() != 0 ? 1.f : 0.f; }
    void u32(uint32_t& v) { v = raw<uint32_t>(); }
    void tick(int64_t& v) { v = (int64_t)raw<uint64_t>(); }
    void vec(float* v) {
        float q[4];
        vec4(q);
        v[0] = q[0];
        v[1] = q[1];
        v[2] = q[2];
    }
    void vec_uu(float* v) {  // SetState: * UU_TO_BT
        float q[4];
        vec4(q);
        for (int k = 0; k < 3; k++) v[k] = q[k] * kUuToBt;
    }
    void rot(float* r) {
        for (int c = 0; c < 3; c++) {
            float q[4];
            vec4(q);
            r[c] = q[0];
            r[3 + c] = q[1];
            r[6 + c] = q[2];
        }
    }
    void controls(float* c) {
        for (int k = 0; k < 5; k++) c[k] = raw<float>();
        for (int k = 5; k < 8; k++) c[k] = raw<uint8_t>() != 0 ? 1.f : 0.f;
        raw<uint8_t>();
    }
    int car(int) {  // DeserializeNew keys the cars by id (Arena.cpp:618-640)
        const uint8_t team = raw<uint8_t>();
        const uint32_t id = raw<uint32_t>();
        if (id < 1 || id > RLGPU_CARS || team != ((id - 1) & 1) || ((seen >> (id - 1)) & 1))
            unsupported("the car ids / teams (ids 1..4 once each, team = (id - 1) & 1)");
        seen |= 1u << (id - 1);
        return (int)id - 1;
    }
    bool hit(uint8_t& valid) {
        b(valid);
        return valid != 0;
    }
};

// ------------------------------------------------------------------ the field lists
template <class S>
void arena_config_fields(S& s) {  // ARENA_CONFIG_SERIALIZATION_FIELDS (ArenaConfig.h:52-53), then useCustomBoostPads
    const char* w = "ArenaConfig";
    s.count(5);
    s.fixed_vec(V3{-4500.f, -6000.f, 0.f}, w);  // minPos
    s.fixed_vec(V3{4500.f, 6000.f, 2500.f}, w);  // maxPos
    s.fixed_f32(370.f, w);                        // maxAABBLen
    s.fixed_u8(1, w);                             // noBallRot
    s.fixed_u8(1, w);                             // useCustomBroadphase
    s.fixed_u8(0, "useCustomBoostPads");
}

template <class S>
void car_config_fields(S& s) {  // CAR_CONFIG_SERIALIZATION_FIELDS (CarConfig.h:35-38) of CAR_CONFIG_OCTANE
    const char* w = "CarConfig (Octane)";
    s.count(9);
    s.fixed_f32(0.5f, w);                               // dodgeDeadzone
    s.fixed_vec(V3{(float)13.87566, 0.f, 20.755f}, w);  // hitboxPosOffset
    s.fixed_vec(V3{120.507f, 86.6994f, 38.6591f}, w);   // hitboxSize
    s.fixed_vec(V3{51.25f, 25.90f, 20.755f}, w);        // frontWheels.connectionPointOffset
    s.fixed_f32(38.755f, w);                            // frontWheels.suspensionRestLength
    s.fixed_f32(12.50f, w);                             // frontWheels.wheelRadius
    s.fixed_vec(V3{-33.75f, 29.50f, 20.755f}, w);       // backWheels.connectionPointOffset
    s.fixed_f32(37.055f, w);                            // backWheels.suspensionRestLength
    s.fixed_f32(15.00f, w);                             // backWheels.wheelRadius
}

template <class S, class C>
void car_controls_fields(S& s, C& c) {  // CAR_CONTROLS_SERIALIZATION_FIELDS (CarControls.h:35-38)
    s.count(8);
    for (int k = 0; k < 5; k++) s.f(c.controls[k]);  // throttle, steer, pitch, yaw, roll
    s.button(c.controls[6]);                          // boost
    s.button(c.controls[5]);                          // jump
    s.button(c.controls[7]);                          // handbrake
}

template <class S, class C>
void ball_hit_fields(S& s, C& c) {  // BallHitInfo::Serialize: isValid, then the fields when valid
    if (!s.hit(c.ball_hit_valid)) return;
    s.count(5);
    s.vec(c.ball_hit_rel_pos);
    s.vec(c.ball_hit_ball_pos);
    s.vec(c.ball_hit_extra_vel);
    s.tick(c.ball_hit_tick);
    s.tick(c.ball_hit_extra_tick);
}

template <class S, class C>
void car_state_fields(S& s, C& c) {  // CARSTATE_SERIALIZATION_FIELDS (Car.h:117-123)
    s.count(28);
    s.vec_uu(c.body.pos);
    s.rot(c.body.rot);
    s.vec_uu(c.body.vel);
    s.vec(c.body.angvel);
    s.b(c.is_on_ground);
    s.b(c.has_jumped);
    s.b(c.has_double_jumped);
    s.b(c.has_flipped);
    s.vec(c.flip_rel_torque);
    s.f(c.jump_time);
    s.b(c.is_flipping);
    s.f(c.flip_time);
    s.b(c.is_jumping);
    s.f(c.air_time_since_jump);
    s.f(c.boost);
    s.f(c.time_spent_boosting);
    s.f(c.supersonic_time);
    s.f(c.handbrake_val);
    s.b(c.is_auto_flipping);
    s.f(c.auto_flip_timer);
    s.f(c.auto_flip_torque_scale);
    s.b(c.is_demoed);
    s.f(c.demo_respawn_timer);
    s.controls(c.last_controls);
    s.b(c.world_contact);
    s.vec(c.world_contact_normal);
    s.u32(c.car_contact_other_id);
    s.f(c.car_contact_cooldown);
}

template <class S, class P>
void pad_fields(S& s, P& p) {  // BOOSTPAD_SERIALIZATION_FIELDS (BoostPad.h:33-34)
    s.count(3);
    s.b(p.is_active);
    s.f(p.cooldown);
    s.u32(p.prev_locked_car_id);
}

template <class S, class A>
void ball_fields(S& s, A& a) {  // BALLSTATE_SERIALIZATION_FIELDS (Ball.h:44-46)
    s.count(7);
    s.vec_uu(a.ball.pos);
    s.rot(a.ball.rot);
    s.vec_uu(a.ball.vel);
    s.vec(a.ball.angvel);
    s.skip_f32(0.f);     // hsInfo.yTargetDir: HeatseekerInfo (Ball.h:23-30) is unused in SOCCAR
    s.skip_f32(2900.f);  // hsInfo.curTargetSpeed = Heatseeker::INITIAL_TARGET_SPEED (RLConst.h:153)
    s.skip_f32(0.f);     // hsInfo.timeSinceHit
}

template <class S>
void mutator_fields(S& s) {  // MutatorConfig::Serialize: u16 field count, then MUTATOR_CONFIG_SERIALIZATION_FIELDS
    const char* w = "MutatorConfig (SOCCAR defaults)";
    s.count16(27);
    s.count(27);
    s.fixed_vec(V3{0.f, 0.f, -650.f}, w);  // gravity = (0, 0, GRAVITY_Z)
    s.fixed_f32(kCarMassBt, w);            // carMass
    s.fixed_f32(0.3f, w);                  // carWorldFriction
    s.fixed_f32(0.3f, w);                  // carWorldRestitution
    s.fixed_f32(kCarMassBt / 6.f, w);      // ballMass = BALL_MASS_BT
    s.fixed_f32(6000.f, w);                // ballMaxSpeed
    s.fixed_f32(0.03f, w);                 // ballDrag
    s.fixed_f32(0.35f, w);                 // ballWorldFriction
    s.fixed_f32(0.6f, w);                  // ballWorldRestitution
    s.fixed_f32(4375.f / 3.f, w);          // jumpAccel
    s.fixed_f32(875.f / 3.f, w);           // jumpImmediateForce
    s.fixed_f32(2975 / 3.f, w);            // boostAccelGround
    s.fixed_f32(3175 / 3.f, w);            // boostAccelAir
    s.fixed_f32(kBoostMax / 3, w);         // boostUsedPerSecond
    s.fixed_f32(3.f, w);                   // respawnDelay = DEMO_RESPAWN_TIME
    s.fixed_f32(kBoostMax / 3, w);         // carSpawnBoostAmount
    s.fixed_f32(0.25f, w);                 // bumpCooldownTime
    s.fixed_f32(10.f, w);                  // boostPadCooldown_Big
    s.fixed_f32(4.f, w);                   // boostPadCooldown_Small
    s.fixed_f32(1.f, w);                   // ballHitExtraForceScale
    s.fixed_f32(1.f, w);                   // bumpForceScale
    s.fixed_f32(91.25f, w);                // ballRadius = BALL_COLLISION_RADIUS_SOCCAR
    s.fixed_u8(0, w);                      // unlimitedFlips
    s.fixed_u8(0, w);                      // unlimitedDoubleJumps
    s.fixed_u8(0, w);                      // demoMode = DemoMode::NORMAL
    s.fixed_u8(0, w);                      // enableTeamDemos
    s.fixed_f32(5124.25f, w);              // goalBaseThresholdY
}

template <class S, class A>
void arena_fields(S& s, A& a) {
    s.count(4);  // Arena::Serialize: WriteMultiple(gameMode, tickTime, tickCount, _lastCarID)
    s.fixed_u8(0, "gameMode (SOCCAR)");
    s.fixed_f32(1.f / 120.f, "tickTime (120 Hz)");
    s.tick(a.env.tick_count);
    s.skip_u32(RLGPU_CARS);  // _lastCarID: the cars are ids 1..4
    arena_config_fields(s);
    s.fixed_u32(RLGPU_CARS, "the car count (2v2)");
    for (int k = 0; k < RLGPU_CARS; k++) {
        auto& c = a.cars[s.car(k)];
        car_controls_fields(s, c);
        car_config_fields(s);
        ball_hit_fields(s, c);
        car_state_fields(s, c);
    }
    s.fixed_u32(RLGPU_PADS, "the boost pad count");
    for (auto& p : a.pads) pad_fields(s, p);
    ball_fields(s, a);
    mutator_fields(s);
}

// DeserializeNew builds a new arena: what the stream does not carry starts as a new car / ball has
// it (CarState() and BallHitInfo() defaults, Car / Ball::SetState's cleared impulse caches, new
// wheels: Car.h:17-100, BallHitInfo.h:11-22, Car.cpp:23-36, Ball.cpp:35-49, Arena.cpp:703-714) and
// a new broadphase's cell lists
void fresh_engine_state(rlgpu_arena_state& s) {
    for (rlgpu_car& c : s.cars) {
        c.is_supersonic = 0;
        c.air_time = 0.f;
        std::memset(c.wheel_contact, 0, sizeof c.wheel_contact);
        std::memset(c.vel_impulse_cache, 0, sizeof c.vel_impulse_cache);
        std::memset(c.wheel_steer, 0, sizeof c.wheel_steer);
        std::memset(c.wheel_engine_force, 0, sizeof c.wheel_engine_force);
        std::memset(c.wheel_brake, 0, sizeof c.wheel_brake);
        std::memset(c.wheel_lat_friction, 0, sizeof c.wheel_lat_friction);
        std::memset(c.wheel_long_friction, 0, sizeof c.wheel_long_friction);
        std::memset(c.wheel_extra_pushback, 0, sizeof c.wheel_extra_pushback);
        c.ball_hit_valid = 0;
        std::memset(c.ball_hit_rel_pos, 0, sizeof c.ball_hit_rel_pos);
        std::memset(c.ball_hit_ball_pos, 0, sizeof c.ball_hit_ball_pos);
        std::memset(c.ball_hit_extra_vel, 0, sizeof c.ball_hit_extra_vel);
        c.ball_hit_tick = c.ball_hit_extra_tick = -1;
    }
    std::memset(s.ball_vel_impulse_cache, 0, sizeof s.ball_vel_impulse_cache);
    s.ball_sleeping = 0;
    // a new broadphase: cell lists in creation order (btRSBroadphase::createProxy)
    std::memset(s.env.bp_cell, 0, sizeof s.env.bp_cell);
    std::memset(s.env.bp_rank, 0, sizeof s.env.bp_rank);
}

void check(int st) {
    if (st != RLGPU_OK) throw Error(st, rlgpu_last_error());
}

}  // namespace

extern "C" int rlgpu_arena_serialized_size(const rlgpu_arena_state* st, uint64_t* out_bytes) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(st && out_bytes, "rlgpu_arena_serialized_size: null argument");
        Out o{nullptr, 0};
        arena_fields(o, *st);
        *out_bytes = o.n;
    });
}

extern "C" int rlgpu_arena_serialize(const rlgpu_arena_state* st, uint8_t* out, uint64_t cap, uint64_t* written) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(st && out && written, "rlgpu_arena_serialize: null argument");
        Out size{nullptr, 0};
        arena_fields(size, *st);
        RLGPU_REQUIRE(size.n <= cap, "rlgpu_arena_serialize: a buffer of " + std::to_string(cap) +
                                         " bytes, the stream needs " + std::to_string(size.n));
        Out o{out, cap};
        arena_fields(o, *st);
        *written = o.n;
    });
}

extern "C" int rlgpu_arena_deserialize(const uint8_t* in, uint64_t n, rlgpu_arena_state* st, uint64_t* consumed) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(st && (in || n == 0), "rlgpu_arena_deserialize: null argument");
        rlgpu_arena_state tmp = *st;  // *st is left untouched by a failed read
        fresh_engine_state(tmp);
        In r{in, n};
        arena_fields(r, tmp);
        *st = tmp;
        if (consumed) *consumed = r.i;
    });
}

extern "C" int rlgpu_envset_serialize_arena(rlgpu_envset* env, int32_t index, uint8_t* out, uint64_t cap,
                                            uint64_t* written) {
    return rlgpu::guarded([&] {
        rlgpu_arena_state s;
        check(rlgpu_envset_get_arenas(env, index, 1, &s));
        check(rlgpu_arena_serialize(&s, out, cap, written));
    });
}

extern "C" int rlgpu_envset_deserialize_arena(rlgpu_envset* env, int32_t index, const uint8_t* in, uint64_t n,
                                              uint64_t* consumed) {
    return rlgpu::guarded([&] {
        rlgpu_arena_state s;
        check(rlgpu_envset_get_arenas(env, index, 1, &s));
        check(rlgpu_arena_deserialize(in, n, &s, consumed));
        check(rlgpu_envset_set_arenas(env, index, 1, &s));
    });
}
