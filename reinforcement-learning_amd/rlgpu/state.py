"""numpy view of the arena wire format (rlgpu_arena_state, include/rlgpu_env.h).

Bullet units (1 = 50 uu) as RocketSim's internal state; rot is btMatrix3x3 row-major whose
columns are forward/right/up (RocketSim RotMat is column-major, MathTypes.h:160-220).
"""
import numpy as np

BT_TO_UU = 50.0
UU_TO_BT = 1.0 / 50.0

CONTACT = np.dtype([("localA", "<f4", 3), ("localB", "<f4", 3), ("normalB", "<f4", 3), ("dist", "<f4"),
                    ("applied", "<f4"), ("friction", "<f4"), ("restitution", "<f4"), ("special", "<i4")], align=True)
MANIFOLD = np.dtype([("key", "<i4"), ("count", "<i4"), ("pts", CONTACT, 4)], align=True)  # per-tick scratch only
BODY = np.dtype([("pos", "<f4", 3), ("rot", "<f4", 9), ("vel", "<f4", 3), ("angvel", "<f4", 3)], align=True)
CAR = np.dtype([
    ("body", BODY), ("controls", "<f4", 8), ("last_controls", "<f4", 8),
    ("boost", "<f4"), ("jump_time", "<f4"), ("flip_time", "<f4"), ("air_time", "<f4"),
    ("air_time_since_jump", "<f4"), ("time_spent_boosting", "<f4"), ("supersonic_time", "<f4"),
    ("handbrake_val", "<f4"), ("auto_flip_timer", "<f4"), ("auto_flip_torque_scale", "<f4"),
    ("demo_respawn_timer", "<f4"), ("car_contact_cooldown", "<f4"),
    ("flip_rel_torque", "<f4", 3), ("world_contact_normal", "<f4", 3), ("vel_impulse_cache", "<f4", 3),
    ("ball_hit_rel_pos", "<f4", 3), ("ball_hit_ball_pos", "<f4", 3), ("ball_hit_extra_vel", "<f4", 3),
    ("ball_hit_tick", "<i8"), ("ball_hit_extra_tick", "<i8"), ("car_contact_other_id", "<u4"),
    ("is_on_ground", "u1"), ("has_jumped", "u1"), ("has_double_jumped", "u1"), ("has_flipped", "u1"),
    ("is_flipping", "u1"), ("is_jumping", "u1"), ("is_supersonic", "u1"), ("is_auto_flipping", "u1"),
    ("world_contact", "u1"), ("is_demoed", "u1"), ("ball_hit_valid", "u1"), ("pad0", "u1"),
    ("wheel_contact", "u1", 4),
    ("wheel_steer", "<f4", 4), ("wheel_engine_force", "<f4", 4), ("wheel_brake", "<f4", 4),
    ("wheel_lat_friction", "<f4", 4), ("wheel_long_friction", "<f4", 4), ("wheel_extra_pushback", "<f4", 4),
], align=True)
PAD = np.dtype([("cooldown", "<f4"), ("is_active", "u1"), ("pad", "u1", 3), ("prev_locked_car_id", "<u4")], align=True)
ENV = np.dtype([
    ("tick_count", "<i8"), ("last_tick_count", "<i8"), ("prev_ball_vel", "<f4", 3), ("prev_boost", "<f4", 4),
    ("prev_is_flipping", "u1", 4), ("prev_on_ground", "u1", 4), ("has_prev", "u1"), ("terminal", "u1"),
    ("pad", "u1", 2), ("prev_action", "<f4", (4, 8)), ("no_touch_time", "<f4"),
    ("score_blue", "<i4"), ("score_orange", "<i4"), ("penalty_blue", "<i4"), ("penalty_orange", "<i4"),
    ("ev_bump", "u1", 4), ("ev_bumped", "u1", 4), ("ev_demo", "u1", 4), ("ev_demoed", "u1", 4),
    ("rng_counter", "<u4"), ("manifold_overflow", "<u4"), ("episode_steps", "<i4"),
    ("bp_cell", "<u2", 5), ("bp_rank", "u1", 5), ("pad1", "u1"),
], align=True)
ARENA = np.dtype([("ball", BODY), ("ball_vel_impulse_cache", "<f4", 3), ("ball_sleeping", "<i4"),
                  ("cars", CAR, 4), ("pads", PAD, 34), ("env", ENV)], align=True)


def view(buf):
    """Structured view of a uint8 buffer holding N serialised arenas."""
    return np.frombuffer(np.ascontiguousarray(buf, np.uint8).tobytes(), dtype=ARENA).copy()


def to_bytes(arr):
    return np.frombuffer(arr.tobytes(), np.uint8).copy()


# RLGC::GameState records (rlgpu_gamestate, include/rlgpu_gamestate.h): RocketSim GetState units (uu, uu/s,
# rad/s), rot = RotMat forward, right, up
CAR_STATE = np.dtype([
    ("pos", "<f4", 3), ("rot", "<f4", 9), ("vel", "<f4", 3), ("ang_vel", "<f4", 3),
    ("is_on_ground", "u1"), ("has_jumped", "u1"), ("has_double_jumped", "u1"), ("has_flipped", "u1"),
    ("is_flipping", "u1"), ("is_jumping", "u1"), ("is_supersonic", "u1"), ("is_auto_flipping", "u1"),
    ("is_demoed", "u1"), ("world_contact_has_contact", "u1"), ("ball_hit_is_valid", "u1"), ("pad0", "u1"),
    ("wheels_with_contact", "u1", 4), ("flip_rel_torque", "<f4", 3),
    ("jump_time", "<f4"), ("flip_time", "<f4"), ("air_time", "<f4"), ("air_time_since_jump", "<f4"),
    ("boost", "<f4"), ("time_spent_boosting", "<f4"), ("supersonic_time", "<f4"), ("handbrake_val", "<f4"),
    ("auto_flip_timer", "<f4"), ("auto_flip_torque_scale", "<f4"), ("demo_respawn_timer", "<f4"),
    ("world_contact_normal", "<f4", 3), ("car_contact_other_car_id", "<u4"), ("car_contact_cooldown_timer", "<f4"),
    ("ball_hit_relative_pos_on_ball", "<f4", 3), ("ball_hit_ball_pos", "<f4", 3), ("ball_hit_extra_hit_vel", "<f4", 3),
    ("ball_hit_tick_count_when_hit", "<i8"), ("ball_hit_tick_count_when_extra_impulse_applied", "<i8"),
    ("last_controls", "<f4", 8),
], align=True)
PLAYER_STATE = np.dtype([
    ("car", CAR_STATE), ("index", "<i4"), ("car_id", "<u4"), ("team", "<i4"),
    ("events", "u1", 9), ("ball_touched_step", "u1"), ("ball_touched_tick", "u1"), ("pad0", "u1"),
    ("prev_action", "<f4", 8),
], align=True)
# PlayerEventState order of PLAYER_STATE["events"]
EVENTS = ("goal", "save", "assist", "shot", "shot_pass", "bump", "bumped", "demo", "demoed")
GAMESTATE = np.dtype([
    ("delta_time", "<f4"), ("goal_scored", "<i4"), ("last_touch_car_id", "<i4"), ("last_tick_count", "<u8"),
    ("ball", np.dtype([("pos", "<f4", 3), ("rot", "<f4", 9), ("vel", "<f4", 3), ("ang_vel", "<f4", 3)], align=True)),
    ("players", PLAYER_STATE, 4),
    ("boost_pads", "u1", 34), ("boost_pads_inv", "u1", 34),
    ("boost_pad_timers", "<f4", 34), ("boost_pad_timers_inv", "<f4", 34),
], align=True)
