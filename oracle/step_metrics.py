"""ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

ExampleMain's StepCallback (src/ExampleMain.cpp:233-283) restated over arena records in numpy, the
checker of the env kernel's device metrics (include/rlgpu_env.h rlgpu_envset_step_metrics).

Per callback call (Learner.cpp:796-797: once per StepSecondHalf), with stepCounter incremented
first (ExampleMain.cpp:236-237): on every 4th call each player of each GameState adds
  In Air Ratio      !isOnGround
  Ball Touch Ratio  ballTouchedStep  (Player.cpp:18-19: hit valid and tickCountWhenHit >= tickCount - tickSkip)
  Demoed Ratio      isDemoed
  Speed             vel.Length()                               (MathTypes.h:35-42)
  Speed Towards Ball RS_MAX(0, vel.Dot((ball.pos - pos).Normalized()))  (MathTypes.h:57-59,88-95, Framework.h:47)
  Boost             boost
  Touch Height      ball.pos.z, only when ballTouchedStep
and on every call each state with goalScored (Arena::IsBallScored) adds Game/Goal Speed =
ball.vel.Length().  Report::AddAvg keeps fp64 (total, count) (Report.h:11-45).  Positions and
velocities are the CarState / BallState values in UU: the record's Bullet-unit floats x 50 in float.

The slots mirror the kernel's per-arena layout so a test can compare them bit for bit: the kernel
adds each arena's values in step order, and so does accumulate() here.
"""
import numpy as np

NAMES = ["Player/In Air Ratio", "Player/Ball Touch Ratio", "Player/Demoed Ratio", "Player/Speed",
         "Player/Speed Towards Ball", "Player/Boost", "Player/Touch Height", "Game/Goal Speed"]
SLOTS = 32
GOAL_SPEED, GOALS, PASSES = 28, 29, 30
BT2UU = np.float32(50.0)
FLT_EPS = np.float32(1.1920928955078125e-07)
GOAL_Y = np.float32(5124.25) + np.float32(91.25)


def _length(v):
    """Vec::Length in float: sqrt of ((x*x + y*y) + z*z) when positive, else 0"""
    l2 = (v[..., 0] * v[..., 0] + v[..., 1] * v[..., 1]) + v[..., 2] * v[..., 2]
    return np.where(l2 > 0, np.sqrt(np.maximum(l2, np.float32(0))), np.float32(0)).astype(np.float32)


def accumulate(slots, prev_recs, recs, players):
    """Add one callback call over the arena records `recs` (the GameStates after the step, before any
    reset) to `slots` [n, SLOTS] (fp64).  prev_recs: the records before the step (their
    last_tick_count gives the step's tickSkip, as GameState::UpdateFromArena)."""
    cars, ball = recs["cars"], recs["ball"]
    cur = recs["env"]["tick_count"].astype(np.int64)
    skip = np.maximum(cur - prev_recs["env"]["last_tick_count"].astype(np.int64), 0)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        if players:
            pos = cars["body"]["pos"].astype(np.float32) * BT2UU          # [n, 4, 3]
            vel = cars["body"]["vel"].astype(np.float32) * BT2UU
            bp = ball["pos"].astype(np.float32) * BT2UU                   # [n, 3]
            lo = (cur - skip).astype(np.uint64)[:, None]
            touched = (cars["ball_hit_valid"] != 0) & (cars["ball_hit_tick"].astype(np.int64).astype(np.uint64) >= lo)
            d = (bp[:, None, :] - pos).astype(np.float32)
            dl = _length(d)
            ok = dl > FLT_EPS * FLT_EPS
            dir_ = np.where(ok[..., None], d / np.where(ok, dl, np.float32(1))[..., None], np.float32(0)).astype(np.float32)
            toward = ((vel[..., 0] * dir_[..., 0] + vel[..., 1] * dir_[..., 1]) + vel[..., 2] * dir_[..., 2]).astype(np.float32)
            vals = [
                np.where(cars["is_on_ground"] != 0, 0.0, 1.0),
                touched.astype(np.float64),
                np.where(cars["is_demoed"] != 0, 1.0, 0.0),
                _length(vel).astype(np.float64),
                np.where(np.float32(0) > toward, np.float32(0), toward).astype(np.float64),
                cars["boost"].astype(np.float64),
            ]
            for k, v in enumerate(vals):
                slots[:, 4 * k:4 * k + 4] += v
            slots[:, 24:28] += np.where(touched, np.broadcast_to(bp[:, None, 2], touched.shape).astype(np.float64), 0.0)
            slots[:, PASSES] += 1.0
        goal = np.abs(ball["pos"][:, 1].astype(np.float32) * BT2UU) > GOAL_Y
        gs = _length(ball["vel"].astype(np.float32) * BT2UU).astype(np.float64)
        slots[:, GOAL_SPEED] += np.where(goal, gs, 0.0)
        slots[:, GOALS] += goal.astype(np.float64)
    return slots


def report(slots):
    """{key: (total, count)} from the slots: fp64 sums over arenas in arena order"""
    out = {}
    passes = 0.0
    goals = 0.0
    tot = [0.0] * 8
    for a in range(slots.shape[0]):
        m = slots[a]
        for k in range(7):
            for p in range(4):
                tot[k] += m[4 * k + p]
        tot[7] += m[GOAL_SPEED]
        goals += m[GOALS]
        passes += m[PASSES]
    counts = [int(4 * passes)] * 6 + [int(tot[1]), int(goals)]
    for k in range(8):
        out[NAMES[k]] = (tot[k], counts[k])
    return out
