"""ORACLE -- RocketSim's arena byte stream (Arena::Serialize / Arena::DeserializeNew) in Python.
TEST INFRASTRUCTURE ONLY: tests/ compare the product's C++ writer / reader
(reinforcement-learning_amd/host/arena_wire.cpp, include/rlgpu_arena_wire.h) with this.

Restated from the reference's field lists with `struct` (little-endian, RS_IS_BIG_ENDIAN = 0);
RS/ = GigaLearnCPP/RLGymCPP/RocketSim/src/:
  DataStreamOut::WriteMultiple    RS/DataStream/DataStreamOut.h:35-44: u32 field count, then each
                                  field's raw bytes (sizeof(T): Vec = 16 B with its 4th lane,
                                  RotMat = 3 Vec = 48 B, bool = 1 B, CarControls = 24 B)
  DataStreamIn::ReadMultiple      RS/DataStream/DataStreamIn.h:73-84: a count mismatch is an error
  Arena::Serialize                RS/Sim/Arena/Arena.cpp:572-599
  Arena::DeserializeNew           RS/Sim/Arena/Arena.cpp:601-671, DeserializeNewCar :703-714
  ArenaConfig                     RS/Sim/Arena/ArenaConfig/ArenaConfig.cpp:5-35, ArenaConfig.h:18-53
  Car::Serialize                  RS/Sim/Car/Car.cpp:316-320 (controls, config, state)
  CarState::Serialize             RS/Sim/Car/Car.cpp:299-305, Car.h:117-123
  BallHitInfo::Serialize          RS/Sim/BallHitInfo/BallHitInfo.cpp:5-10, BallHitInfo.h:9-30
  CarControls                     RS/Sim/CarControls.h:7-38
  CarConfig (Octane)              RS/Sim/Car/CarConfig/CarConfig.h:18-38, CarConfig.cpp:20-81
  BoostPadState::Serialize        RS/Sim/BoostPad/BoostPad.cpp:21-25, BoostPad.h:23-34
  BallState::Serialize            RS/Sim/Ball/Ball.cpp:19-21, Ball.h:17-46
  MutatorConfig::Serialize        RS/Sim/MutatorConfig/MutatorConfig.cpp:36-39, MutatorConfig.h:16-83
  unit conversion                 Car::GetState (Car.cpp:10-19), Ball::GetState (Ball.cpp:27-33):
                                  pos, vel * BT_TO_UU (50.f), angVel as is; RotMat columns from the
                                  row-major bullet basis (MathTypes.h:171-177); SetState multiplies
                                  by UU_TO_BT (Car.cpp:23-36, Ball.cpp:35-49)
  RS_VERSION_ID                   RS/Framework.h:3,100-106 (the u32 WriteToFile prepends)

Parity unpinned at the byte level: the reference holds no serialized arena and cannot be built
or run here, so this restatement of its field lists is the anchor.  The product
writer must match it byte for byte and the reader must agree with deserialize() below.

Cars are written in id order (1..4, team = (id - 1) & 1: ExampleMain's EnvSet adds blue, orange,
blue, orange).  The reference iterates an unordered_set<Car*> (Arena.h:35), so its car order is
unspecified; DeserializeNew re-keys cars by id (Arena.cpp:618-640).
"""
import struct

import numpy as np

F = np.float32
BT_TO_UU = F(50.0)
UU_TO_BT = F(1.0) / F(50.0)
TICK_TIME = F(1.0) / F(120.0)  # Arena.cpp:437 with tickRate 120

# CarConfig CAR_CONFIG_OCTANE (CarConfig.cpp:20-81)
OCTANE = dict(hitbox_size=(120.507, 86.6994, 38.6591), hitbox_offset=(13.87566, 0.0, 20.755),
              front=((51.25, 25.90, 20.755), 38.755, 12.50), back=((-33.75, 29.50, 20.755), 37.055, 15.00),
              dodge_deadzone=0.5)

# MutatorConfig(GameMode::SOCCAR) in MUTATOR_CONFIG_SERIALIZATION_FIELDS order (MutatorConfig.h:77-83)
# with the RLConst.h defaults (RLConst.h:12-205), evaluated in float as the C++ initialisers are
MUTATORS = [
    ("gravity", "vec", (0.0, 0.0, -650.0)), ("carMass", "f", F(180)), ("carWorldFriction", "f", F(0.3)),
    ("carWorldRestitution", "f", F(0.3)), ("ballMass", "f", F(180) / F(6)), ("ballMaxSpeed", "f", F(6000)),
    ("ballDrag", "f", F(0.03)), ("ballWorldFriction", "f", F(0.35)), ("ballWorldRestitution", "f", F(0.6)),
    ("jumpAccel", "f", F(4375) / F(3)), ("jumpImmediateForce", "f", F(875) / F(3)),
    ("boostAccelGround", "f", F(2975) / F(3)), ("boostAccelAir", "f", F(3175) / F(3)),
    ("boostUsedPerSecond", "f", F(100) / F(3)), ("respawnDelay", "f", F(3)),
    ("carSpawnBoostAmount", "f", F(100) / F(3)), ("bumpCooldownTime", "f", F(0.25)),
    ("boostPadCooldown_Big", "f", F(10)), ("boostPadCooldown_Small", "f", F(4)),
    ("ballHitExtraForceScale", "f", F(1)), ("bumpForceScale", "f", F(1)), ("ballRadius", "f", F(91.25)),
    ("unlimitedFlips", "?", False), ("unlimitedDoubleJumps", "?", False), ("demoMode", "B", 0),
    ("enableTeamDemos", "?", False), ("goalBaseThresholdY", "f", F(5124.25)),
]

# bytes of one arena with no valid BallHitInfo, and what each valid one adds (u32 count + 3 Vec + 2 u64)
BASE_BYTES = 2076
HIT_BYTES = 68


def rs_version_id(version="2.1.1"):
    """__RS_GET_VERSION_ID (RS/Framework.h:100-105): over sizeof(RS_VERSION) chars, NUL included,
    result = max(c - '0' + 1, 0) + result * 10 in uint32"""
    r = 0
    for ch in version.encode() + b"\0":
        r = (max(ch - ord("0") + 1, 0) + r * 10) & 0xFFFFFFFF
    return r


class _Out:
    def __init__(self):
        self.b = bytearray()

    def raw(self, fmt, *v):
        self.b += struct.pack("<" + fmt, *v)

    def vec(self, v):
        x, y, z = (float(F(c)) for c in v)
        self.raw("4f", x, y, z, 0.0)

    def many(self, fields):
        """WriteMultiple: u32 count + raw fields; a field is (kind, value)"""
        self.raw("I", len(fields))
        for kind, v in fields:
            if kind == "vec":
                self.vec(v)
            elif kind == "rot":  # RotMat forward, right, up = columns of the row-major basis
                r = np.asarray(v, F).reshape(3, 3)
                for c in range(3):
                    self.vec(r[:, c])
            elif kind == "ctrl":  # a CarControls struct: 5 floats, jump, boost, handbrake, 1 pad byte
                c = np.asarray(v, F)
                self.raw("5f", *(float(x) for x in c[:5]))
                self.raw("3?x", bool(c[5] != 0), bool(c[6] != 0), bool(c[7] != 0))
            elif kind == "f":
                self.raw("f", float(F(v)))
            else:
                self.raw(kind, v)


def _ctrl_fields(c):
    c = np.asarray(c, F)
    # CAR_CONTROLS_SERIALIZATION_FIELDS (CarControls.h:35-38): boost before jump; the record's
    # order is throttle, steer, pitch, yaw, roll, jump, boost, handbrake
    return [("f", c[0]), ("f", c[1]), ("f", c[2]), ("f", c[3]), ("f", c[4]),
            ("?", bool(c[6] != 0)), ("?", bool(c[5] != 0)), ("?", bool(c[7] != 0))]


def _config_fields():
    o = OCTANE  # CAR_CONFIG_SERIALIZATION_FIELDS (CarConfig.h:35-38)
    return [("f", o["dodge_deadzone"]), ("vec", o["hitbox_offset"]), ("vec", o["hitbox_size"]),
            ("vec", o["front"][0]), ("f", o["front"][1]), ("f", o["front"][2]),
            ("vec", o["back"][0]), ("f", o["back"][1]), ("f", o["back"][2])]


def _u64(x):
    return int(x) & (2**64 - 1)


def serialize(rec):
    """bytes of Arena::Serialize for one arena record (a numpy record of rlgpu.state.ARENA)"""
    o = _Out()
    o.many([("B", 0), ("f", TICK_TIME), ("Q", _u64(rec["env"]["tick_count"])), ("I", 4)])
    o.many([("vec", (-4500, -6000, 0)), ("vec", (4500, 6000, 2500)), ("f", 370.0), ("?", True), ("?", True)])
    o.raw("?", False)  # useCustomBoostPads
    o.raw("I", 4)
    for i in range(4):
        c = rec["cars"][i]
        o.raw("B", i & 1)  # team
        o.raw("I", i + 1)  # id
        o.many(_ctrl_fields(c["controls"]))
        o.many(_config_fields())
        o.raw("?", bool(c["ball_hit_valid"]))
        if c["ball_hit_valid"]:
            o.many([("vec", c["ball_hit_rel_pos"]), ("vec", c["ball_hit_ball_pos"]), ("vec", c["ball_hit_extra_vel"]),
                    ("Q", _u64(c["ball_hit_tick"])), ("Q", _u64(c["ball_hit_extra_tick"]))])
        b = c["body"]
        o.many([
            ("vec", b["pos"] * BT_TO_UU), ("rot", b["rot"]), ("vec", b["vel"] * BT_TO_UU), ("vec", b["angvel"]),
            ("?", bool(c["is_on_ground"])), ("?", bool(c["has_jumped"])), ("?", bool(c["has_double_jumped"])),
            ("?", bool(c["has_flipped"])), ("vec", c["flip_rel_torque"]), ("f", c["jump_time"]),
            ("?", bool(c["is_flipping"])), ("f", c["flip_time"]), ("?", bool(c["is_jumping"])),
            ("f", c["air_time_since_jump"]), ("f", c["boost"]), ("f", c["time_spent_boosting"]),
            ("f", c["supersonic_time"]), ("f", c["handbrake_val"]), ("?", bool(c["is_auto_flipping"])),
            ("f", c["auto_flip_timer"]), ("f", c["auto_flip_torque_scale"]), ("?", bool(c["is_demoed"])),
            ("f", c["demo_respawn_timer"]), ("ctrl", c["last_controls"]), ("?", bool(c["world_contact"])),
            ("vec", c["world_contact_normal"]), ("I", int(c["car_contact_other_id"])),
            ("f", c["car_contact_cooldown"])])
    o.raw("I", 34)
    for p in rec["pads"]:
        o.many([("?", bool(p["is_active"])), ("f", p["cooldown"]), ("I", int(p["prev_locked_car_id"]))])
    bl = rec["ball"]
    o.many([("vec", bl["pos"] * BT_TO_UU), ("rot", bl["rot"]), ("vec", bl["vel"] * BT_TO_UU), ("vec", bl["angvel"]),
            ("f", 0.0), ("f", 2900.0), ("f", 0.0)])  # HeatseekerInfo defaults (Ball.h:23-30, RLConst.h:153)
    o.raw("H", len(MUTATORS))
    o.many([(k, v) for _, k, v in MUTATORS])
    return bytes(o.b)


class _In:
    def __init__(self, b):
        self.b, self.p = bytes(b), 0

    def raw(self, fmt):
        fmt = "<" + fmt
        n = struct.calcsize(fmt)
        if self.p + n > len(self.b):
            raise ValueError("arena stream truncated")
        v = struct.unpack_from(fmt, self.b, self.p)
        self.p += n
        return v

    def count(self, n):
        (k,) = self.raw("I")
        if k != n:
            raise ValueError(f"prop count mismatch: expected {n}, have {k}")

    def vec(self):
        return np.array(self.raw("4f")[:3], F)

    def rot(self):
        return np.stack([self.vec() for _ in range(3)], 1).reshape(9)


def _same(got, kind, want):
    if kind == "vec":
        return [F(x) for x in got] == [F(x) for x in want]
    if kind == "f":
        return F(got) == F(want)
    return got == want


def _fresh(rec):
    """what DeserializeNew's new arena holds for state the stream does not carry: CarState() and
    BallHitInfo() defaults, Car / Ball::SetState's cleared velocity-impulse caches, new wheels
    (Car.h:17-100, BallHitInfo.h:11-22, Car.cpp:23-36, Ball.cpp:35-49, Arena.cpp:703-714)"""
    for i in range(4):
        c = rec["cars"][i]
        c["is_supersonic"] = 0
        c["air_time"] = 0
        c["wheel_contact"] = 0
        c["vel_impulse_cache"] = 0
        for k in ("wheel_steer", "wheel_engine_force", "wheel_brake", "wheel_lat_friction", "wheel_long_friction",
                  "wheel_extra_pushback"):
            c[k] = 0
        c["ball_hit_valid"] = 0
        c["ball_hit_rel_pos"] = 0
        c["ball_hit_ball_pos"] = 0
        c["ball_hit_extra_vel"] = 0
        c["ball_hit_tick"] = -1
        c["ball_hit_extra_tick"] = -1
    rec["ball_vel_impulse_cache"] = 0
    rec["ball_sleeping"] = 0
    rec["env"]["bp_cell"] = 0  # a new broadphase: cell lists in creation order (btRSBroadphase::createProxy)
    rec["env"]["bp_rank"] = 0


def deserialize(data, rec):
    """Arena::DeserializeNew of the stream at the start of `data` into the record `rec` (in place);
    returns the bytes consumed.  Fields the stream does not carry are reset as a new arena has them
    (_fresh); the RLGym bookkeeping in rec["env"] other than tick_count is left as it was."""
    s = _In(data)
    _fresh(rec)
    s.count(4)
    mode, tick_time, tick, _last = s.raw("BfQI")
    if mode != 0 or F(tick_time) != TICK_TIME:
        raise ValueError("only SOCCAR arenas at 120 Hz")
    rec["env"]["tick_count"] = np.array(tick, np.uint64).astype(np.int64)
    s.count(5)
    for kind, want in (("vec", (-4500, -6000, 0)), ("vec", (4500, 6000, 2500)), ("f", 370.0), ("?", True),
                       ("?", True)):
        got = s.vec() if kind == "vec" else s.raw(kind)[0]
        if not _same(got, kind, want):
            raise ValueError("only the default ArenaConfig")
    if s.raw("?")[0]:
        raise ValueError("custom boost pads are not supported")
    (ncars,) = s.raw("I")
    if ncars != 4:
        raise ValueError("2v2 arenas only")
    seen = set()
    for _ in range(4):
        team, cid = s.raw("BI")
        i = cid - 1
        if not (0 <= i < 4) or team != (i & 1) or i in seen:
            raise ValueError("car ids must be 1..4, once each, with team = (id - 1) & 1")
        seen.add(i)
        c = rec["cars"][i]
        s.count(8)
        th, st, pi, ya, ro, boost, jump, hb = s.raw("5f3?")
        c["controls"] = np.array([th, st, pi, ya, ro, jump, boost, hb], F)
        s.count(9)
        for kind, want in _config_fields():
            got = s.vec() if kind == "vec" else s.raw("f")[0]
            if not _same(got, kind, want):
                raise ValueError("only the Octane car config is supported")
        (valid,) = s.raw("?")
        if valid:
            c["ball_hit_valid"] = 1
            s.count(5)
            c["ball_hit_rel_pos"] = s.vec()
            c["ball_hit_ball_pos"] = s.vec()
            c["ball_hit_extra_vel"] = s.vec()
            t0, t1 = s.raw("QQ")
            c["ball_hit_tick"] = np.array(t0, np.uint64).astype(np.int64)
            c["ball_hit_extra_tick"] = np.array(t1, np.uint64).astype(np.int64)
        s.count(28)
        b = c["body"]
        b["pos"] = s.vec() * UU_TO_BT
        b["rot"] = s.rot()
        b["vel"] = s.vec() * UU_TO_BT
        b["angvel"] = s.vec()
        c["is_on_ground"], c["has_jumped"], c["has_double_jumped"], c["has_flipped"] = s.raw("4?")
        c["flip_rel_torque"] = s.vec()
        (c["jump_time"],) = s.raw("f")
        (c["is_flipping"],) = s.raw("?")
        (c["flip_time"],) = s.raw("f")
        (c["is_jumping"],) = s.raw("?")
        (c["air_time_since_jump"], c["boost"], c["time_spent_boosting"], c["supersonic_time"],
         c["handbrake_val"]) = s.raw("5f")
        (c["is_auto_flipping"],) = s.raw("?")
        c["auto_flip_timer"], c["auto_flip_torque_scale"] = s.raw("2f")
        (c["is_demoed"],) = s.raw("?")
        (c["demo_respawn_timer"],) = s.raw("f")
        c["last_controls"] = np.array(s.raw("5f3?x"), F)
        (c["world_contact"],) = s.raw("?")
        c["world_contact_normal"] = s.vec()
        c["car_contact_other_id"], c["car_contact_cooldown"] = s.raw("If")
    (npads,) = s.raw("I")
    if npads != 34:
        raise ValueError("SOCCAR has 34 boost pads")  # Arena.cpp:643-650
    for p in rec["pads"]:
        s.count(3)
        p["is_active"], p["cooldown"], p["prev_locked_car_id"] = s.raw("?fI")
    s.count(7)
    bl = rec["ball"]
    bl["pos"] = s.vec() * UU_TO_BT
    bl["rot"] = s.rot()
    bl["vel"] = s.vec() * UU_TO_BT
    bl["angvel"] = s.vec()
    s.raw("3f")  # HeatseekerInfo: unused in SOCCAR
    (nmut,) = s.raw("H")
    if nmut != len(MUTATORS):
        raise ValueError("mutator field count mismatch")  # MutatorConfig.cpp:41-46
    s.count(len(MUTATORS))
    for name, kind, want in MUTATORS:
        got = s.vec() if kind == "vec" else s.raw(kind)[0]
        if not _same(got, kind, want):
            raise ValueError(f"mutator {name} differs from the SOCCAR default")
    return s.p
