"""RocketSim's arena byte stream: the product's host C++ writer / reader (include/rlgpu_arena_wire.h,
host/arena_wire.cpp, rlgpu/arena_wire.py) against the oracle's Python restatement of
Arena::Serialize / Arena::DeserializeNew (oracle/arena_wire.py; RS/Sim/Arena/Arena.cpp:572-671).

The entry points are host code, so the byte-level tests run in the CPU suite; the env-set round
trip is marked gpu.  Parity unpinned at the byte level: the reference holds no serialized arena
and cannot be run here; the anchor is the restatement of its field lists, checked
here byte for byte, by layout spot checks against the field lists and by total size."""
import struct

import numpy as np
import pytest

from oracle import arena_wire as ow
from rlgpu import arena_wire as aw
from rlgpu._lib import RLGPUError
from rlgpu.state import ARENA


def _fill(a, rng):
    """every field of the structured array `a` random (flags 0 / 1)"""
    for name in a.dtype.names:
        v = a[name]
        if v.dtype.names:
            _fill(v, rng)
        elif v.dtype.kind == "f":
            v[...] = rng.normal(0.0, 300.0, v.shape)
        elif v.dtype == np.uint8:
            v[...] = rng.integers(0, 2, v.shape)
        else:
            info = np.iinfo(v.dtype)
            v[...] = rng.integers(max(info.min, -1), min(info.max, 2**40), v.shape, dtype=np.int64)


def _data(rec):
    """the record's field bytes (struct padding normalised: it carries no data). Fields are copied
    one by one into a zeroed record: a whole-record copy would carry the padding bytes along."""
    def copy(dst, src):
        for name in dst.dtype.names:
            if dst[name].dtype.names:
                copy(dst[name], src[name])
            else:
                dst[name] = src[name]
    out = np.zeros(1, ARENA)
    copy(out, np.asarray(rec).reshape(1))
    return out.tobytes()


def random_arena(seed):
    rng = np.random.default_rng(seed)
    arr = np.zeros(1, ARENA)
    _fill(arr, rng)
    ctl = rng.uniform(-1, 1, (1, 4, 2, 8)).astype(np.float32)
    ctl[..., 5:] = rng.integers(0, 2, (1, 4, 2, 3))  # jump, boost, handbrake are buttons
    arr["cars"]["controls"] = ctl[:, :, 0]
    arr["cars"]["last_controls"] = ctl[:, :, 1]
    return arr


@pytest.mark.parametrize("seed", range(8))
def test_writer_matches_oracle_bytes(seed):
    arr = random_arena(seed)
    want = ow.serialize(arr[0])
    got = aw.serialize(arr[0])
    assert got == want
    nvalid = int((arr["cars"]["ball_hit_valid"] != 0).sum())
    assert len(got) == ow.BASE_BYTES + ow.HIT_BYTES * nvalid == aw.serialized_size(arr[0])


def test_stream_layout():
    """spot checks against the reference's field lists"""
    arr = random_arena(3)
    arr["env"]["tick_count"] = 123456789
    b = aw.serialize(arr[0])
    # Arena::Serialize: WriteMultiple(gameMode SOCCAR, tickTime, tickCount, _lastCarID)
    assert struct.unpack_from("<IBfQI", b, 0) == (4, 0, float(ow.TICK_TIME), 123456789, 4)
    # ArenaConfig: minPos, maxPos, maxAABBLen, noBallRot, useCustomBroadphase; then useCustomBoostPads
    assert struct.unpack_from("<I4f4ff??", b, 21) == (5, -4500, -6000, 0, 0, 4500, 6000, 2500, 0, 370, True, True)
    assert struct.unpack_from("<?I", b, 21 + 42) == (False, 4)
    # the first car: team BLUE, id 1, then its CarControls field count
    assert struct.unpack_from("<BII", b, 68) == (0, 1, 8)
    # MutatorConfig closes the stream: u16 27, u32 27, gravity (0, 0, -650), ..., goalBaseThresholdY
    tail = b[-114:]
    assert struct.unpack_from("<HI4f", tail, 0) == (27, 27, 0, 0, -650, 0)
    assert struct.unpack_from("<f", tail, 110)[0] == 5124.25
    # RS_VERSION_ID of RocketSim 2.1.1 (Framework.h:100-106)
    assert ow.rs_version_id() == aw.RS_VERSION_ID == 302020


@pytest.mark.parametrize("seed", range(4))
def test_reader_matches_oracle_and_inverts_writer(seed):
    arr = random_arena(seed)
    data = aw.serialize(arr[0])
    base = random_arena(100 + seed)
    want = base.copy()
    assert ow.deserialize(data + b"tail", want[0]) == len(data)
    got, n = aw.deserialize(data + b"tail", base[0])
    assert n == len(data)
    assert _data(got) == _data(want[0])
    r = arr[0]
    for i in range(4):
        g, c = got["cars"][i], r["cars"][i]
        for k in ("pos", "vel"):  # GetState's * 50, then SetState's * (1 / 50), in float
            np.testing.assert_array_equal(g["body"][k], (c["body"][k] * np.float32(50)) * ow.UU_TO_BT)
        for k in ("rot", "angvel"):
            np.testing.assert_array_equal(g["body"][k], c["body"][k])
        for k in ("controls", "last_controls", "flip_rel_torque", "world_contact_normal"):
            np.testing.assert_array_equal(g[k], c[k])
        for k in ("boost", "jump_time", "flip_time", "air_time_since_jump", "time_spent_boosting", "supersonic_time",
                  "handbrake_val", "auto_flip_timer", "auto_flip_torque_scale", "demo_respawn_timer",
                  "car_contact_cooldown", "car_contact_other_id", "is_on_ground", "has_jumped", "has_double_jumped",
                  "has_flipped", "is_flipping", "is_jumping", "is_auto_flipping", "is_demoed", "world_contact",
                  "ball_hit_valid"):
            assert g[k] == c[k], k
        if c["ball_hit_valid"]:
            assert g["ball_hit_tick"] == c["ball_hit_tick"]
            np.testing.assert_array_equal(g["ball_hit_rel_pos"], c["ball_hit_rel_pos"])
        else:
            assert g["ball_hit_tick"] == -1
        # not in the stream: what DeserializeNew's new arena holds
        assert g["is_supersonic"] == 0 and g["air_time"] == 0 and not g["wheel_brake"].any()
    np.testing.assert_array_equal(got["pads"]["cooldown"], r["pads"]["cooldown"])
    np.testing.assert_array_equal(got["ball"]["angvel"], r["ball"]["angvel"])
    assert got["env"]["tick_count"] == r["env"]["tick_count"]
    assert got["env"]["score_blue"] == base[0]["env"]["score_blue"]  # RLGym bookkeeping kept


def _status(fn):
    with pytest.raises(RLGPUError) as e:
        fn()
    return str(e.value)


def test_reader_rejects_malformed_and_unsupported_streams():
    data = aw.serialize(random_arena(5)[0])

    def patched(off, fmt, *v):
        b = bytearray(data)
        struct.pack_into(fmt, b, off, *v)
        return bytes(b)

    assert "(-1)" in _status(lambda: aw.deserialize(data[:1000]))                          # truncated
    assert "(-1)" in _status(lambda: aw.deserialize(patched(0, "<I", 5)))                  # header field count
    assert "(-1)" in _status(lambda: aw.deserialize(patched(len(data) - 114, "<H", 26)))   # mutator field count
    assert "(-5)" in _status(lambda: aw.deserialize(patched(4, "<B", 1)))                  # GameMode::HOOPS
    assert "(-5)" in _status(lambda: aw.deserialize(patched(len(data) - 12, "<f", 92.0)))  # ballRadius
    assert "(-5)" in _status(lambda: aw.deserialize(patched(69, "<I", 7)))                 # car id outside 1..4
    for bad in (data[:1000], patched(4, "<B", 1), patched(len(data) - 12, "<f", 92.0)):
        with pytest.raises(ValueError):
            ow.deserialize(bad, random_arena(0)[0])


def test_file_version_prefix(tmp_path):
    data = aw.serialize(random_arena(2)[0])
    p = tmp_path / "arena.rsa"
    aw.to_file(p, data)
    raw = p.read_bytes()
    assert struct.unpack_from("<I", raw)[0] == ow.rs_version_id() and raw[4:] == data
    assert aw.from_file(p) == data


@pytest.mark.gpu
def test_envset_round_trip():
    import torch
    from rlgpu import state
    from rlgpu.env import EnvSet
    env = EnvSet(8, seed=7)
    g = torch.Generator().manual_seed(0)
    for _ in range(24):
        env.step(torch.randint(0, 90, (env.num_players,), generator=g, dtype=torch.int32).to(env.device))
    recs = state.view(env.get_arenas())
    data = env.serialize_arena(3)
    assert data == aw.serialize(recs[3]) == ow.serialize(recs[3])
    want = recs.copy()
    ow.deserialize(data, want[5])
    assert env.deserialize_arena(5, data) == len(data)
    after = state.view(env.get_arenas())
    assert _data(after[5]) == _data(want[5])
    for i in (0, 1, 2, 3, 4, 6, 7):
        assert _data(after[i]) == _data(recs[i])
    env.close()
