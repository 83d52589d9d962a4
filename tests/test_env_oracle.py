"""Known-answer tests pinning the CPU oracle (oracle/rsim_ref.cpp + oracle/env_ref.cpp) to the
constants and rules the reference's own files state (the reference ships no tests,
so these are the anchors).  CPU only."""
import numpy as np
import pytest

import oracle
from rlgpu.state import ARENA, BT_TO_UU, UU_TO_BT

# DefaultAction.cpp:13-88 (RF = {-1, 0, 1}, RB = {0, 1})
RF, RB = (-1.0, 0.0, 1.0), (0.0, 1.0)


def expected_action_table():
    rows = []
    for th in RF:
        for st in RF:
            for bo in RB:
                for hb in RB:
                    if bo == 1 and th != 1:
                        continue
                    rows.append([th, st, 0, st, 0, 0, bo, hb])
    ng = len(rows)
    for pi in RF:
        for ya in RF:
            for ro in RF:
                for ju in RB:
                    for bo in RB:
                        if ju == 1 and ya != 0:
                            continue
                        if pi == ro == ju == 0:
                            continue
                        hb = float(ju == 1 and (pi != 0 or ya != 0 or ro != 0))
                        rows.append([bo, ya, pi, ya, ro, ju, bo, hb])
    return np.array(rows, np.float32), ng


def _state(env):
    return np.frombuffer(env.get_arenas().tobytes(), ARENA).copy()


def _set(env, st):
    env.set_arenas(np.frombuffer(st.tobytes(), np.uint8))


def _act(n, idx):
    return np.full(4 * n, idx, np.int32)


NOOP = 8  # throttle 0, steer 0, boost 0, handbrake 0 (th=-1 rows 0-5; th=0: steer -1 rows 6-7, steer 0 rows 8-9)


def test_sizes_obs_actions():
    """run_out.log:50-51: obs 167 = 9 + 8 + 34 + 29*4, 90 actions."""
    env = oracle.EnvSet(2, seed=1)
    assert env.obs.shape == (8, 167) and env.masks.shape == (8, 90)
    assert oracle.OBS == 9 + 8 + 34 + 29 * 4 == 167


def test_action_table_matches_default_action():
    table, masks = oracle.action_table()
    want, ng = expected_action_table()
    assert ng == 24 and want.shape == (90, 8)
    np.testing.assert_array_equal(table, want)
    np.testing.assert_array_equal(table[NOOP], [0, 0, 0, 0, 0, 0, 0, 0])
    ground, air, jump, boost = masks
    assert ground[:24].all() and not ground[24:].any()
    # DefaultAction.cpp:74-88: air = (i > numGroundActions && !jump) -- the `>` quirk drops the
    # first air action -- plus the ground rows with throttle == boost and steer/yaw == handbrake
    want_air = np.zeros(90, np.uint8)
    for i in range(90):
        x = want[i]
        want_air[i] = (i > ng and x[5] == 0) or (i < ng and x[0] == x[6] and (x[3] != 0) == (x[7] != 0))
    np.testing.assert_array_equal(air, want_air)
    assert air[24] == 0 and want[24][5] == 0  # the quirk bites a jump-free air action
    np.testing.assert_array_equal(jump, (want[:, 5] != 0).astype(np.uint8))
    np.testing.assert_array_equal(boost, (want[:, 6] != 0).astype(np.uint8))


def test_kickoff_spawns():
    """RLConst.h:297-303 kickoff slots, orange mirrored (Arena.cpp:183-186), CAR_SPAWN_REST_Z 17,
    BOOST_SPAWN_AMOUNT 100/3, BALL_REST_Z 93.15, all pads active."""
    slots = {(-2048, -2560), (2048, -2560), (-256, -3840), (256, -3840), (0, -4608)}
    env = oracle.EnvSet(16, seed=5)
    st = _state(env)
    for a in range(16):
        seen = []
        for c in range(4):
            p = st["cars"][a]["body"]["pos"][c] * BT_TO_UU
            assert abs(p[2] - 17.0) < 1e-3
            xy = (round(float(p[0])), round(float(p[1])))
            if c % 2 == 1:  # orange
                xy = (-xy[0], -xy[1])
            assert xy in slots
            seen.append(xy)
            assert abs(st["cars"][a]["boost"][c] - 100.0 / 3.0) < 1e-4
        assert len(set(seen[0::2])) == 2  # two distinct slots per team, mirrored for orange
        assert seen[0::2] == seen[1::2]
        np.testing.assert_allclose(st["ball"][a]["pos"] * BT_TO_UU, [0, 0, 93.15], atol=1e-3)
        assert (st["pads"][a]["is_active"] == 1).all()


def test_zero_velocity_ball_sleeps_midair():
    """Arena.cpp:721-727: zero linear and angular velocity -> ISLAND_SLEEPING, no gravity."""
    env = oracle.EnvSet(1, seed=3)
    st = _state(env)
    st["ball"][0]["pos"] = np.array([0, 0, 1000], np.float32) * UU_TO_BT
    st["ball"][0]["vel"] = 0
    st["ball"][0]["angvel"] = 0
    _set(env, st)
    env.step(_act(1, NOOP), False)
    assert float(_state(env)["ball"][0]["pos"][2] * BT_TO_UU) == pytest.approx(1000.0)


def test_ball_sleeps_at_kickoff_until_touched():
    env = oracle.EnvSet(4, seed=2)
    before = _state(env)["ball"]["pos"].copy()
    for _ in range(3):
        env.step(_act(4, NOOP), False)
    np.testing.assert_array_equal(_state(env)["ball"]["pos"], before)


def test_gravity_and_ball_damping():
    """Gravity -650 uu/s^2 (RLConst GRAVITY_Z), ball drag 0.03 (Ball.cpp:94), symplectic Euler.
    A ball at exactly zero velocity is put to sleep and hangs (Arena.cpp:721-727), so it gets a
    tiny horizontal velocity to stay active."""
    env = oracle.EnvSet(1, seed=3)
    st = _state(env)
    st["ball"][0]["pos"] = np.array([0, 0, 1000], np.float32) * UU_TO_BT
    st["ball"][0]["vel"] = np.array([1e-3, 0, 0], np.float32)
    _set(env, st)
    env.step(_act(1, NOOP), False)
    z = float(_state(env)["ball"][0]["pos"][2] * BT_TO_UU)
    v, p, dt, d = 0.0, 1000.0, 1 / 120, (1 - 0.03) ** (1 / 120)
    for _ in range(8):
        v = (v - 650 * dt) * d
        p += v * dt
    assert abs(z - p) < 1e-2, (z, p)


def test_boost_consumption_rate():
    """BOOST_USED_PER_SECOND = 100/3 (RLConst.h:48): 8 ticks of boost cost 8/120 * 100/3."""
    env = oracle.EnvSet(1, seed=4)
    table, _ = oracle.action_table()
    boost_idx = int(np.nonzero((table[:, 0] == 1) & (table[:, 6] == 1) & (table[:, 1] == 0) & (table[:, 7] == 0))[0][0])
    b0 = float(_state(env)["cars"][0]["boost"][0])
    env.step(_act(1, boost_idx), False)   # 7 ticks with the old (no-op) controls + 1 tick boosting
    env.step(_act(1, boost_idx), False)   # 8 more boosting ticks
    b = float(_state(env)["cars"][0]["boost"][0])
    assert abs((b0 - b) - 9 * (100 / 3) / 120) < 1e-3, (b0, b)


def test_small_pad_pickup_and_cooldown():
    """Small pad: +12 boost, cooldown 4 s (RLConst.h:192-209)."""
    env = oracle.EnvSet(1, seed=6)
    pm = oracle.pad_map()
    st = _state(env)
    # the first small pad in arena order (big pads come first, Arena.cpp:532-556)
    pad_uu = np.array([0, -4240, 70], np.float32)  # small pad from RLConst BOOST_LOCATIONS
    st["cars"][0]["body"]["pos"][0] = np.array([pad_uu[0], pad_uu[1], 17], np.float32) * UU_TO_BT
    st["cars"][0]["body"]["vel"][0] = 0
    st["cars"][0]["boost"][0] = 10.0
    _set(env, st)
    env.step(_act(1, NOOP), False)
    s2 = _state(env)
    assert abs(s2["cars"][0]["boost"][0] - 22.0) < 1e-4
    inactive = np.nonzero(s2["pads"][0]["is_active"] == 0)[0]
    assert len(inactive) == 1
    cd = float(s2["pads"][0]["cooldown"][inactive[0]])
    assert 3.9 < cd <= 4.0, cd
    assert pm.shape == (34,)


def test_throttle_top_speed():
    """Drive-torque curve reaches 0 at 1410 uu/s (RLConst.h:342-437): full throttle saturates there."""
    env = oracle.EnvSet(1, seed=8)
    table, _ = oracle.action_table()
    th = int(np.nonzero((table[:, 0] == 1) & (table[:, 1] == 0) & (table[:, 6] == 0) & (table[:, 7] == 0))[0][0])
    for _ in range(75):  # 5 s
        env.step(_act(1, th), False)
    v = _state(env)["cars"][0]["body"]["vel"][0] * BT_TO_UU
    speed = float(np.hypot(v[0], v[1]))
    assert 1380 < speed < 1411, speed


@pytest.mark.parametrize("seed", [0, 1])
def test_oracle_deterministic(seed):
    a, b = oracle.EnvSet(8, seed=seed), oracle.EnvSet(8, seed=seed, threads=4)
    rng = np.random.default_rng(seed)
    for _ in range(20):
        m = a.masks.astype(bool)
        act = np.argmax(rng.random(m.shape) * m, axis=1).astype(np.int32)
        a.step(act, True)
        b.step(act, True)
    assert a.get_arenas().tobytes() == b.get_arenas().tobytes()
    np.testing.assert_array_equal(a.obs, b.obs)


def test_broadphase_cell_lists_follow_home_cell_changes():
    """btRSBroadphase (btRSBroadphase.cpp:160-176,284-320): a body whose home cell changes is re-appended to
    its cells' dynamic lists, so it moves to the end of the list order (bp_rank) while the others keep theirs;
    a body that stays in its cell keeps its place.  Cars 1-4 teleport at kickoff, ball stays: creation order."""
    env = oracle.EnvSet(2, seed=5)
    noop = np.full(8, 8, np.int32)
    for _ in range(2):
        env.step(noop)
    s = _state(env)
    for a in range(2):
        assert sorted(s["env"][a]["bp_rank"]) == [0, 1, 2, 3, 4]
        assert (s["env"][a]["bp_cell"] > 0).all()
    before = s.copy()
    car = s["cars"][0][1]  # body 2
    car["body"]["pos"][0] += -30.0 if car["body"]["pos"][0] > 0 else 30.0  # bullet units: several cells
    env.set_arenas(np.frombuffer(s.tobytes(), np.uint8))
    env.step(noop)
    t = _state(env)
    cells0, cells1 = before["env"][0]["bp_cell"], t["env"][0]["bp_cell"]
    assert cells1[2] != cells0[2]
    others = [0, 1, 3, 4]
    np.testing.assert_array_equal(cells1[others], cells0[others])  # nobody else changed cell
    r0, r1 = before["env"][0]["bp_rank"], t["env"][0]["bp_rank"]
    assert r1[2] == 4
    assert list(np.argsort(r1[others])) == list(np.argsort(r0[others]))
