"""The env set's reward / terminal registry (include/rlgpu_env.h rlgpu_reward_spec / rlgpu_terminal_spec),
the boundary for the EnvCreateFn's plugin lists (RG/EnvSet/EnvSet.h:14-24, src/ExampleMain.cpp:128-226).

CPU: ExampleMain's default lists as the library holds them, and the rejection of unknown plugin
types / over-long lists by rlgpu_envset_create before any device work (RLGPU_ERR_UNSUPPORTED /
RLGPU_ERR_INVALID_ARG, message in rlgpu_last_error()).
GPU: custom lists -- every registry reward type with non-default parameters, reordered, dropped and
re-weighted, ZeroSum wrappers, all terminal types merged -- bit-exact against the oracle given the
same lists, on every arena record, obs, reward, terminal, trajectory code and lastRewards value.
"""
import ctypes

import numpy as np
import pytest

import oracle
from rlgpu import plugins
from tests_util import arena_diff, random_actions


def _create(rewards=None, terminals=None, n_rewards=None, n_terminals=None):
    from rlgpu import _lib
    from rlgpu.env import _Config, _bind
    L = _bind()
    cfg = _Config(4, 8, 7, 1, 1, 0)
    if rewards is not None:
        cfg.rewards, cfg.n_rewards = rewards.ctypes.data, rewards.size if n_rewards is None else n_rewards
    if terminals is not None:
        cfg.terminals, cfg.n_terminals = terminals.ctypes.data, terminals.size if n_terminals is None else n_terminals
    h = ctypes.c_void_p()
    st = L.rlgpu_envset_create(ctypes.byref(cfg), ctypes.byref(h))
    return st, _lib.last_error()


def test_default_plugins_are_example_main():
    from rlgpu.env import _bind
    L = _bind()
    rw = np.zeros(32, plugins.REWARD_SPEC)
    tc = np.zeros(8, plugins.TERMINAL_SPEC)
    nr, nt = ctypes.c_int32(), ctypes.c_int32()
    assert L.rlgpu_envset_default_plugins(rw.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nr),
                                          tc.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nt)) == 0
    want_rw, want_tc = plugins.example_main()
    assert (nr.value, nt.value) == (13, 2)
    assert rw[:13].tobytes() == want_rw.tobytes()
    assert tc[:2].tobytes() == want_tc.tobytes()
    # the weights of src/ExampleMain.cpp:132-177 in order
    np.testing.assert_array_equal(want_rw["weight"], np.float32([0.25, 0.12, 5, 4, 60, 6, 8, 0.1, 0.01, 20, 80, 150, 1]))


def test_unknown_plugin_types_are_rejected():
    rw = plugins.rewards_array([plugins.reward("AirReward", 1.0)])
    bad = rw.copy()
    bad["type"] = 99
    st, msg = _create(rewards=bad)
    assert st == -5 and "unknown type 99" in msg, (st, msg)
    tc = plugins.terminals_array([plugins.terminal("GoalScoreCondition")])
    badt = tc.copy()
    badt["type"] = -1
    st, msg = _create(terminals=badt)
    assert st == -5 and "terminal condition 0" in msg, (st, msg)
    st, msg = _create(rewards=rw, n_rewards=33)
    assert st == -1 and "n_rewards" in msg
    with pytest.raises(plugins.UnknownPlugin):
        plugins.reward("MyOwnCppReward", 1.0)
    with pytest.raises(plugins.UnknownPlugin):
        plugins.terminal("TimeoutCondition", 300)


CUSTOM_REWARDS = [
    plugins.reward("GoalReward", 90, -0.5),
    plugins.reward("TouchBallReward", 3.0),
    plugins.reward("FaceBallReward", 0.02),
    plugins.reward("SaveBoostReward", 0.3, 0.7),
    plugins.zero_sum(plugins.reward("DemoedPenalty", 7.0), 0.3, 0.8),
    plugins.reward("StrongTouchReward", 11, 10, 90),
    plugins.reward("VelocityReward", 0.5, True),
    plugins.reward("SpeedReward", 0.25),
    plugins.reward("BumpedPenalty", 4.0),
    plugins.reward("VelocityBallToGoalReward", 2.0, True),
    plugins.reward("KickoffProximityReward2v2Enhanced", 1.5),
    plugins.reward("LosingPenaltyReward", 2.0, 0.05),
    plugins.reward("PickupBoostReward", 0.7),
    plugins.reward("AirReward", 0.1),
    plugins.reward("WavedashReward", 0.4),
    plugins.reward("TouchAccelReward", 5.0),
    plugins.reward("VelocityPlayerToBallReward", 1.25),
    plugins.reward("BumpReward", 9.0),
    plugins.reward("DemoReward", 12.0),
    plugins.reward("AirReward", -0.05),  # a type twice
    # its member tunables (KickoffProximityReward2v2Enhanced.h:9-12) as device parameters
    plugins.reward("KickoffProximityReward2v2Enhanced", 2.5, goer_reward=1.7, rotation_prep_weight=0.35),
]


def test_kickoff_tunables_spec():
    r = plugins.reward("KickoffProximityReward2v2Enhanced", 2.5, goer_reward=1.7, rotation_prep_weight=0.35)
    assert list(r["params"]) == [np.float32(1.7), np.float32(0.35), 1.0]
    d = plugins.reward("KickoffProximityReward2v2Enhanced", 2.5, goer_reward=1.2)  # the defaults: registry zeros
    assert list(d["params"]) == [0.0, 0.0, 0.0]
    with pytest.raises(TypeError):
        plugins.reward("AirReward", 1.0, goer_reward=1.0)
CUSTOM_TERMINALS = [plugins.terminal("NoTouchCondition", 2.5), plugins.terminal("GoalScoreCondition"),
                    plugins.terminal("ScoreLimitCondition", 2), plugins.terminal("NoTouchCondition", 4.0)]


def _check(g, o, what):
    import torch
    from rlgpu.state import ARENA
    torch.cuda.synchronize()
    d = arena_diff(np.frombuffer(g.get_arenas().tobytes(), ARENA), np.frombuffer(o.get_arenas().tobytes(), ARENA))
    assert not d, f"{what}: arena state differs\n" + "\n".join(d)
    np.testing.assert_array_equal(g.obs.cpu().numpy().view(np.uint32), o.obs.view(np.uint32), err_msg=what)
    np.testing.assert_array_equal(g.rewards.cpu().numpy().view(np.uint32), o.rewards.view(np.uint32),
                                  err_msg=what + ": rewards")
    np.testing.assert_array_equal(g.terminals.cpu().numpy(), o.terminals, err_msg=what + ": terminals")
    np.testing.assert_array_equal(g.last_rewards.cpu().numpy().view(np.uint32), o.last_rewards.view(np.uint32),
                                  err_msg=what + ": lastRewards")


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["custom", "subset", "empty"])
def test_registry_lists_bit_exact_vs_oracle(gpu, case):
    import torch
    from rlgpu.env import EnvSet, StepOutputs
    from rlgpu.state import ARENA
    if case == "custom":
        rw, tc = CUSTOM_REWARDS, CUSTOM_TERMINALS
    elif case == "subset":  # ExampleMain's list reordered, two dropped, re-weighted; GoalScore only
        em, _ = plugins.example_main()
        rw = [em[i].copy() for i in (12, 3, 0, 11, 6, 5, 4, 8, 9, 10, 2)]
        for k, r in enumerate(rw):
            r["weight"] = r["weight"] * (0.5 + 0.1 * k)
        tc = [plugins.terminal("GoalScoreCondition")]
    else:
        rw, tc = [], []
    rwa, tca = plugins.rewards_array(rw), plugins.terminals_array(tc)
    n = 64
    g = EnvSet(n, seed=41, device=gpu, rewards=rwa, terminals=tca)
    o = oracle.EnvSet(n, seed=41, rewards=rwa, terminals=tca)
    assert g.num_rewards == o.num_rewards == len(rw)
    rng = np.random.default_rng(6)
    terms = torch.empty(4 * n, dtype=torch.int8, device=gpu)
    saw = set()
    for t in range(140):
        if t == 30:  # throw balls at cars and goals, cars at each other: touches, bumps, demos, goals
            st = np.frombuffer(o.get_arenas().tobytes(), ARENA).copy()
            for i in range(n):
                c = st["cars"][i]["body"]["pos"][i % 4]
                goal_y = 5200 / 50.0 * (1 if i % 2 else -1)
                tgt = c if i % 3 else np.float32([0, goal_y, 1.0])
                d = tgt - st["ball"][i]["pos"]
                st["ball"][i]["vel"] = (d / (np.linalg.norm(d) + 1e-6) * rng.uniform(30, 110)).astype(np.float32)
                for k in range(4):
                    dd = st["cars"][i]["body"]["pos"][(k + 1) % 4] - st["cars"][i]["body"]["pos"][k]
                    st["cars"][i]["body"]["vel"][k] = (dd / (np.linalg.norm(dd) + 1e-6) * rng.uniform(20, 46)).astype(np.float32)
            buf = np.frombuffer(st.tobytes(), np.uint8)
            o.set_arenas(buf)
            g.set_arenas(buf)
        a = random_actions(o.masks, rng)
        o.step(a, True)
        g.step(torch.from_numpy(a).to(gpu), True, StepOutputs.of(terminals=terms))
        _check(g, o, f"{case} step {t}")
        np.testing.assert_array_equal(terms.cpu().numpy(), o.traj_terms, err_msg=f"{case} step {t}: codes")
        saw.update(np.unique(o.terminals).tolist())
    if case == "empty":
        assert saw == {0} and float(g.rewards.abs().max()) == 0.0
    else:
        assert 1 in saw, saw  # goals ended episodes through the list's NORMAL conditions
    if case == "custom":
        assert 2 in saw  # NoTouch(2.5 s) truncations
