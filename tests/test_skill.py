"""Skill (ELO) matches against old policy versions: rlgpu.skill (PolicyVersionManager::RunSkillMatches,
PolicyVersionManager.cpp:156-300; SkillRating, PolicyVersionManager.h:12-52) and FuzzedKickoffState
(RG/StateSetters/FuzzedKickoffState.h) on the device.

CPU: the ELO update's known answers and conservation, GetModeName, the oracle's FuzzedKickoffState (every car
within FUZZ_POS_RANGE of its kickoff spot, the Philox stream advanced by the 12 fuzz draws).
GPU: the skill env set (no rewards, GoalScoreCondition, fuzzed kickoffs) bit for bit against the oracle; a
whole skill run whose mixed-version rollout is checked step by step -- the new team's actions are the current
policy's, the old team's the old version's (separate single-policy inference), the arenas equal the oracle
stepped with the same actions, and the ratings equal an independent fp32 replay of the oracle's goals.
"""
import numpy as np
import pytest

import oracle


def _f(x):
    return np.float32(x)


def test_elo_known_answers_and_conservation():
    from rlgpu.skill import SkillRating, elo_update
    a, b = SkillRating(), SkillRating()
    elo_update(a, b, "2v2", 5.0, 0.0)  # equal ratings: expected 0.5
    assert a.data["2v2"] == _f(2.5) and b.data["2v2"] == _f(-2.5)
    rng = np.random.default_rng(0)
    for _ in range(2000):
        w, lo = (a, b) if rng.random() < 0.7 else (b, a)
        before = (float(w.data["2v2"]), float(lo.data["2v2"]))
        elo_update(w, lo, "2v2", 5.0, 0.0)
        gain = float(w.data["2v2"]) - before[0]
        loss = before[1] - float(lo.data["2v2"])
        # winner gains inc * (1 - expected), the loser loses the same amount (exact negation in fp32)
        exp = 1.0 / (10.0 ** ((before[1] - before[0]) / 400.0) + 1.0)
        assert abs(gain - 5.0 * (1 - exp)) < 1e-3 and abs(loss - gain) < 1e-3
    assert abs(float(a.data["2v2"]) + float(b.data["2v2"])) < 0.05  # zero-sum up to fp32 rounding
    assert float(a.data["2v2"]) > 0 > float(b.data["2v2"])  # 70 % wins
    # the winner's rating is read once, the loser's after it (GetRating references)
    c = SkillRating({"1v1": 100.0})
    elo_update(c, SkillRating(), "1v1", 5.0, 0.0)
    assert c.data["1v1"] > 100.0


def test_mode_name():
    from rlgpu.skill import SkillRating
    assert SkillRating.mode_name([0, 1, 0, 1]) == "2v2"
    assert SkillRating.mode_name([0, 0, 0, 1]) == "1v3"
    assert SkillRating.mode_name([1, 1]) == "0v2"


def test_oracle_fuzzed_kickoff():
    from rlgpu.state import ARENA
    n = 64
    plain = np.frombuffer(oracle.EnvSet(n, seed=3).get_arenas().tobytes(), ARENA)
    fuzz = np.frombuffer(oracle.EnvSet(n, seed=3, state_setter=1).get_arenas().tobytes(), ARENA)
    d = (fuzz["cars"]["body"]["pos"] - plain["cars"]["body"]["pos"]) * np.float32(50)  # uu
    assert np.abs(d).max() <= 0.1 + 1e-3 and np.abs(d).max() > 0.05
    assert (np.abs(d) > 0).mean() > 0.9
    np.testing.assert_array_equal(fuzz["env"]["rng_counter"], plain["env"]["rng_counter"] + 12)
    np.testing.assert_array_equal(fuzz["cars"]["body"]["rot"], plain["cars"]["body"]["rot"])
    np.testing.assert_array_equal(fuzz["ball"]["pos"], plain["ball"]["pos"])


# ------------------------------------------------------------------ GPU
def _skill_envs(n, seed, gpu):
    from rlgpu import plugins
    from rlgpu.env import EnvSet, FUZZED_KICKOFF_STATE
    tc = plugins.terminals_array([plugins.terminal("GoalScoreCondition")])
    rw = plugins.rewards_array([])
    g = EnvSet(n, seed=seed, device=gpu, save_rewards=False, rewards=rw, terminals=tc, state_setter=FUZZED_KICKOFF_STATE)
    o = oracle.EnvSet(n, seed=seed, rewards=rw, terminals=tc, state_setter=1)
    return g, o


def _arenas(e):
    from rlgpu.state import ARENA
    return np.frombuffer(e.get_arenas().tobytes(), ARENA)


@pytest.mark.gpu
def test_skill_env_fuzzed_kickoff_parity(gpu):
    import torch
    from tests_util import arena_diff, random_actions
    g, o = _skill_envs(32, 9, gpu)
    d = arena_diff(_arenas(g), _arenas(o))
    assert not d, "create:\n" + "\n".join(d)
    rng = np.random.default_rng(4)
    for t in range(60):
        a = random_actions(o.masks, rng)
        o.step(a, True)
        g.step(torch.from_numpy(a).to(gpu), True)
        torch.cuda.synchronize()
        d = arena_diff(_arenas(g), _arenas(o))
        assert not d, f"step {t}:\n" + "\n".join(d)
        np.testing.assert_array_equal(g.terminals.cpu().numpy(), o.terminals)


def _shots(st, rng):
    """Balls flying at a goal from close range, so the run scores."""
    n = st.shape[0]
    side = rng.choice([-1.0, 1.0], n)
    st["ball"]["pos"][:, 0] = rng.uniform(-10, 10, n)
    st["ball"]["pos"][:, 1] = side * rng.uniform(88, 96, n)
    st["ball"]["pos"][:, 2] = 3.0
    st["ball"]["vel"][:, 0] = 0
    st["ball"]["vel"][:, 1] = side * rng.uniform(20, 40, n)
    st["ball"]["vel"][:, 2] = 0
    return st


@pytest.mark.gpu
def test_skill_run_mixed_version_rollout_oracle_checked(gpu):
    import torch
    from tests_util import arena_diff
    from rlgpu.ppo import PPO
    from rlgpu.skill import SkillRating, SkillTracker, SkillTrackerConfig
    from rlgpu.versions import PolicyVersion
    ppo = PPO(policy_layers=(64, 64), critic_layers=(64,), max_rows=4096, seed=11, device=gpu)
    old_ppo = PPO(policy_layers=(64, 64), critic_layers=(64,), max_rows=4096, seed=12, device=gpu)
    versions = [PolicyVersion(1000, old_ppo.policy_version().clone(), SkillRating({"2v2": 7.0}))]
    cfg = SkillTrackerConfig(enabled=True, num_arenas=24, sim_time=3.0, max_sim_time=240.0, deterministic=True)
    tr = SkillTracker(cfg, ppo, gpu, seed=5)
    from rlgpu import plugins
    tc = plugins.terminals_array([plugins.terminal("GoalScoreCondition")])
    o = oracle.EnvSet(cfg.num_arenas, seed=5 + 7919, rewards=plugins.rewards_array([]), terminals=tc, state_setter=1)
    d = arena_diff(_arenas(tr.env), _arenas(o))
    assert not d, "skill env create:\n" + "\n".join(d)
    st = _shots(_arenas(o).copy(), np.random.default_rng(1))
    buf = np.frombuffer(st.tobytes(), np.uint8)
    o.set_arenas(buf)
    tr.env.set_arenas(buf)
    tr.env.build_obs()
    o.build_obs()
    oracle_goals = []
    steps = [0]

    def on_step(actions, old_rows):
        torch.cuda.synchronize()
        # the mixed inference == each policy's own inference on its team's rows
        a = actions.cpu().numpy()
        want_new, _ = ppo.infer_actions(tr.env.obs, tr.env.action_masks, deterministic=True)
        want_old, _ = old_ppo.infer_actions(tr.env.obs, tr.env.action_masks, deterministic=True)
        rows = old_rows.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(a[~rows], want_new.cpu().numpy()[~rows])
        np.testing.assert_array_equal(a[rows], want_old.cpu().numpy()[rows])
        # the oracle follows: Reset, StepFirstHalf, compare, StepSecondHalf with the same actions
        o.reset()
        o.step_first_half()
        dd = arena_diff(_arenas(tr.env), _arenas(o))
        assert not dd, f"step {steps[0]}:\n" + "\n".join(dd)
        o.step_second_half(a)
        s = _arenas(o)
        for i in np.nonzero(o.terminals)[0]:
            oracle_goals.append((steps[0], int(i), float(s["ball"]["pos"][i][1]) * 50.0))
        steps[0] += 1

    report = {}
    goals = tr.run(versions, report, on_step=on_step)
    torch.cuda.synchronize()
    dd = arena_diff(_arenas(tr.env), _arenas(o))
    assert not dd, "after the run:\n" + "\n".join(dd)
    log = tr.log[-1]
    assert steps[0] == tr.steps_run and steps[0] >= 5
    assert len(goals) == len(oracle_goals) and len(goals) >= 4, (len(goals), len(oracle_goals))
    # an independent fp32 replay of the ratings from the oracle's goals
    new_team = log["new_team"]
    cur, oldr = np.float32(0), np.float32(7)
    for (_, i, y), (gi, new_won) in zip(oracle_goals, goals):
        assert i == gi
        ball_team = 0 if y < 0 else 1
        assert new_won == (ball_team != new_team)
        w, lo = (cur, oldr) if new_won else (oldr, cur)
        e = np.float32(1) / (np.power(np.float32(10), np.float32((lo - w) / np.float32(400))) + np.float32(1))
        w2 = np.float32(w + np.float32(5) * np.float32(1 - e))
        l2 = np.float32(lo + np.float32(5) * np.float32(e - 1))
        cur, oldr = (w2, l2) if new_won else (l2, w2)
    assert tr.cur_ratings.data["2v2"] == cur and versions[0].ratings.data["2v2"] == oldr
    assert report["Rating/2v2"] == float(cur)
    print(f"skill run: {steps[0]} steps, {len(goals)} goals, new team {new_team}, rating {float(cur):.4f} "
          f"vs old version {float(oldr):.4f}; continuation {log['continuation']}")
    tr.close()
