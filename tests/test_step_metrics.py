"""ExampleMain's StepCallback metrics on the device (include/rlgpu_env.h rlgpu_envset_step_metrics,
the env kernel's step_metrics()) against the numpy restatement oracle/step_metrics.py over the CPU
oracle's GameStates (src/ExampleMain.cpp:233-283, Report.h:11-45).

Bar: the per-arena fp64 slots BIT-EXACT (both sides add the same float values in step order), the
report totals / counts equal to the oracle's arena-order fp64 reduction."""
import numpy as np
import pytest

import oracle
from oracle import step_metrics as osm
from tests_util import arena_diff, random_actions


def _recs(env):
    from rlgpu.state import ARENA
    return np.frombuffer(env.get_arenas().tobytes(), ARENA).copy()


def test_oracle_metrics_known_answers():
    """hand-made GameStates: every metric of one pass by value"""
    from rlgpu.state import ARENA
    prev = np.zeros(2, ARENA)
    recs = np.zeros(2, ARENA)
    recs["env"]["tick_count"] = 100
    prev["env"]["last_tick_count"] = 92           # tickSkip 8
    recs["ball"]["pos"][:, 2] = 93.15 / 50
    recs["ball"]["pos"][1, 1] = 5300.0 / 50         # arena 1: ball past the goal line (goal scored)
    recs["ball"]["vel"][1] = [3.0, 4.0, 0.0]        # 250 uu/s
    c = recs["cars"]
    c["is_on_ground"][0] = [1, 0, 1, 1]
    c["is_demoed"][0, 3] = 1
    c["boost"][0] = [0, 33.0, 100, 12]
    c["body"]["vel"][0, 0] = [10.0, 0, 0]           # 500 uu/s along +x
    c["body"]["pos"][0, 0] = [-1.0, 0, 93.15 / 50]  # ball straight ahead along +x
    c["ball_hit_valid"][0, 1] = 1
    c["ball_hit_tick"][0, 1] = 92                   # inside [100 - 8, ...]: touched this step
    c["ball_hit_valid"][0, 2] = 1
    c["ball_hit_tick"][0, 2] = 91                   # one tick too early
    s = osm.accumulate(np.zeros((2, osm.SLOTS)), prev, recs, players=True)
    assert list(s[0, 0:4]) == [0, 1, 0, 0]
    assert list(s[0, 4:8]) == [0, 1, 0, 0]
    assert list(s[0, 8:12]) == [0, 0, 0, 1]
    assert s[0, 12] == 500.0 and s[0, 16] == np.float32(500.0)
    assert list(s[0, 20:24]) == [0, 33.0, 100, 12]
    assert s[0, 25] == np.float32(93.15 / 50) * np.float32(50) and s[0, 24] == 0
    assert s[1, osm.GOALS] == 1 and s[1, osm.GOAL_SPEED] == 250.0 and s[0, osm.GOALS] == 0
    r = osm.report(s)
    assert r["Player/Ball Touch Ratio"] == (1.0, 8) and r["Player/Touch Height"][1] == 1
    assert r["Game/Goal Speed"] == (250.0, 1)
    s2 = osm.accumulate(np.zeros((2, osm.SLOTS)), prev, recs, players=False)
    assert not s2[:, :28].any() and s2[:, osm.PASSES].sum() == 0 and s2[1, osm.GOALS] == 1


@pytest.mark.gpu
def test_step_metrics_match_oracle(gpu):
    import torch
    from rlgpu.env import EnvSet
    n, steps = 64, 160
    g, o = EnvSet(n, seed=21, device=gpu), oracle.EnvSet(n, seed=21)
    g.enable_step_metrics()
    slots = np.zeros((n, osm.SLOTS))
    rng = np.random.default_rng(4)
    goals = touches = 0
    for t in range(steps):
        if t in (20, 90):  # balls thrown at cars (touches) or into a goal mouth (goals)
            st = _recs(o)
            for i in range(n):
                if i % 4 == 3:
                    side = 1.0 if (i // 4) % 2 else -1.0
                    st["ball"][i]["pos"] = np.float32([0.0, side * 100.0, 3.0])
                    st["ball"][i]["vel"] = np.float32([0.0, side * 60.0, 0.0])
                else:
                    d = st["cars"][i]["body"]["pos"][i % 4] - st["ball"][i]["pos"]
                    st["ball"][i]["vel"] = (d / (np.linalg.norm(d) + 1e-6) * rng.uniform(40, 110)).astype(np.float32)
            buf = np.frombuffer(st.tobytes(), np.uint8)
            o.set_arenas(buf)
            g.set_arenas(buf)
        a = random_actions(o.masks, rng)
        prev = _recs(o)
        o.step(a, False)               # the GameStates the callback sees: before the reset
        cur = _recs(o)
        osm.accumulate(slots, prev, cur, players=(t + 1) % 4 == 0)
        o.reset()                      # EnvSet::Reset of the terminated arenas
        g.step(torch.from_numpy(a).to(gpu), True)
        goals, touches = slots[:, osm.GOALS].sum(), slots[:, 4:8].sum()
    torch.cuda.synchronize()
    d = arena_diff(_recs(g), _recs(o))
    assert not d, "env diverged: " + "; ".join(d[:3])
    got = g.step_metric_slots()
    np.testing.assert_array_equal(got.view(np.uint64), slots.view(np.uint64))
    assert touches >= 4 and goals >= 4, f"sample too quiet: {touches} touches, {goals} goals"
    want = osm.report(slots)
    rep = g.step_metrics(reset=True)
    for k in osm.NAMES:
        assert rep[k][1] == want[k][1], k
        assert rep[k][0] == want[k][0], k
    assert rep["Player/Speed"][1] == 4 * n * (steps // 4)
    assert not g.step_metric_slots().any()
    g.enable_step_metrics(False)
    with pytest.raises(Exception):
        g.step_metric_slots()
    g.close()
    print(f"goals {goals:.0f} touches {touches:.0f}")


@pytest.mark.gpu
def test_learner_reports_step_metrics(gpu):
    from rlgpu.learner import Learner, LearnerConfig
    cfg = LearnerConfig(num_arenas=32, rollout_len=16, mini_batch_size=512, policy_layers=(64, 64),
                        critic_layers=(64, 64))
    L = Learner(cfg, device=gpu)
    L.iterate()
    rep = L.step_metrics()
    assert 0.0 <= rep["Player/In Air Ratio"] <= 1.0 and 0.0 <= rep["Player/Boost"] <= 100.0
    assert rep["Player/Speed"] >= 0.0
    assert L.step_metrics() == {}     # reset by the previous call
    L.close()
