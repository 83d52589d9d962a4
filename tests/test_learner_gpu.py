"""End-to-end Learner iteration on the GPU (rlgpu/learner.py): collection with the fused
experience append, critic + GAE consumption, PPO learn.

Parity anchors:
  * the rollout buffer (obs / masks / rewards / trajectory codes for every step) equals what the
    CPU oracle EnvSet produces when fed the Learner's own sampled actions -- bit-exact;
  * advantages / targets / returns equal oracle.gae_rollout on the buffer's rewards, codes and the
    critic values -- bit-exact (GAE [T, N] is a same-order restatement);
  * one Learn pass moves the parameters, keeps them finite and reports sane PPO metrics.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _learner(gpu, **kw):
    from rlgpu.learner import Learner, LearnerConfig
    cfg = LearnerConfig(num_arenas=24, rollout_len=24, mini_batch_size=512, seed=5, **kw)
    return Learner(cfg, device=gpu)


def test_rollout_buffer_matches_oracle_env(gpu):
    import torch
    L = _learner(gpu, max_episode_duration=1.2)  # 18-step trajectory cap: exercises TRUNCATED codes
    o = oracle.EnvSet(L.cfg.num_arenas, seed=L.cfg.seed * 1000003, max_episode_steps=18)
    np.testing.assert_array_equal(L.obs[0].cpu().numpy().view(np.uint32), o.obs.view(np.uint32))
    L.collect()
    torch.cuda.synchronize()
    acts = L.actions.cpu().numpy()
    obs, masks = L.obs.cpu().numpy(), L.masks.cpu().numpy()
    rews, terms, trunc = L.rewards.cpu().numpy(), L.terms.cpu().numpy(), L.trunc_obs.cpu().numpy()
    for t in range(L.T):
        assert (masks[t][np.arange(L.P), acts[t]] == 1).all(), "sampled a masked action"
        o.step(acts[t], True)
        np.testing.assert_array_equal(obs[t + 1].view(np.uint32), o.obs.view(np.uint32), err_msg=f"obs t={t}")
        np.testing.assert_array_equal(masks[t + 1], o.masks, err_msg=f"masks t={t}")
        np.testing.assert_array_equal(rews[t].view(np.uint32), o.rewards.view(np.uint32), err_msg=f"rewards t={t}")
        np.testing.assert_array_equal(terms[t], o.traj_terms, err_msg=f"codes t={t}")
        sel = o.traj_terms == 2
        if sel.any():
            np.testing.assert_array_equal(trunc[t][sel], o.trunc_obs[sel])
    assert (terms == 2).any()


def test_consume_gae_matches_oracle(gpu):
    import torch
    L = _learner(gpu)
    L.collect()
    L.consume()
    torch.cuda.synchronize()
    T = L.T
    rews, terms = L.rewards.cpu().numpy(), L.terms.cpu().numpy()
    vals, tv = L.values.cpu().numpy(), L.trunc_vals.cpu().numpy()
    std = 1.0  # first iteration: WelfordStat with < 2 samples -> 1 (WelfordStat.h)
    adv, tgt, ret = oracle.gae_rollout(rews, terms, vals[:T], tv, vals[T], L.cfg.gamma, L.cfg.gae_lambda, std,
                                       L.cfg.reward_clip_range)
    np.testing.assert_array_equal(L.adv.cpu().numpy(), adv)
    np.testing.assert_array_equal(L.target.cpu().numpy(), tgt)
    np.testing.assert_array_equal(L.ret.cpu().numpy(), ret)
    assert L.return_stat.n == L.cfg.return_samples


def test_learn_updates_parameters(gpu):
    import torch
    L = _learner(gpu)
    before = L.ppo.flat().clone()
    rep = L.iterate()
    after = L.ppo.flat()
    assert torch.isfinite(after).all()
    delta = (after - before).abs()
    assert delta.max() > 0
    m = L.ppo.read_metrics()
    assert 0.0 < m["Policy Entropy"] <= 1.0 + 1e-5
    assert m["Mean KL Divergence"] >= -1e-6
    assert np.isfinite(m["Critic Loss"]) and rep["iteration_s"] > 0
    # a second iteration starts from the last obs of the first
    L.iterate()
    assert torch.isfinite(L.ppo.flat()).all()
