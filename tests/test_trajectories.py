"""The reference's experience scheduling (rlgpu_learner_config.experience_mode = 1): complete
trajectories only, unfinished ones carried to the next iteration, collection until tsPerItr steps
of complete trajectories, GAE over them with their truncation values.

Reference: GL/public/GigaLearnCPP/Learner.cpp:504-547 (per-player Trajectory, Append),
:643-861 (the collection loop: states / masks before the step, then action, reward, log prob and the
terminal code; maxEpisodeLength truncation; finished trajectories appended to combinedTraj in player
order, nextStates for truncations; loop while combinedTraj.Length() < tsPerItr), :863-990 (tensors,
InferCriticBatched, GAE::Compute, return samples), GL/private/GigaLearnCPP/PPO/GAE.cpp:7-208.

Checker: a host restatement of that bookkeeping over the steps the GPU took (its store rows), with
the CPU oracle env replaying the Learner's own actions for the obs / codes / truncation rows, and
oracle.gae_flat -- the reference's sequential GAE -- over the combined batch.  Bit-exact, three
iterations (so trajectories carried across iterations are covered).
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def test_reference_mode_combined_batch_and_gae_bit_exact(gpu):
    import torch
    from rlgpu.learner import Learner, LearnerConfig
    n, seed, dur = 16, 5, 1.0
    cfg = LearnerConfig(num_arenas=n, rollout_len=8, mini_batch_size=700, seed=seed, max_episode_duration=dur,
                        experience_mode=1, ts_per_itr=1200, train_against_old_versions=False)
    L = Learner(cfg, device=gpu)
    P, W = 4 * n, L.W
    max_len = int(dur * (120.0 / 8))
    o = oracle.EnvSet(n, seed=seed * 1000003, max_episode_steps=max_len)
    np.testing.assert_array_equal(L.obs[0].cpu().numpy().view(np.uint32), o.obs.view(np.uint32))
    # desynchronise the arenas' maxEpisodeLength counters (else every trajectory would end on the same
    # step and no iteration would end with open trajectories to carry over)
    from rlgpu.state import ARENA
    st = np.frombuffer(L.env.get_arenas().tobytes(), ARENA).copy()
    st["env"]["episode_steps"] = np.random.default_rng(1).integers(0, max_len, n)
    buf = np.frombuffer(st.tobytes(), np.uint8)
    L.env.set_arenas(buf)
    o.set_arenas(buf)
    carried = [[] for _ in range(P)]  # the reference's per-player Trajectory, carried across iterations
    for it in range(3):
        std = L.return_stat.std()
        L.collect()
        torch.cuda.synchronize()
        b = L.batch()
        Tm, S, first = b["store_rows"], b["steps"], b["first_step"]
        obs, masks = L.obs.cpu().numpy(), L.masks.cpu().numpy()
        acts, logp, rews, terms = (x.cpu().numpy() for x in (L.actions, L.logp, L.rewards, L.terms))
        combined, truncs, ends = [], [], []
        fin = 0
        for s in range(S):
            r, rn = (first + s) % Tm, (first + s + 1) % Tm
            state, mask = obs[r].copy(), masks[r].copy()
            o.step(acts[r], True)
            np.testing.assert_array_equal(obs[rn][:, :167].view(np.uint32), o.obs.view(np.uint32), err_msg=f"it {it} s {s}")
            np.testing.assert_array_equal(terms[r], o.traj_terms, err_msg=f"codes it {it} s {s}")
            for p in range(P):
                carried[p].append((state[p], mask[p], acts[r][p], logp[r][p], rews[r][p], terms[r][p]))
                if terms[r][p]:
                    if terms[r][p] == 2:
                        truncs.append(o.trunc_obs[p].copy())
                    combined += carried[p]
                    fin += len(carried[p])
                    carried[p] = []
            assert (fin >= cfg.ts_per_itr) == (s == S - 1), (it, s, fin)  # stops at the first crossing
        L.consume()
        torch.cuda.synchronize()
        b = L.batch()
        M = b["num_rows"]
        assert M == len(combined) >= cfg.ts_per_itr
        want = [np.stack([c[k] for c in combined]) for k in range(6)]
        got = [b[k].cpu().numpy() for k in ("obs", "masks", "actions", "logp", "rewards", "terms")]
        for name, g, w in zip(("obs", "masks", "actions", "logp", "rewards", "terms"), got, want):
            np.testing.assert_array_equal(g.view(np.uint8), w.astype(g.dtype).view(np.uint8), err_msg=f"it {it} {name}")
        assert b["num_truncs"] == len(truncs)
        if truncs:
            np.testing.assert_array_equal(b["trunc_obs"].cpu().numpy().view(np.uint32), np.stack(truncs).view(np.uint32))
        vals, tv = b["values"].cpu().numpy(), b["trunc_vals"].cpu().numpy()
        adv, tgt, ret, _, st = oracle.gae_flat(want[4], want[5], vals, tv if truncs else None, cfg.gamma, cfg.gae_lambda,
                                               std, cfg.reward_clip_range)
        assert st == 0
        np.testing.assert_array_equal(b["adv"].cpu().numpy().view(np.uint32), adv.view(np.uint32), err_msg=f"adv it {it}")
        np.testing.assert_array_equal(b["target"].cpu().numpy().view(np.uint32), tgt.view(np.uint32))
        np.testing.assert_array_equal(b["ret"].cpu().numpy().view(np.uint32), ret.view(np.uint32))
        # the critic values are the 16-bit critic over the combined rows
        np.testing.assert_array_equal(vals, L.ppo.infer_critic(b["obs"].contiguous()).cpu().numpy())
        before = L.total_steps
        L.learn()
        L.finish_iteration()
        assert L.total_steps - before == S * P
        opened = sum(len(c) > 0 for c in carried)
        assert opened > 0, it  # open trajectories carried into the next iteration
