"""ORACLE -- the BASELINE config C1 training loop on CPU.  TEST INFRASTRUCTURE ONLY.

C1 = 64 parallel arenas, actor / critic [256, 256] (LayerNorm + LeakyReLU), the reference's CPU
libtorch path (BASELINE.json configs[0]).  The reference binary cannot be run here, so
this restates its collection -> consumption -> learn loop with the oracle's CPU arena step
(oracle.EnvSet, the C++ restatement of RocketSim + RLGymCPP) and torch CPU fp32 for the MLP (the op
family libtorch runs on CPU), following GigaLearnCPP:
  InferActions (PPOLearner.cpp:78-184): logits + (-1e10)*!mask, softmax, clamp [1e-11, 1], multinomial
  GAE (GAE.cpp:7-208): oracle.gae_rollout
  Learn (PPOLearner.cpp:278-581): advantage normalisation, clipped policy loss - entropy, MSE critic,
  clip_grad_norm_ 0.5, AdamW (lr 2.5e-4)
Only bench.py's cpu_baseline leg uses it, to time "PPO wall-clock per 1M agent-steps" on the box's
host cores beside the GPU engine.
"""
import math
import time

import numpy as np

from . import EnvSet, gae_rollout

OBS, ACTIONS = 167, 90


def _mlp(inp, out, layers):
    import torch
    mods, prev = [], inp
    for h in layers:
        mods += [torch.nn.Linear(prev, h), torch.nn.LayerNorm(h), torch.nn.LeakyReLU(0.01)]
        prev = h
    mods.append(torch.nn.Linear(prev, out))
    return torch.nn.Sequential(*mods)


def run_c1(seconds=10.0, arenas=64, rollout=64, layers=(256, 256), threads=16, seed=1234):
    """Iterations of the C1 loop until `seconds` have passed; returns timing per 1M agent-steps."""
    import torch
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(seed)
    torch.manual_seed(seed)
    pol, crit = _mlp(OBS, ACTIONS, layers), _mlp(OBS, 1, layers)
    opt_p = torch.optim.AdamW(pol.parameters(), lr=2.5e-4)
    opt_c = torch.optim.AdamW(crit.parameters(), lr=2.5e-4)
    env = EnvSet(arenas, seed=seed, threads=threads, max_episode_steps=4500)
    P = 4 * arenas
    agent_steps, t_env, t_inf, t_learn = 0, 0.0, 0.0, 0.0
    t0 = time.perf_counter()
    its = 0
    while True:
        obs = np.zeros((rollout + 1, P, OBS), np.float32)
        masks = np.zeros((rollout + 1, P, ACTIONS), np.uint8)
        acts = np.zeros((rollout, P), np.int64)
        logp = np.zeros((rollout, P), np.float32)
        rews = np.zeros((rollout, P), np.float32)
        terms = np.zeros((rollout, P), np.int8)
        obs[0], masks[0] = env.obs, env.masks
        trunc = []  # (t, player rows, pre-reset obs) of trajectories ending TRUNCATED
        for t in range(rollout):
            a = time.perf_counter()
            with torch.no_grad():
                logits = pol(torch.from_numpy(obs[t])) + (-1e10) * torch.from_numpy(masks[t] == 0).float()
                probs = torch.softmax(logits, -1).clamp(1e-11, 1.0)
                act = torch.multinomial(probs, 1, generator=g).squeeze(1)
                logp[t] = probs.gather(1, act[:, None]).squeeze(1).log().numpy()
            acts[t] = act.numpy()
            b = time.perf_counter()
            env.step(acts[t].astype(np.int32), True)
            c = time.perf_counter()
            obs[t + 1], masks[t + 1], rews[t], terms[t] = env.obs, env.masks, env.rewards, env.traj_terms
            rows = np.nonzero(env.traj_terms == 2)[0]
            if rows.size:
                trunc.append((t, rows, env.trunc_obs[rows].copy()))
            t_inf += b - a
            t_env += c - b
        a = time.perf_counter()
        with torch.no_grad():
            vals = crit(torch.from_numpy(obs.reshape(-1, OBS))).view(rollout + 1, P).numpy()
        tv = np.zeros((rollout, P), np.float32)
        for t, rows, o in trunc:  # truncation values on the pre-reset obs
            with torch.no_grad():
                tv[t, rows] = crit(torch.from_numpy(o)).view(-1).numpy()
        adv, tgt, _ = gae_rollout(rews, terms, vals[:rollout], tv, vals[rollout], 0.99, 0.95, 1.0, 200.0)
        M = rollout * P
        X = torch.from_numpy(obs[:rollout].reshape(M, OBS))
        MK = torch.from_numpy(masks[:rollout].reshape(M, ACTIONS))
        A = torch.from_numpy(acts.reshape(M))
        OL = torch.from_numpy(logp.reshape(M))
        AD = torch.from_numpy(adv.reshape(M))
        TG = torch.from_numpy(tgt.reshape(M))
        for _ in range(2):  # epochs; batch = minibatch = the whole iteration (ExampleMain at C1 size)
            perm = torch.randperm(M, generator=g)
            x, mk, ac, ol, ad, tg = X[perm], MK[perm], A[perm], OL[perm], AD[perm], TG[perm]
            ad = (ad - ad.mean()) / (ad.std() + 1e-8)
            logits = pol(x) + (-1e10) * (mk == 0).float()
            probs = torch.softmax(logits, -1).clamp(1e-11, 1.0)
            lp = probs.gather(1, ac[:, None]).squeeze(1).log()
            ent = (-(probs.log() * probs).sum(-1) / math.log(ACTIONS)).mean()
            ratio = (lp - ol).exp()
            pl = -torch.min(ratio * ad, ratio.clamp(0.8, 1.2) * ad).mean()
            cl = torch.nn.functional.mse_loss(crit(x).view(-1), tg)
            opt_p.zero_grad()
            opt_c.zero_grad()
            (pl - 0.035 * ent + cl).backward()
            torch.nn.utils.clip_grad_norm_(pol.parameters(), 0.5)
            torch.nn.utils.clip_grad_norm_(crit.parameters(), 0.5)
            opt_p.step()
            opt_c.step()
        t_learn += time.perf_counter() - a
        agent_steps += M
        its += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"ppo_s_per_1M_agent_steps": el / agent_steps * 1e6, "env_steps_per_s": agent_steps / 4 / el,
            "agent_steps": agent_steps, "iterations": its, "threads": threads,
            "phase_s": {"env": t_env, "inference": t_inf, "learn": t_learn}}
