"""Learner -- the GigaLearnCPP training loop for one GPU rank, every array resident in HBM.

Mirrors GGL::Learner::Start (GigaLearnCPP/src/public/GigaLearnCPP/Learner.cpp:482-1056):
  collection   infer actions (bf16 policy) -> fused env step with experience append     :669-861
  consumption  critic over the rollout (InferCriticBatched), GAE, return-std Welford    :863-990
  learning     PPOLearner::Learn: epochs x shuffled minibatches, clip_grad_norm_, AdamW :990-1000
Distributed: one Learner per rank (arenas sharded), PPO gradients all-reduced (sum) over
RCCL before clip_grad_norm_; advantage moments and return samples reduced too.

Experience layout ([T, P] time-major, P = 4 * arenas): the reference keeps per-player
trajectory vectors and trains only on finished trajectories (unfinished ones carry over to the
next iteration); here every collected step is trained in the iteration that collected it, with
the unfinished tail bootstrapped from V(obs_T) -- see DESIGN.md "Deviations".
"""
import math
import time

import numpy as np

from . import dist as _dist
from . import gae as _gae
from .env import EnvSet, StepOutputs
from .ppo import PPO, permutation

OBS, ACTIONS = 167, 90


class WelfordStat:
    """GGL::WelfordStat (Util/WelfordStat.h:7-67): fp64 running mean / variance, the reference's
    update order (delta, delta / (count + 1), variance += delta * deltaN * count)."""

    def __init__(self):
        self.n, self.mean, self.m2 = 0, 0.0, 0.0

    def add(self, xs):
        for x in np.asarray(xs, np.float32).ravel():
            delta = float(x) - self.mean
            delta_n = delta / (self.n + 1)
            self.mean += delta_n
            self.m2 += delta * delta_n * self.n
            self.n += 1

    def get_mean(self):
        return 0.0 if self.n < 2 else self.mean

    def std(self):
        if self.n < 2:
            return 1.0
        var = self.m2 / (self.n - 1)
        if var <= 0:
            var = 1.0
        return math.sqrt(var)

    def to_json(self):  # WelfordStat::ToJSON
        return {"mean": self.mean, "var": self.m2, "count": self.n}

    def read_json(self, j):  # WelfordStat::ReadFromJSON
        self.mean, self.m2, self.n = float(j["mean"]), float(j["var"]), int(j["count"])


def batch_ranges(exp_size, batch_size, overbatching=True):
    """ExperienceBuffer::GetAllBatchesShuffled batch boundaries (ExperienceBuffer.cpp:117-162):
    consecutive [start, start + batch) slices of the shuffled order; with overbatching the last
    batch absorbs a remainder that would leave less than one more full batch; without it the
    remainder is dropped."""
    out = []
    if exp_size <= 0:
        return out
    start = 0
    while start < exp_size:
        end = start + batch_size
        if end + batch_size > exp_size and overbatching:
            end = exp_size
        if end > exp_size:
            break
        if end - start <= 0:
            break
        out.append((start, end))
        if end == exp_size:
            break
        start += batch_size
    return out


class LearnerConfig:
    """The subset of GGL::LearnerConfig / PPOLearnerConfig on the hot path (ExampleMain values)."""

    def __init__(self, **kw):
        self.num_arenas = 4096
        self.tick_skip = 8
        self.action_delay = 7
        self.seed = 123
        self.rollout_len = 128
        self.epochs = 2
        self.mini_batch_size = 50_000
        self.batch_size = None            # None = the whole iteration (ExampleMain: batchSize = tsPerItr)
        self.overbatching = True          # PPOLearnerConfig::overbatching
        self.gamma = 0.99
        self.gae_lambda = 0.95
        self.clip_range = 0.2
        self.entropy_scale = 0.035
        self.policy_lr = 2.5e-4
        self.critic_lr = 2.5e-4
        self.reward_clip_range = 200.0       # PPOLearnerConfig::rewardClipRange
        self.return_samples = 150         # Learner.cpp:959-967
        self.policy_layers = (512, 512)
        self.critic_layers = (512, 512)
        self.max_episode_duration = 300.0  # seconds (ExampleMain)
        self.deterministic = False
        # checkpoints (LearnerConfig.h:31-38): None = no save / load
        self.checkpoint_folder = None
        self.ts_per_save = 10_000_000     # 0 = every iteration (Learner.cpp:44-45)
        self.checkpoints_to_keep = 8      # -1 keeps all
        # self-play against old policy versions (LearnerConfig.h:62-68)
        self.train_against_old_versions = True
        self.train_against_old_chance = 0.15
        self.ts_per_version = 25_000_000
        self.max_old_versions = 32
        for k, v in kw.items():
            if not hasattr(self, k):
                raise AttributeError(f"unknown LearnerConfig field {k}")
            setattr(self, k, v)


class Learner:
    def __init__(self, cfg, device="cuda:0", rank=0, world=1, group=None):
        import torch
        self.cfg, self.rank, self.world, self.group = cfg, rank, world, group
        self.device = torch.device(device)
        T, N = cfg.rollout_len, cfg.num_arenas
        P = 4 * N
        self.P, self.T = P, T
        max_ep = int(cfg.max_episode_duration * (120.0 / cfg.tick_skip))
        self.env = EnvSet(N, seed=cfg.seed * 1000003 + rank, tick_skip=cfg.tick_skip, action_delay=cfg.action_delay,
                          device=device, max_episode_steps=max_ep)
        mb = min(cfg.mini_batch_size, T * P)
        self.ppo = PPO(OBS, ACTIONS, cfg.policy_layers, cfg.critic_layers, policy_lr=cfg.policy_lr,
                       critic_lr=cfg.critic_lr, clip_range=cfg.clip_range, entropy_scale=cfg.entropy_scale,
                       max_rows=max(mb, min(P, 65536)), seed=cfg.seed, device=device)
        if world > 1:  # identical initial weights on every rank
            torch.distributed.broadcast(self.ppo.params, 0, group=group)
            self.ppo.refresh_half()
        d = self.device
        # experience buffer (HBM)
        self.obs = torch.empty((T + 1, P, OBS), device=d)
        self.masks = torch.empty((T + 1, P, ACTIONS), dtype=torch.uint8, device=d)
        self.actions = torch.empty((T, P), dtype=torch.int32, device=d)
        self.logp = torch.empty((T, P), device=d)
        self.rewards = torch.empty((T, P), device=d)
        self.terms = torch.empty((T, P), dtype=torch.int8, device=d)
        self.trunc_obs = torch.zeros((T, P, OBS), device=d)
        self.values = torch.empty((T + 1, P), device=d)
        self.trunc_vals = torch.zeros((T, P), device=d)
        self.adv = torch.empty((T, P), device=d)
        self.target = torch.empty((T, P), device=d)
        self.ret = torch.empty((T, P), device=d)
        self.obs[0].copy_(self.env.obs)
        self.masks[0].copy_(self.env.action_masks)
        self.return_stat = WelfordStat()
        self.total_steps = 0
        self.iteration = 0
        self._rng_step = 0
        self.rng = np.random.default_rng(cfg.seed + 7919 * rank)
        self.env_events = None  # optional list collecting (start, end) events around env steps
        # self-play: the manager of old versions, this iteration's version and team (None = all
        # players use the current policy); the draw is rank-independent so every rank agrees
        self.versions = None
        self.old_version, self.old_team = None, 0
        self._vrng = np.random.default_rng(cfg.seed + 104729)
        if cfg.train_against_old_versions:
            from .versions import PolicyVersionManager
            import os
            vf = os.path.join(cfg.checkpoint_folder, "policy_versions") if cfg.checkpoint_folder else None
            self.versions = PolicyVersionManager(self.ppo, vf, cfg.max_old_versions, cfg.ts_per_version)
        # old-version player rows: team of player p is p % 2 (cars 0, 2 blue; 1, 3 orange)
        team = torch.arange(P, device=d) % 2
        self._old_rows = [(team == k).to(torch.uint8) for k in range(2)]
        self.last_checkpoint = None
        if cfg.checkpoint_folder:  # Learner ctor: load the most recent checkpoint (Learner.cpp:145-153)
            from . import checkpoint as _ckpt
            self.last_checkpoint = _ckpt.load(self, cfg.checkpoint_folder)
            if self.versions is not None:
                self.versions.load_versions(self.total_steps)

    def save(self):
        """Learner::Save (rank 0 writes; every rank holds the same weights)."""
        from . import checkpoint as _ckpt
        if not self.cfg.checkpoint_folder:
            raise ValueError("Learner.save: cfg.checkpoint_folder is not set")
        if self.rank == 0:
            self.last_checkpoint = _ckpt.save(self, self.cfg.checkpoint_folder, self.cfg.checkpoints_to_keep)
            if self.versions is not None:
                self.versions.save_versions()
        return self.last_checkpoint

    # ---------------------------------------------------------------- collection
    def collect(self):
        """T env steps: bf16 policy inference, fused env step + experience append."""
        import torch
        ppo, env = self.ppo, self.env
        for t in range(self.T):
            if self.old_version is None:
                ppo.infer_actions(self.obs[t], self.masks[t], step=self._rng_step, deterministic=self.cfg.deterministic,
                                  actions=self.actions[t], logp=self.logp[t])
            else:  # one team plays the old version (Learner.cpp:733-767)
                ppo.infer_actions_mixed(self.obs[t], self.masks[t], self._old_rows[self.old_team], step=self._rng_step,
                                        deterministic=self.cfg.deterministic, actions=self.actions[t],
                                        logp=self.logp[t])
            self._rng_step += 1
            if self.env_events is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
            env.step(self.actions[t], True,
                     StepOutputs.of(obs=self.obs[t + 1], masks=self.masks[t + 1], rewards=self.rewards[t],
                                    terminals=self.terms[t], trunc_obs=self.trunc_obs[t]))
            if self.env_events is not None:
                e1.record()
                self.env_events.append((e0, e1))

    # ---------------------------------------------------------------- consumption
    def consume(self):
        """InferCriticBatched over obs[0..T] and the truncation rows, GAE, return statistics."""
        import torch
        T, P = self.T, self.P
        self.ppo.infer_critic(self.obs.view(-1, OBS), out=self.values.view(-1))
        # truncation values only where a trajectory was truncated (code 2): InferCritic on the
        # truncated next-states (Learner.cpp:944); the other rows of trunc_vals are never read
        rows = torch.nonzero(self.terms.view(-1) == 2).squeeze(1)
        if rows.numel():
            tv = self.ppo.infer_critic(self.trunc_obs.view(-1, OBS).index_select(0, rows))
            self.trunc_vals.view(-1).index_copy_(0, rows, tv)
        std = self.return_stat.std()
        _gae.GAE.compute_rollout(self.rewards, self.terms, self.values[:T], self.trunc_vals, self.values[T],
                                 self.cfg.gamma, self.cfg.gae_lambda, std, self.cfg.reward_clip_range,
                                 adv=self.adv, target=self.target, ret=self.ret)
        # return-std Welford over randomly sampled returns (Learner.cpp:959-967)
        k = self.cfg.return_samples
        if self.old_version is None:
            idx = torch.from_numpy(self.rng.integers(0, T * P, size=k)).to(self.device)
        else:  # only the current policy's players have trajectories
            idx = self._train_rows()[torch.from_numpy(self.rng.integers(0, T * P // 2, size=k)).to(self.device)]
        samples = _dist.gather_samples(self.ret.view(-1)[idx], self.group)
        self.return_stat.add(samples.cpu().numpy())

    def _train_rows(self):
        """Sample indices (t * P + p) of the players on the current policy in an old-version iteration."""
        import torch
        new_team = 1 - self.old_team
        p = torch.arange(new_team, self.P, 2, device=self.device)
        t = torch.arange(self.T, device=self.device)
        return (t[:, None] * self.P + p[None, :]).reshape(-1).to(torch.int32)

    # ---------------------------------------------------------------- learning
    def learn(self):
        cfg, ppo = self.cfg, self.ppo
        rows = None if self.old_version is None else self._train_rows()
        M = self.T * self.P if rows is None else rows.numel()
        global_m = M * self.world
        batch = global_m if cfg.batch_size is None else cfg.batch_size
        obs = self.obs[:self.T].reshape(-1, OBS)
        masks = self.masks[:self.T].reshape(-1, ACTIONS)
        acts, logp = self.actions.view(-1), self.logp.view(-1)
        adv, tgt = self.adv.view(-1), self.target.view(-1)
        local_batch = M if cfg.batch_size is None else max(1, cfg.batch_size // self.world)
        for epoch in range(cfg.epochs):
            perm = permutation(M, cfg.seed + self.rank, self.iteration * cfg.epochs + epoch, device=self.device)
            if rows is not None:
                perm = rows[perm.long()]
            for b0, b1 in batch_ranges(M, local_batch, cfg.overbatching):
                # batch advantage normalisation (PPOLearner.cpp:360-371), global over ranks
                whole = rows is None and (b0, b1) == (0, M)
                badv = adv if whole else adv.index_select(0, perm[b0:b1].long())
                if self.world > 1:
                    ppo.adv_stats.copy_(_dist.global_mean_std(badv, self.group))
                else:
                    ppo.adv_normalizer(badv)
                for s0 in range(b0, b1, cfg.mini_batch_size):
                    n = min(cfg.mini_batch_size, b1 - s0)
                    ppo.minibatch(obs, masks, acts, logp, adv, tgt, perm, s0, n, batch)
                _dist.allreduce_grads(ppo.grads, self.group)  # RCCL over xGMI, before clip_grad_norm_
                ppo.optimizer_step()

    def iterate(self):
        """One PPO iteration (collect T steps, consume, learn); returns a report dict."""
        import torch
        t0 = time.perf_counter()
        self.old_version = None
        if self.versions is not None and self.versions.versions:  # Learner.cpp:587-627
            if self._vrng.random() < self.cfg.train_against_old_chance:
                self.old_version = self.versions.versions[int(self._vrng.integers(0, len(self.versions.versions)))]
                self.old_team = int(self._vrng.integers(0, 2))
                self.ppo.set_version(self.old_version.params)
        self.collect()
        self.consume()
        self.learn()
        # next rollout starts from the last obs
        self.obs[0].copy_(self.obs[self.T])
        self.masks[0].copy_(self.masks[self.T])
        self.iteration += 1
        prev = self.total_steps
        real_players = self.P if self.old_version is None else self.P // 2  # numRealPlayers (Learner.cpp:629)
        self.total_steps += self.T * real_players * self.world
        if self.versions is not None:
            self.versions.on_iteration(self.total_steps, prev)
        torch.cuda.synchronize(self.device)
        rep = {"iteration_s": time.perf_counter() - t0, "old_version": None if self.old_version is None
               else (self.old_version.timesteps, self.old_team)}
        if self.cfg.checkpoint_folder:  # auto-save (Learner.cpp:1011-1015)
            per = self.cfg.ts_per_save or self.T * self.P * self.world
            if self.total_steps // per > prev // per:
                rep["checkpoint"] = self.save()
        return rep
