"""Learner -- Python binding of the C++ host Learner (reinforcement-learning_amd/host/learner.cpp,
include/rlgpu_learner.h): the GigaLearnCPP training loop for one GPU rank, every array resident
in HBM.

The loop itself (GGL::Learner::Start, GigaLearnCPP/src/public/GigaLearnCPP/Learner.cpp:482-1056)
is C++:
  collection   infer actions (bf16 policy) -> fused env step with experience append     :669-861
  consumption  critic over the rollout (InferCriticBatched), GAE, return-std Welford    :863-990
  learning     PPOLearner::Learn: epochs x shuffled minibatches, clip_grad_norm_, AdamW :990-1000
This module adds what sits around it in the reference: the config object, torch views of the
rollout buffers, checkpoints (rlgpu/checkpoint.py) and the old-version manager for self-play
(rlgpu/versions.py).  Distributed: the C++ Learner's exchanges go through rlgpu/dist.py's
TorchCollective (RCCL over xGMI on MI355X).

Experience layout ([T, P] time-major, P = 4 * arenas): the reference keeps per-player
trajectory vectors and trains only on finished trajectories (unfinished ones carry over to the
next iteration); here every collected step is trained in the iteration that collected it, with
the unfinished tail bootstrapped from V(obs_T) -- see DESIGN.md "Deviations".
"""
import ctypes
import time

import numpy as np

from . import _lib
from .ppo import MAX_LAYERS, NUM_METRICS

OBS, ACTIONS = 167, 90


# ------------------------------------------------------------------ host building blocks (C++)
def _host_lib():
    L = _lib.lib()
    i64p, f64p = ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)
    L.rlgpu_batch_ranges.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64]
    L.rlgpu_batch_ranges.restype = ctypes.c_int64
    L.rlgpu_welford_add.argtypes = [i64p, f64p, f64p, ctypes.c_void_p, ctypes.c_int64]
    L.rlgpu_welford_std.argtypes = [ctypes.c_int64, ctypes.c_double]
    L.rlgpu_welford_std.restype = ctypes.c_double
    L.rlgpu_sample_indices.argtypes = [ctypes.c_uint64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.c_void_p]
    L.rlgpu_sample_finished_rows.argtypes = [ctypes.c_uint64, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                                             ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                             ctypes.POINTER(ctypes.c_int32)]
    return L


class WelfordStat:
    """GGL::WelfordStat (Util/WelfordStat.h:7-67) -- the C++ implementation (host/learner.cpp),
    fp64 state in the reference's update order."""

    def __init__(self):
        self.n, self.mean, self.m2 = 0, 0.0, 0.0

    def add(self, xs):
        x = np.ascontiguousarray(np.asarray(xs, np.float32).ravel())
        c, m, s = ctypes.c_int64(self.n), ctypes.c_double(self.mean), ctypes.c_double(self.m2)
        _lib.check(_host_lib().rlgpu_welford_add(ctypes.byref(c), ctypes.byref(m), ctypes.byref(s), x.ctypes.data, x.size),
                   "rlgpu_welford_add")
        self.n, self.mean, self.m2 = c.value, m.value, s.value

    def get_mean(self):
        return 0.0 if self.n < 2 else self.mean

    def std(self):
        return _host_lib().rlgpu_welford_std(self.n, self.m2)

    def to_json(self):  # WelfordStat::ToJSON
        return {"mean": self.mean, "var": self.m2, "count": self.n}

    def read_json(self, j):  # WelfordStat::ReadFromJSON
        self.n, self.mean, self.m2 = int(j["count"]), float(j["mean"]), float(j["var"])


def host_uniform(seed, stream, counter):
    """rlgpu_host_uniform: the counter-based host draw of the self-play / skill-match picks (include/rlgpu_learner.h),
    the same in the C++ trainer facade."""
    L = _host_lib()
    L.rlgpu_host_uniform.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
    L.rlgpu_host_uniform.restype = ctypes.c_double
    return float(L.rlgpu_host_uniform(seed & (2**64 - 1), stream, counter))


def batch_ranges(exp_size, batch_size, overbatching=True):
    """ExperienceBuffer::GetAllBatchesShuffled batch boundaries (ExperienceBuffer.cpp:117-162),
    from the C++ ExperienceBuffer (GGL::BatchRanges)."""
    L = _host_lib()
    n = L.rlgpu_batch_ranges(exp_size, batch_size, int(overbatching), None, 0)
    out = np.zeros(2 * max(n, 1), np.int64)
    L.rlgpu_batch_ranges(exp_size, batch_size, int(overbatching), out.ctypes.data, n)
    return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(n)]


def sample_indices(seed, rank, iteration, rng, n):
    """rlgpu_sample_indices: the return-sample draws of one iteration."""
    out = np.zeros(max(n, 1), np.int64)
    _lib.check(_host_lib().rlgpu_sample_indices(seed, rank, iteration, rng, n, out.ctypes.data), "rlgpu_sample_indices")
    return out[:n]


def last_ends(terms):
    """Per column of a [T, P] trajectory-code array: the last step with a nonzero code, -1 if none."""
    t = np.asarray(terms)
    nz = t != 0
    T = t.shape[0]
    last = T - 1 - np.argmax(nz[::-1], axis=0)
    return np.where(nz.any(axis=0), last, -1).astype(np.int32)


def sample_finished_rows(seed, rank, iteration, ends, n):
    """rlgpu_sample_finished_rows: the return-sample rows t * P + p (t <= ends[p]) of one iteration,
    drawn from finished trajectories only (Learner.cpp:823-861, 959-967)."""
    e = np.ascontiguousarray(ends, np.int32)
    out = np.zeros(max(n, 1), np.int64)
    m = ctypes.c_int32()
    _lib.check(_host_lib().rlgpu_sample_finished_rows(seed, rank, iteration, e.ctypes.data, e.size, n, out.ctypes.data,
                                                      ctypes.byref(m)), "rlgpu_sample_finished_rows")
    return out[:m.value]


def sync_from_rank0(learner, group=None, error=None):
    """Every rank takes rank 0's training state: parameters, AdamW moments and step, step counters,
    return statistics and the old policy versions.  Only rank 0 reads the checkpoint folder
    (Learner.cpp:145-153 loads in the single-process reference); the ranks need not share a
    filesystem, and replicas can never start diverged.  `error`: rank 0's load failure -- the
    header carries it first, so every rank raises together instead of waiting in a broadcast rank 0
    never reaches."""
    import torch
    from .dist import broadcast_
    st = learner._stats()
    ppo = learner.ppo
    step, m, v = ppo.optimizer_state()
    vers = learner.versions.versions if learner.versions is not None else []
    hdr = torch.tensor([float(error is None), float(learner.last_checkpoint is not None), st.total_steps,
                        st.iteration, st.return_n, st.return_mean, st.return_m2, step, len(vers)], dtype=torch.float64)
    broadcast_(hdr, group)
    ok, loaded, total, it, rn, rmean, rm2, step, nv = hdr.tolist()
    if not ok:
        raise RuntimeError(f"rank 0 failed to load the checkpoint: {error!r}" if error is not None else
                           "rank 0 failed to load the checkpoint (see its log)")
    if loaded:
        for t in (ppo.params, m, v):
            broadcast_(t, group)
        st.total_steps, st.iteration, st.return_n = int(total), int(it), int(rn)
        st.return_mean, st.return_m2 = rmean, rm2
        learner._set_stats(st)
        ppo.set_optimizer_step(int(step))
        ppo.refresh_half()
    # old versions whenever rank 0 holds any (policy_versions/ may exist without a checkpoint)
    if learner.versions is not None and int(nv) > 0:
        ts = torch.tensor([float(x.timesteps) for x in vers] if vers else [0.0] * int(nv), dtype=torch.float64)
        broadcast_(ts, group)
        like = ppo.policy_version()
        params = [x.params for x in vers] if vers else [torch.empty_like(like) for _ in range(int(nv))]
        for t in params:
            broadcast_(t, group)
        if not vers:
            for k, t in enumerate(params):
                learner.versions.add_version(int(ts[k]), t)


# ------------------------------------------------------------------ config
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
        self.shared_layers = ()            # PPOLearnerConfig::sharedHead ((384, 384) in the reference's run log)
        self.experience_mode = 0           # 0: fixed [T, P] rollout; 1: the reference's complete trajectories
                                           # with carry-over (rlgpu_learner_config.experience_mode)
        self.ts_per_itr = 0                # mode 1: PPOLearnerConfig::tsPerItr (0 = rollout_len * players)
        self.experience_capacity = 0       # mode 1: per-player step store rows (0 = automatic)
        self.arith = 0                     # the reference build's Bullet arithmetic (rlgpu.arith; 0 = MSVC x64)
        self.rewards = None                # EnvCreateFn reward list (rlgpu.plugins.reward specs); None = ExampleMain's
        self.terminals = None              # terminal conditions (rlgpu.plugins.terminal specs); None = ExampleMain's
        self.mesh = None                   # arena collision meshes (rlgpu.mesh.ArenaMesh); None = the built-in synthetic arena
        self.max_episode_duration = 300.0  # seconds (ExampleMain)
        self.deterministic = False
        self.train_gemm = 2               # rlgpu_ppo_config.train_gemm: 2 = f32 via scaled fp16 split (H3), 0 = bf16 x6 split, 1 = f32 MFMA
        self.infer_fp16 = False           # rlgpu_ppo_config.infer_fp16: fp16 inference copy (C5) instead of bf16
        self.frame_stack = 1              # K >= 2: stacked AdvancedObs frames (C4; no reference counterpart)
        self.collect_groups = 0           # rollout collection in arena groups on their own streams (0 = automatic)
        # checkpoints (LearnerConfig.h:31-38): None = no save / load
        self.checkpoint_folder = None
        self.ts_per_save = 10_000_000     # 0 = every iteration (Learner.cpp:44-45)
        self.checkpoints_to_keep = 8      # -1 keeps all
        # self-play against old policy versions (LearnerConfig.h:62-68)
        self.train_against_old_versions = True
        self.train_against_old_chance = 0.15
        self.ts_per_version = 25_000_000
        self.max_old_versions = 32
        # ELO skill matches against the old versions (LearnerConfig.h:70, SkillTrackerConfig.h): a
        # rlgpu.skill.SkillTrackerConfig, or None = disabled
        self.skill_tracker = None
        for k, v in kw.items():
            if not hasattr(self, k):
                raise AttributeError(f"unknown LearnerConfig field {k}")
            setattr(self, k, v)


class _CConfig(ctypes.Structure):
    """rlgpu_learner_config (include/rlgpu_learner.h)."""
    _fields_ = [("num_arenas", ctypes.c_int32), ("tick_skip", ctypes.c_int32), ("action_delay", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("max_episode_duration", ctypes.c_float),
                ("rollout_len", ctypes.c_int32), ("epochs", ctypes.c_int32), ("mini_batch_size", ctypes.c_int32),
                ("batch_size", ctypes.c_int64), ("overbatching", ctypes.c_int32),
                ("gamma", ctypes.c_float), ("gae_lambda", ctypes.c_float), ("clip_range", ctypes.c_float),
                ("entropy_scale", ctypes.c_float), ("policy_lr", ctypes.c_float), ("critic_lr", ctypes.c_float),
                ("reward_clip_range", ctypes.c_float), ("return_samples", ctypes.c_int32),
                ("policy_layers", ctypes.c_int32 * MAX_LAYERS), ("n_policy_layers", ctypes.c_int32),
                ("critic_layers", ctypes.c_int32 * MAX_LAYERS), ("n_critic_layers", ctypes.c_int32),
                ("deterministic", ctypes.c_int32), ("train_gemm", ctypes.c_int32), ("infer_fp16", ctypes.c_int32),
                ("frame_stack", ctypes.c_int32), ("rank", ctypes.c_int32), ("world", ctypes.c_int32),
                ("mesh_tris", ctypes.c_void_p), ("mesh_ntris", ctypes.c_int32), ("mesh_objects", ctypes.c_int32),
                ("mesh_object_ntris", ctypes.c_void_p),
                ("shared_layers", ctypes.c_int32 * MAX_LAYERS), ("n_shared_layers", ctypes.c_int32),
                ("rewards", ctypes.c_void_p), ("n_rewards", ctypes.c_int32),
                ("terminals", ctypes.c_void_p), ("n_terminals", ctypes.c_int32),
                ("experience_mode", ctypes.c_int32), ("ts_per_itr", ctypes.c_int64),
                ("experience_capacity", ctypes.c_int32), ("arith", ctypes.c_int32),
                ("activation", ctypes.c_int32), ("optimizer", ctypes.c_int32), ("collect_groups", ctypes.c_int32)]


class _CBatch(ctypes.Structure):
    """rlgpu_batch_view (include/rlgpu_learner.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("obs", "masks", "actions", "logp", "rewards", "terms", "values", "adv",
                                               "target", "ret")] + \
               [("num_rows", ctypes.c_int64), ("trunc_obs", ctypes.c_void_p), ("trunc_vals", ctypes.c_void_p),
                ("num_truncs", ctypes.c_int64)] + \
               [(n, ctypes.c_void_p) for n in ("seg_player", "seg_start", "seg_len", "seg_code", "seg_tidx", "seg_off")] + \
               [("num_segments", ctypes.c_int64), ("store_rows", ctypes.c_int32), ("steps", ctypes.c_int32),
                ("first_step", ctypes.c_int64)]


class _CRollout(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("obs", "masks", "actions", "logp", "rewards", "terms", "trunc_obs",
                                               "values", "trunc_vals", "adv", "target", "ret")] + \
               [("T", ctypes.c_int32), ("P", ctypes.c_int32), ("obs_width", ctypes.c_int32)]


class _CStats(ctypes.Structure):
    _fields_ = [("total_steps", ctypes.c_int64), ("iteration", ctypes.c_int64), ("return_n", ctypes.c_int64),
                ("return_mean", ctypes.c_double), ("return_m2", ctypes.c_double), ("rng_step", ctypes.c_int64)]


class _CReport(ctypes.Structure):
    _fields_ = [("collect_s", ctypes.c_double), ("consume_s", ctypes.c_double), ("learn_s", ctypes.c_double),
                ("env_kernel_ms", ctypes.c_double), ("env_steps", ctypes.c_int64), ("learn_issue_s", ctypes.c_double),
                ("collect_issue_s", ctypes.c_double), ("env_launch_arenas", ctypes.c_int32),
                ("env_kernel_min_ms", ctypes.c_double), ("env_kernel_median_ms", ctypes.c_double),
                ("env_kernel_max_ms", ctypes.c_double)]


def _bind():
    L = _lib.lib()
    vp = ctypes.c_void_p
    L.rlgpu_learner_create.argtypes = [ctypes.POINTER(_CConfig), vp, vp, ctypes.POINTER(vp)]
    L.rlgpu_learner_destroy.argtypes = [vp]
    L.rlgpu_learner_handles.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.rlgpu_learner_rollout.argtypes = [vp, ctypes.POINTER(_CRollout)]
    L.rlgpu_learner_batch.argtypes = [vp, ctypes.POINTER(_CBatch)]
    L.rlgpu_learner_iterate.argtypes = [vp, ctypes.POINTER(_CReport)]
    for f in ("collect", "consume", "learn", "finish_iteration"):
        getattr(L, "rlgpu_learner_" + f).argtypes = [vp]
    L.rlgpu_learner_set_old_team.argtypes = [vp, ctypes.c_int32]
    L.rlgpu_learner_get_stats.argtypes = [vp, ctypes.POINTER(_CStats)]
    L.rlgpu_learner_set_stats.argtypes = [vp, ctypes.POINTER(_CStats)]
    L.rlgpu_learner_metrics.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_int64), ctypes.c_int32]
    L.rlgpu_learner_set_env_timing.argtypes = [vp, ctypes.c_int32]
    L.rlgpu_learner_step_metrics.argtypes = [vp, vp, vp, ctypes.c_int32]
    return L


class _ReturnStat:
    """The C++ Learner's return-std WelfordStat, seen through get/set_stats (checkpoint JSON)."""

    def __init__(self, learner):
        self._L = learner

    n = property(lambda self: self._L._stats().return_n)
    mean = property(lambda self: self._L._stats().return_mean)
    m2 = property(lambda self: self._L._stats().return_m2)

    def std(self):
        return _host_lib().rlgpu_welford_std(self.n, self.m2)

    def to_json(self):
        return {"mean": self.mean, "var": self.m2, "count": self.n}

    def read_json(self, j):
        st = self._L._stats()
        st.return_n, st.return_mean, st.return_m2 = int(j["count"]), float(j["mean"]), float(j["var"])
        self._L._set_stats(st)


class Learner:
    """GGL::Learner for one rank (the C++ host Learner) with torch views of its HBM rollout."""

    def __init__(self, cfg, device="cuda:0", rank=0, world=1, group=None, native_rccl=False):
        """world > 1: the C++ Learner's exchanges go through rlgpu.dist.TorchCollective (torch.distributed,
        RCCL for the nccl backend), or with native_rccl through its own RCCL communicator
        (rlgpu.dist.RcclCollective: no Python in the exchange path)."""
        import torch
        from .env import EnvSet
        from .ppo import PPO
        if not torch.cuda.is_available():
            raise _lib.RLGPUError("Learner needs an MI355X: the product path has no CPU fallback")
        self.cfg, self.rank, self.world, self.group = cfg, rank, world, group
        self.device = torch.device(device)
        torch.cuda.set_device(self.device)
        L = _bind()
        c = _CConfig()
        c.num_arenas, c.tick_skip, c.action_delay, c.seed = cfg.num_arenas, cfg.tick_skip, cfg.action_delay, cfg.seed
        c.max_episode_duration, c.rollout_len, c.epochs = cfg.max_episode_duration, cfg.rollout_len, cfg.epochs
        c.mini_batch_size = cfg.mini_batch_size
        c.batch_size = 0 if cfg.batch_size is None else cfg.batch_size
        c.overbatching = int(cfg.overbatching)
        c.gamma, c.gae_lambda, c.clip_range, c.entropy_scale = cfg.gamma, cfg.gae_lambda, cfg.clip_range, cfg.entropy_scale
        c.policy_lr, c.critic_lr, c.reward_clip_range = cfg.policy_lr, cfg.critic_lr, cfg.reward_clip_range
        c.return_samples = cfg.return_samples
        for i, v in enumerate(cfg.policy_layers):
            c.policy_layers[i] = v
        for i, v in enumerate(cfg.critic_layers):
            c.critic_layers[i] = v
        c.n_policy_layers, c.n_critic_layers = len(cfg.policy_layers), len(cfg.critic_layers)
        for i, v in enumerate(cfg.shared_layers):
            c.shared_layers[i] = v
        c.n_shared_layers = len(cfg.shared_layers)
        from . import plugins
        if cfg.rewards is not None:
            rw = plugins.rewards_array(cfg.rewards)
            self._rw = np.ascontiguousarray(rw if rw.size else np.zeros(1, plugins.REWARD_SPEC))
            c.rewards, c.n_rewards = self._rw.ctypes.data, rw.size
        if cfg.terminals is not None:
            tc = plugins.terminals_array(cfg.terminals)
            self._tc = np.ascontiguousarray(tc if tc.size else np.zeros(1, plugins.TERMINAL_SPEC))
            c.terminals, c.n_terminals = self._tc.ctypes.data, tc.size
        if cfg.mesh is not None:  # copied by the env set at create
            self._mesh = cfg.mesh
            c.mesh_tris, c.mesh_ntris = cfg.mesh.tris.ctypes.data, cfg.mesh.num_tris
            c.mesh_objects, c.mesh_object_ntris = cfg.mesh.num_objects, cfg.mesh.object_ntris.ctypes.data
        c.deterministic, c.train_gemm, c.infer_fp16 = int(cfg.deterministic), cfg.train_gemm, int(cfg.infer_fp16)
        c.frame_stack = cfg.frame_stack
        c.experience_mode, c.ts_per_itr, c.experience_capacity = cfg.experience_mode, cfg.ts_per_itr, cfg.experience_capacity
        c.arith = cfg.arith
        c.collect_groups = cfg.collect_groups
        c.rank, c.world = rank, world
        self._coll = None
        coll = None
        if world > 1:
            if native_rccl:
                from .dist import RcclCollective
                self._coll = RcclCollective(rank, world, group=group)
            else:
                from .dist import TorchCollective
                self._coll = TorchCollective(group, self.device)
            coll = ctypes.byref(self._coll.c_struct())
        h = ctypes.c_void_p()
        _lib.check(L.rlgpu_learner_create(ctypes.byref(c), coll, _lib.stream_ptr(), ctypes.byref(h)),
                   "rlgpu_learner_create")
        self._h = h
        eh, ph = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(L.rlgpu_learner_handles(h, ctypes.byref(eh), ctypes.byref(ph)), "rlgpu_learner_handles")
        self.env = EnvSet.wrap(eh.value, self.device, cfg.tick_skip, cfg.action_delay, owner=self)
        rows_cap = cfg.mini_batch_size if cfg.experience_mode == 1 else cfg.rollout_len * 4 * cfg.num_arenas
        max_rows = max(min(cfg.mini_batch_size, rows_cap), min(4 * cfg.num_arenas, 65536))  # host/learner.cpp
        self.ppo = PPO.wrap(ph.value, self.device, cfg.policy_layers, cfg.critic_layers, max_rows,
                            obs_size=OBS * max(1, cfg.frame_stack), metrics_source=self._metrics, owner=self,
                            shared_layers=cfg.shared_layers,
                            optim_options={"lr": (cfg.policy_lr, cfg.critic_lr, min(cfg.policy_lr, cfg.critic_lr)),
                                           "betas": (0.9, 0.999), "eps": 1e-8, "weight_decay": 1e-2})
        r = _CRollout()
        _lib.check(L.rlgpu_learner_rollout(h, ctypes.byref(r)), "rlgpu_learner_rollout")
        T, P, W = r.T, r.P, r.obs_width
        self.T, self.P, self.W = T, P, W
        a, f32, u8, i32, i8 = _lib.alias, torch.float32, torch.uint8, torch.int32, torch.int8
        d = self.device
        self.obs = a(r.obs, (T + 1, P, W), f32, d)
        self.masks = a(r.masks, (T + 1, P, ACTIONS), u8, d)
        self.actions = a(r.actions, (T, P), i32, d)
        self.logp = a(r.logp, (T, P), f32, d)
        self.rewards = a(r.rewards, (T, P), f32, d)
        self.terms = a(r.terms, (T, P), i8, d)
        self.trunc_obs = a(r.trunc_obs, (T, P, W), f32, d)
        self.values = a(r.values, (T + 1, P), f32, d)
        self.trunc_vals = a(r.trunc_vals, (T, P), f32, d)
        self.adv = a(r.adv, (T, P), f32, d)
        self.target = a(r.target, (T, P), f32, d)
        self.ret = a(r.ret, (T, P), f32, d)
        self.return_stat = _ReturnStat(self)
        # old-version player rows: team of player p is p % 2 (cars 0, 2 blue; 1, 3 orange)
        team = torch.arange(P, device=d) % 2
        self._old_rows = [(team == k).to(torch.uint8) for k in range(2)]
        # self-play: the manager of old versions, this iteration's version and team (None = all
        # players use the current policy); the draw is rank-independent so every rank agrees
        self.versions = None
        self.old_version, self.old_team = None, 0
        self.skill = None
        # rank 0 plays the skill matches (ratings are a report; every rank holds the same versions)
        if cfg.skill_tracker is not None and cfg.skill_tracker.enabled and rank == 0:  # PolicyVersionManager.cpp:24-31
            from .skill import SkillTracker
            self.skill = SkillTracker(cfg.skill_tracker, self.ppo, self.device, cfg.tick_skip, cfg.action_delay,
                                      seed=cfg.seed, mesh=cfg.mesh, arith=cfg.arith)
        if cfg.train_against_old_versions or self.skill is not None:  # Learner.cpp:131-142
            import os
            from .versions import PolicyVersionManager
            vf = os.path.join(cfg.checkpoint_folder, "policy_versions") if cfg.checkpoint_folder else None
            self.versions = PolicyVersionManager(self.ppo, vf, cfg.max_old_versions, cfg.ts_per_version, self.skill)
        self.last_checkpoint = None
        if cfg.checkpoint_folder:  # Learner ctor: load the most recent checkpoint (Learner.cpp:145-153)
            from . import checkpoint as _ckpt
            err = None
            if rank == 0:  # rank 0 reads the folder, every other rank receives its state
                try:
                    self.last_checkpoint = _ckpt.load(self, cfg.checkpoint_folder)
                    if self.versions is not None:
                        self.versions.load_versions(self.total_steps)
                except Exception as e:  # noqa: BLE001 -- re-raised below, on every rank
                    err = e
            if world > 1:
                sync_from_rank0(self, group, err)
            elif err is not None:
                raise err

    def close(self):
        if getattr(self, "_h", None):
            import torch
            torch.cuda.synchronize(self.device)
            if self.skill is not None:
                self.skill.close()
            self.env.close()
            self.ppo.close()
            _lib.check(_lib.lib().rlgpu_learner_destroy(self._h), "rlgpu_learner_destroy")
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- state
    def _stats(self):
        st = _CStats()
        _lib.check(_lib.lib().rlgpu_learner_get_stats(self._h, ctypes.byref(st)), "rlgpu_learner_get_stats")
        return st

    def _set_stats(self, st):
        _lib.check(_lib.lib().rlgpu_learner_set_stats(self._h, ctypes.byref(st)), "rlgpu_learner_set_stats")

    def _set_stat(self, name, v):
        st = self._stats()
        setattr(st, name, int(v))
        self._set_stats(st)

    total_steps = property(lambda self: self._stats().total_steps, lambda self, v: self._set_stat("total_steps", v))
    iteration = property(lambda self: self._stats().iteration, lambda self, v: self._set_stat("iteration", v))

    def _metrics(self, reset):
        out = np.zeros(NUM_METRICS, np.float32)
        cnt = ctypes.c_int64()
        _lib.check(_lib.lib().rlgpu_learner_metrics(self._h, out.ctypes.data, ctypes.byref(cnt), int(reset)),
                   "rlgpu_learner_metrics")
        return out.tolist(), cnt.value

    def step_metrics(self, reset=True):
        """ExampleMain's StepCallback report (ExampleMain.cpp:233-283): {key: average} over the
        collection steps since the last reset (keys without samples are left out, as a Report without
        that AddAvg)."""
        import numpy as np
        from .env import EnvSet
        tot, cnt = np.zeros(8, np.float64), np.zeros(8, np.uint64)
        _lib.check(_lib.lib().rlgpu_learner_step_metrics(self._h, tot.ctypes.data, cnt.ctypes.data, int(reset)),
                   "rlgpu_learner_step_metrics")
        return {k: float(t) / int(c) for k, t, c in zip(EnvSet.step_metric_names(), tot, cnt) if c}

    _HOOK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32)
    _GRAD_HOOK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                  ctypes.c_int32)

    def set_step_hook(self, fn):
        """rlgpu_learner_set_step_hook: fn(phase) after every collection step (0: post-step, pre-reset -- it may
        rewrite self.env's rewards / terminals; 1: after the arenas whose terminal is set were reset); None restores
        the fused step.  An exception in fn fails the iteration."""
        L = _lib.lib()
        if fn is None:
            self._hook = None
            _lib.check(L.rlgpu_learner_set_step_hook(self._h, None, None), "rlgpu_learner_set_step_hook")
            return

        def thunk(_user, phase):
            try:
                fn(int(phase))
                return 0
            except Exception:  # noqa: BLE001 -- reported by the iteration's failure
                import traceback
                traceback.print_exc()
                return 1
        self._hook = self._HOOK(thunk)  # kept alive with the learner
        L.rlgpu_learner_set_step_hook.argtypes = [ctypes.c_void_p, self._HOOK, ctypes.c_void_p]
        _lib.check(L.rlgpu_learner_set_step_hook(self._h, self._hook, None), "rlgpu_learner_set_step_hook")

    def set_grad_hook(self, fn):
        """rlgpu_learner_set_grad_hook: fn(grads, epoch, batch) after each batch's gradient all-reduce, before
        clip_grad_norm_ / AdamW; grads is a torch view of the flat fp32 gradient in HBM (valid during the call,
        read-only).  None removes the tap.  An exception in fn fails the iteration."""
        import torch
        from ._lib import alias
        L = _lib.lib()
        if fn is None:
            self._ghook = None
            _lib.check(L.rlgpu_learner_set_grad_hook(self._h, None, None), "rlgpu_learner_set_grad_hook")
            return

        def thunk(_user, ptr, n, epoch, batch):
            try:
                fn(alias(ptr, (n,), torch.float32, self.device), int(epoch), int(batch))
                return 0
            except Exception:  # noqa: BLE001 -- reported by the iteration's failure
                import traceback
                traceback.print_exc()
                return 1
        self._ghook = self._GRAD_HOOK(thunk)
        L.rlgpu_learner_set_grad_hook.argtypes = [ctypes.c_void_p, self._GRAD_HOOK, ctypes.c_void_p]
        _lib.check(L.rlgpu_learner_set_grad_hook(self._h, self._ghook, None), "rlgpu_learner_set_grad_hook")

    def set_env_timing(self, on=True):
        _lib.check(_lib.lib().rlgpu_learner_set_env_timing(self._h, int(on)), "rlgpu_learner_set_env_timing")

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

    # ---------------------------------------------------------------- phases (C++)
    def collect(self):
        """T env steps: bf16 policy inference, fused env step + experience append."""
        _lib.check(_lib.lib().rlgpu_learner_collect(self._h), "rlgpu_learner_collect")

    def consume(self):
        """InferCriticBatched over obs[0..T] and the truncation rows, GAE, return statistics."""
        _lib.check(_lib.lib().rlgpu_learner_consume(self._h), "rlgpu_learner_consume")

    def learn(self):
        _lib.check(_lib.lib().rlgpu_learner_learn(self._h), "rlgpu_learner_learn")

    def batch(self):
        """The trained batch of experience_mode 1 (after consume): combined complete trajectories,
        their values / GAE outputs, the truncation list and the trajectory records, as torch views."""
        import torch
        b = _CBatch()
        _lib.check(_lib.lib().rlgpu_learner_batch(self._h, ctypes.byref(b)), "rlgpu_learner_batch")
        d, M, K, nt, W = self.device, max(b.num_rows, 1), max(b.num_segments, 1), max(b.num_truncs, 1), self.W

        def a(ptr, shape, dtype, dev):  # arrays are allocated at the first consume
            return _lib.alias(ptr, shape, dtype, dev) if ptr else torch.empty((0,) + tuple(shape[1:]), dtype=dtype, device=dev)
        f32, i32 = torch.float32, torch.int32
        out = {"obs": a(b.obs, (M, W), f32, d), "masks": a(b.masks, (M, ACTIONS), torch.uint8, d),
               "actions": a(b.actions, (M,), i32, d), "logp": a(b.logp, (M,), f32, d),
               "rewards": a(b.rewards, (M,), f32, d), "terms": a(b.terms, (M,), torch.int8, d),
               "values": a(b.values, (M,), f32, d), "adv": a(b.adv, (M,), f32, d), "target": a(b.target, (M,), f32, d),
               "ret": a(b.ret, (M,), f32, d), "trunc_obs": a(b.trunc_obs, (nt, W), f32, d),
               "trunc_vals": a(b.trunc_vals, (nt,), f32, d)}
        for k in ("seg_player", "seg_start", "seg_len", "seg_code", "seg_tidx"):
            out[k] = a(getattr(b, k), (K,), i32, d)[:b.num_segments]
        out["seg_off"] = a(b.seg_off, (K,), torch.int64, d)[:b.num_segments]
        for k in ("obs", "masks", "actions", "logp", "rewards", "terms", "values", "adv", "target", "ret"):
            out[k] = out[k][:b.num_rows]
        out["trunc_obs"], out["trunc_vals"] = out["trunc_obs"][:b.num_truncs], out["trunc_vals"][:b.num_truncs]
        out.update(num_rows=b.num_rows, num_truncs=b.num_truncs, num_segments=b.num_segments, store_rows=b.store_rows,
                   steps=b.steps, first_step=b.first_step)
        return out

    def finish_iteration(self):
        _lib.check(_lib.lib().rlgpu_learner_finish_iteration(self._h), "rlgpu_learner_finish_iteration")

    def iterate(self):
        """One PPO iteration (collect T steps, consume, learn); returns a report dict."""
        import torch
        t0 = time.perf_counter()
        self.old_version = None
        if self.cfg.train_against_old_versions and self.versions is not None and self.versions.versions:  # Learner.cpp:587-627
            it, n = self.iteration, len(self.versions.versions)
            if host_uniform(self.cfg.seed, 1, 3 * it) < self.cfg.train_against_old_chance:  # the C++ facade's picks
                self.old_version = self.versions.versions[min(n - 1, int(host_uniform(self.cfg.seed, 1, 3 * it + 1) * n))]
                self.old_team = min(1, int(host_uniform(self.cfg.seed, 1, 3 * it + 2) * 2))
                self.ppo.set_version(self.old_version.params)
        team = -1 if self.old_version is None else self.old_team
        _lib.check(_lib.lib().rlgpu_learner_set_old_team(self._h, team), "rlgpu_learner_set_old_team")
        prev = self.total_steps
        rep = _CReport()
        _lib.check(_lib.lib().rlgpu_learner_iterate(self._h, ctypes.byref(rep)), "rlgpu_learner_iterate")
        report = {}
        if self.versions is not None:
            self.versions.on_iteration(self.total_steps, prev, report)
        torch.cuda.synchronize(self.device)
        out = {"report": report, "iteration_s": time.perf_counter() - t0, "collect_s": rep.collect_s, "consume_s": rep.consume_s,
               "learn_s": rep.learn_s, "learn_issue_s": rep.learn_issue_s, "collect_issue_s": rep.collect_issue_s, "env_kernel_ms": rep.env_kernel_ms,
               "env_launch_arenas": rep.env_launch_arenas, "env_kernel_min_ms": rep.env_kernel_min_ms,
               "env_kernel_median_ms": rep.env_kernel_median_ms, "env_kernel_max_ms": rep.env_kernel_max_ms,
               "old_version": None if self.old_version is None else (self.old_version.timesteps, self.old_team)}
        if self.cfg.checkpoint_folder:  # auto-save (Learner.cpp:1011-1015)
            per = self.cfg.ts_per_save or self.T * self.P * self.world
            if self.total_steps // per > prev // per:
                out["checkpoint"] = self.save()
        return out
