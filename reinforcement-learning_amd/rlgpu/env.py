"""EnvSet -- Python mirror of RLGC::EnvSet (GigaLearnCPP/RLGymCPP/src/RLGymCPP/EnvSet/EnvSet.h:67-124)
over the C ABI of include/rlgpu_env.h.  Every arena lives in HBM; the state buffers
(obs, action masks, rewards, terminals) are exposed as torch tensors that alias the
library's device memory, so the policy reads observations without a copy.

Method map (reference -> here):
    EnvSet(config)          EnvSet.cpp:46-111    -> EnvSet(num_arenas, seed, tick_skip, action_delay)
    StepFirstHalf(async)    EnvSet.cpp:113-130   -> step_first_half()
    StepSecondHalf(a, async)EnvSet.cpp:132-273   -> step_second_half(actions)
    Sync()                  EnvSet.h:107         -> sync()
    Reset()                 EnvSet.cpp:331-354   -> reset()
    ResetArena(i)           EnvSet.cpp:275-329   -> reset_arenas(mask)
    state.obs / actionMasks / rewards / terminals EnvSet.h:35-65 -> .obs / .action_masks / ...
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import alias as _alias
from .state import ARENA, GAMESTATE

OBS, ACTIONS, REWARDS, PADS, CARS = 167, 90, 13, 34, 4


class _Config(ctypes.Structure):
    _fields_ = [("num_arenas", ctypes.c_int32), ("tick_skip", ctypes.c_int32), ("action_delay", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("save_rewards", ctypes.c_int32), ("max_episode_steps", ctypes.c_int32),
                ("mesh_tris", ctypes.c_void_p), ("mesh_ntris", ctypes.c_int32), ("mesh_objects", ctypes.c_int32),
                ("mesh_object_ntris", ctypes.c_void_p), ("rewards", ctypes.c_void_p), ("n_rewards", ctypes.c_int32),
                ("terminals", ctypes.c_void_p), ("n_terminals", ctypes.c_int32), ("arith", ctypes.c_int32),
                ("arena_offset", ctypes.c_int32), ("state_setter", ctypes.c_int32)]

# the reference build whose Bullet arithmetic the arenas follow (include/rlgpu_arith.h)
ARITH_MSVC_X64, ARITH_GCC_X64, ARITH_SCALAR = 0, 1, 2
# EnvCreateResult::stateSetter (include/rlgpu_env.h RLGPU_SS_*)
KICKOFF_STATE, FUZZED_KICKOFF_STATE = 0, 1


class StepOutputs(ctypes.Structure):
    """rlgpu_step_outputs: experience-append destinations of the fused step (device pointers)."""
    _fields_ = [("obs", ctypes.c_void_p), ("masks", ctypes.c_void_p), ("rewards", ctypes.c_void_p),
                ("terminals", ctypes.c_void_p), ("trunc_obs", ctypes.c_void_p)]

    @classmethod
    def of(cls, obs=None, masks=None, rewards=None, terminals=None, trunc_obs=None):
        for t, n in ((obs, "obs"), (masks, "masks"), (rewards, "rewards"), (terminals, "terminals"),
                     (trunc_obs, "trunc_obs")):
            _lib.require_gpu_tensor(t, n)
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        return cls(p(obs), p(masks), p(rewards), p(terminals), p(trunc_obs))


class _Buffers(ctypes.Structure):
    _fields_ = [("obs", ctypes.c_void_p), ("action_masks", ctypes.c_void_p), ("rewards", ctypes.c_void_p),
                ("terminals", ctypes.c_void_p), ("last_rewards", ctypes.c_void_p), ("trunc_obs", ctypes.c_void_p),
                ("num_players", ctypes.c_int32), ("num_arenas", ctypes.c_int32), ("num_rewards", ctypes.c_int32),
                ("arena_player_start", ctypes.c_void_p)]


_bound = False


def _bind():
    global _bound
    if _bound:
        return _lib.lib()
    L = _lib.lib()
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    L.rlgpu_envset_create.argtypes = [ctypes.POINTER(_Config), ctypes.POINTER(vp)]
    L.rlgpu_envset_destroy.argtypes = [vp]
    L.rlgpu_envset_buffers_get.argtypes = [vp, ctypes.POINTER(_Buffers)]
    L.rlgpu_envset_reset.argtypes = [vp, vp]
    L.rlgpu_envset_reset_arenas.argtypes = [vp, vp, vp]
    L.rlgpu_envset_step_first_half.argtypes = [vp, vp]
    L.rlgpu_envset_step_second_half.argtypes = [vp, vp, vp]
    L.rlgpu_envset_step.argtypes = [vp, vp, i32, ctypes.POINTER(StepOutputs), vp]
    L.rlgpu_envset_sync.argtypes = [vp, vp]
    L.rlgpu_envset_build_obs.argtypes = [vp, vp]
    L.rlgpu_envset_get_arenas.argtypes = [vp, i32, i32, vp]
    L.rlgpu_envset_set_arenas.argtypes = [vp, i32, i32, vp]
    L.rlgpu_step_metric_name.argtypes = [i32]
    L.rlgpu_step_metric_name.restype = ctypes.c_char_p
    L.rlgpu_envset_enable_step_metrics.argtypes = [vp, i32]
    L.rlgpu_envset_step_metrics.argtypes = [vp, vp, vp, i32, vp]
    L.rlgpu_envset_step_metric_slots.argtypes = [vp, vp, vp]
    L.rlgpu_envset_download_gamestates.argtypes = [vp, i32, i32, vp, vp]
    L.rlgpu_gamestates_from_arenas.argtypes = [vp, i32, i32, vp]
    L.rlgpu_envset_enable_reward_values.argtypes = [vp, i32]
    L.rlgpu_envset_reward_values.argtypes = [vp]
    L.rlgpu_envset_reward_values.restype = vp
    _bound = True
    return L


def arena_state_size():
    return _lib.lib().rlgpu_arena_state_size()


def gamestate_size():
    return _lib.lib().rlgpu_gamestate_size()


def gamestates_from_arenas(buf, tick_skip=8):
    """GameState records (numpy GAMESTATE array) of wire-format arena records (rlgpu_gamestates_from_arenas,
    GameState::UpdateFromArena on the record)."""
    L = _bind()
    buf = np.ascontiguousarray(buf, np.uint8)
    count = buf.size // ARENA.itemsize
    out = np.zeros(count, GAMESTATE)
    _lib.check(L.rlgpu_gamestates_from_arenas(buf.ctypes.data_as(ctypes.c_void_p), count, int(tick_skip),
                                              out.ctypes.data_as(ctypes.c_void_p)), "rlgpu_gamestates_from_arenas")
    return out


class EnvSet:
    """Vectorised 2v2 arena set resident in HBM (AdvancedObs, DefaultAction, KickoffState, and a
    reward / terminal list from the device registry -- ExampleMain's 13 rewards and NoTouch(8 s) +
    ScoreLimit(3) by default)."""

    def __init__(self, num_arenas, seed=1234, tick_skip=8, action_delay=7, save_rewards=True, device="cuda:0",
                 max_episode_steps=0, mesh=None, rewards=None, terminals=None, arith=ARITH_MSVC_X64, arena_offset=0,
                 state_setter=KICKOFF_STATE):
        """mesh: an rlgpu.mesh.ArenaMesh (e.g. ArenaMesh.from_folder("collision_meshes")), or None for
        the built-in synthetic arena mesh.  rewards / terminals: lists of rlgpu.plugins.reward(...) /
        terminal(...) specs (or structured arrays), None = ExampleMain's.  arith: the reference build
        whose Bullet arithmetic the step follows (ARITH_MSVC_X64 = build.ps1's, ARITH_GCC_X64, ARITH_SCALAR).
        arena_offset: global index of arena 0 for the arenas' random streams (a rank's first arena).
        state_setter: KICKOFF_STATE, or FUZZED_KICKOFF_STATE (the skill tracker's, rlgpu.skill)."""
        import torch
        if not torch.cuda.is_available():
            raise _lib.RLGPUError("EnvSet needs an MI355X: the product path has no CPU fallback")
        L = _bind()
        self.device = torch.device(device)
        torch.cuda.set_device(self.device)
        cfg = _Config(num_arenas, tick_skip, action_delay, seed, int(save_rewards), max_episode_steps)
        cfg.arith = int(arith)
        cfg.arena_offset = int(arena_offset)
        cfg.state_setter = int(state_setter)
        self.arith = int(arith)
        if mesh is not None:
            cfg.mesh_tris = mesh.tris.ctypes.data
            cfg.mesh_ntris = mesh.num_tris
            cfg.mesh_objects = mesh.num_objects
            cfg.mesh_object_ntris = mesh.object_ntris.ctypes.data
        from . import plugins
        # a non-NULL list pointer selects the given list, even an empty one (a 1-record buffer then)
        if rewards is not None:
            rw = rewards if isinstance(rewards, np.ndarray) else plugins.rewards_array(rewards)
            self._rw = np.ascontiguousarray(rw if rw.size else np.zeros(1, plugins.REWARD_SPEC))
            cfg.rewards, cfg.n_rewards = self._rw.ctypes.data, rw.size
        if terminals is not None:
            tc = terminals if isinstance(terminals, np.ndarray) else plugins.terminals_array(terminals)
            self._tc = np.ascontiguousarray(tc if tc.size else np.zeros(1, plugins.TERMINAL_SPEC))
            cfg.terminals, cfg.n_terminals = self._tc.ctypes.data, tc.size
        h = ctypes.c_void_p()
        _lib.check(L.rlgpu_envset_create(ctypes.byref(cfg), ctypes.byref(h)), "rlgpu_envset_create")
        self._h = h
        self.tick_skip, self.action_delay = tick_skip, action_delay
        self._alias_buffers(L)

    @classmethod
    def wrap(cls, handle, device, tick_skip=8, action_delay=7, owner=None):
        """An EnvSet view of a handle owned elsewhere (the C++ Learner's RLGC::EnvSetGPU)."""
        import torch
        L = _bind()
        self = cls.__new__(cls)
        self._h, self._owned, self._owner = ctypes.c_void_p(handle), False, owner
        self.device = torch.device(device)
        self.tick_skip, self.action_delay = tick_skip, action_delay
        self._alias_buffers(L)
        return self

    _owned = True

    def _alias_buffers(self, L):
        import torch
        b = _Buffers()
        _lib.check(L.rlgpu_envset_buffers_get(self._h, ctypes.byref(b)), "rlgpu_envset_buffers_get")
        self.num_arenas, self.num_players, self.num_rewards = b.num_arenas, b.num_players, b.num_rewards
        P, N, dev = b.num_players, b.num_arenas, self.device
        self.obs = _alias(b.obs, (P, OBS), torch.float32, dev)
        self.action_masks = _alias(b.action_masks, (P, ACTIONS), torch.uint8, dev)
        self.rewards = _alias(b.rewards, (P,), torch.float32, dev)
        self.terminals = _alias(b.terminals, (N,), torch.uint8, dev)
        self.last_rewards = _alias(b.last_rewards, (N, self.num_rewards), torch.float32, dev)
        self.trunc_obs = _alias(b.trunc_obs, (P, OBS), torch.float32, dev)
        self.arena_player_start = _alias(b.arena_player_start, (N,), torch.int32, dev)

    def close(self):
        if getattr(self, "_h", None):
            if self._owned:
                _lib.check(_lib.lib().rlgpu_envset_destroy(self._h), "rlgpu_envset_destroy")
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _actions(actions):
        import torch
        _lib.require_gpu_tensor(actions, "actions")
        if actions.dtype != torch.int32 or not actions.is_contiguous():
            raise _lib.RLGPUError("actions must be a contiguous int32 device tensor [num_players]")
        return _lib.ptr(actions)

    def step_first_half(self, stream=None):
        _lib.check(_lib.lib().rlgpu_envset_step_first_half(self._h, _lib.stream_ptr(stream)), "step_first_half")

    def step_second_half(self, actions, stream=None):
        _lib.check(_lib.lib().rlgpu_envset_step_second_half(self._h, self._actions(actions), _lib.stream_ptr(stream)),
                   "step_second_half")

    def step(self, actions, reset_terminated=True, out=None, stream=None):
        """Fused StepFirstHalf + StepSecondHalf (+ Reset of terminated arenas); `out` is a
        StepOutputs (experience append into rollout rows) or None."""
        o = ctypes.byref(out) if out is not None else None
        _lib.check(_lib.lib().rlgpu_envset_step(self._h, self._actions(actions), int(reset_terminated), o,
                                                _lib.stream_ptr(stream)), "rlgpu_envset_step")

    def set_output_only(self, on=True):
        """rlgpu_envset_set_output_only: rows given to step(out=...) go only there, not also to self.obs /
        self.action_masks / self.trunc_obs."""
        _lib.check(_lib.lib().rlgpu_envset_set_output_only(self._h, int(on)), "rlgpu_envset_set_output_only")

    def sync(self, stream=None):
        _lib.check(_lib.lib().rlgpu_envset_sync(self._h, _lib.stream_ptr(stream)), "sync")

    def reset(self, stream=None):
        _lib.check(_lib.lib().rlgpu_envset_reset(self._h, _lib.stream_ptr(stream)), "reset")

    def reset_arenas(self, mask=None, stream=None):
        _lib.require_gpu_tensor(mask, "mask")
        _lib.check(_lib.lib().rlgpu_envset_reset_arenas(self._h, _lib.ptr(mask), _lib.stream_ptr(stream)),
                   "reset_arenas")

    def build_obs(self, stream=None):
        _lib.check(_lib.lib().rlgpu_envset_build_obs(self._h, _lib.stream_ptr(stream)), "build_obs")

    def get_arenas(self, first=0, count=None):
        """Wire-format snapshot (uint8 [count * arena_state_size()]) of arenas [first, first+count)."""
        import torch
        torch.cuda.synchronize(self.device)
        count = self.num_arenas - first if count is None else count
        buf = np.zeros(count * ARENA.itemsize, np.uint8)
        _lib.check(_lib.lib().rlgpu_envset_get_arenas(self._h, first, count, buf.ctypes.data_as(ctypes.c_void_p)),
                   "get_arenas")
        return buf

    def set_arenas(self, buf, first=0):
        import torch
        torch.cuda.synchronize(self.device)
        buf = np.ascontiguousarray(buf, np.uint8)
        count = buf.size // ARENA.itemsize
        _lib.check(_lib.lib().rlgpu_envset_set_arenas(self._h, first, count, buf.ctypes.data_as(ctypes.c_void_p)),
                   "set_arenas")

    def gamestates(self, first=0, count=None, stream=None):
        """RLGC::GameState records (numpy GAMESTATE array, rlgpu.state) of arenas [first, first+count) as the
        last step left them: what the reference hands a StepCallbackFn (Learner.cpp:796-797)."""
        count = self.num_arenas - first if count is None else count
        out = np.zeros(count, GAMESTATE)
        _lib.check(_bind().rlgpu_envset_download_gamestates(self._h, first, count, out.ctypes.data_as(ctypes.c_void_p),
                                                            _lib.stream_ptr(stream)), "download_gamestates")
        return out

    def enable_reward_values(self, on=True):
        """Every later builders launch writes each reward's value before its weight: reward_values() is then
        a [num_players, num_rewards] device tensor (None while disabled)."""
        _lib.check(_bind().rlgpu_envset_enable_reward_values(self._h, int(on)), "enable_reward_values")

    def reward_values(self):
        import torch
        p = _bind().rlgpu_envset_reward_values(self._h)
        if not p:
            return None
        return _alias(p, (self.num_players, max(self.num_rewards, 1)), torch.float32, self.device)

    # ---- ExampleMain's StepCallback metrics (include/rlgpu_env.h rlgpu_envset_step_metrics)
    STEP_METRIC_SLOTS = 32

    @staticmethod
    def step_metric_names():
        L = _bind()
        return [L.rlgpu_step_metric_name(i).decode() for i in range(8)]

    def enable_step_metrics(self, on=True):
        """Every later builders launch (fused step / second half) is one StepCallback call."""
        _lib.check(_bind().rlgpu_envset_enable_step_metrics(self._h, int(on)), "enable_step_metrics")

    def step_metrics(self, reset=False, stream=None):
        """{Report key: (total, count)} since the last reset (Report::Avg, Report.h:11-45)."""
        tot, cnt = np.zeros(8, np.float64), np.zeros(8, np.uint64)
        _lib.check(_bind().rlgpu_envset_step_metrics(self._h, tot.ctypes.data_as(ctypes.c_void_p),
                                                     cnt.ctypes.data_as(ctypes.c_void_p), int(reset),
                                                     _lib.stream_ptr(stream)), "step_metrics")
        return {k: (float(t), int(c)) for k, t, c in zip(self.step_metric_names(), tot, cnt)}

    def step_metric_slots(self, stream=None):
        """The raw per-arena fp64 slots [num_arenas, 32]."""
        out = np.zeros((self.num_arenas, self.STEP_METRIC_SLOTS), np.float64)
        _lib.check(_bind().rlgpu_envset_step_metric_slots(self._h, out.ctypes.data_as(ctypes.c_void_p),
                                                          _lib.stream_ptr(stream)), "step_metric_slots")
        return out

    def serialize_arena(self, index):
        """RocketSim Arena::Serialize bytes of arena `index` (rlgpu.arena_wire)."""
        from . import arena_wire
        return arena_wire.envset_serialize(self, index)

    def deserialize_arena(self, index, data):
        """Arena::DeserializeNew of `data` into arena `index`; returns the bytes consumed (build_obs()
        refreshes the arena's obs / mask rows)."""
        from . import arena_wire
        return arena_wire.envset_deserialize(self, index, data)
