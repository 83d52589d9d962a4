"""GAE -- mirror of GGL::GAE::Compute (GigaLearnCPP/src/private/GigaLearnCPP/PPO/GAE.h:9-13).

`GAE.compute` takes and returns device tensors and runs the HIP kernels in
csrc/gae.hip through the C ABI (include/rlgpu_gae.h).
"""
import ctypes
import functools

import torch

from . import _lib
from ._lib import check, lib, ptr, require_gpu_tensor, stream_ptr

TERMINAL_NOT = 0
TERMINAL_NORMAL = 1      # RLGC::TerminalType::NORMAL (TerminalCondition.h:8)
TERMINAL_TRUNCATED = 2   # RLGC::TerminalType::TRUNCATED (TerminalCondition.h:9)


@functools.lru_cache(maxsize=None)
def _sig():  # the prototypes, set once
    L = lib()
    f = L.rlgpu_gae_flat
    f.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_int64] + [ctypes.c_float] * 4 + \
        [ctypes.c_void_p] * 3 + [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p]
    g = L.rlgpu_gae_rollout
    g.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int32, ctypes.c_int32] + [ctypes.c_float] * 4 + \
        [ctypes.c_void_p] * 4 + [ctypes.c_void_p]
    return f, g


class GAE:
    @staticmethod
    def compute(rews, terminals, val_preds, trunc_val_preds, gamma, lam, return_std, clip_range):
        """Flat (episode-concatenated) GAE. Returns (advantages, target_values, returns, rew_clip_portion).

        Argument meaning and order follow GAE::Compute (GAE.cpp:7-11)."""
        for n, t in (("rews", rews), ("terminals", terminals), ("val_preds", val_preds),
                     ("trunc_val_preds", trunc_val_preds)):
            require_gpu_tensor(t, n)
        rews = rews.contiguous().float()
        terminals = terminals.contiguous().to(torch.int8)
        val_preds = val_preds.contiguous().float()
        n = rews.numel()
        nt = 0 if trunc_val_preds is None else trunc_val_preds.numel()
        tv = None if trunc_val_preds is None else trunc_val_preds.contiguous().float()
        # one allocation; rows padded to 4 floats so each output starts 16-byte aligned (the kernels' float4 path)
        adv, tgt, ret = torch.empty((3, (n + 3) // 4 * 4), dtype=torch.float32, device=rews.device)[:, :n]
        clip = ctypes.c_float(0.0)
        f, _ = _sig()
        check(f(ptr(rews), ptr(terminals), ptr(val_preds), ptr(tv), n, nt, gamma, lam, return_std,
                clip_range, ptr(adv), ptr(tgt), ptr(ret), ctypes.byref(clip), stream_ptr()),
              "rlgpu_gae_flat")
        return adv, tgt, ret, clip.value

    @staticmethod
    def compute_rollout(rews, terminals, val_preds, trunc_vals, boot_vals, gamma, lam, return_std,
                        clip_range, clip_partials=None, adv=None, target=None, ret=None):
        """[T, N] rollout-layout GAE (the engine's own experience buffer); optional outputs."""
        for n_, t in (("rews", rews), ("terminals", terminals), ("val_preds", val_preds),
                      ("trunc_vals", trunc_vals), ("boot_vals", boot_vals)):
            require_gpu_tensor(t, n_)
        T, N = rews.shape
        adv = torch.empty((T, N), dtype=torch.float32, device=rews.device) if adv is None else adv
        tgt = torch.empty_like(adv) if target is None else target
        ret = torch.empty_like(adv) if ret is None else ret
        _, g = _sig()
        check(g(ptr(rews), ptr(terminals), ptr(val_preds), ptr(trunc_vals), ptr(boot_vals), T, N,
                gamma, lam, return_std, clip_range, ptr(adv), ptr(tgt), ptr(ret), ptr(clip_partials),
                stream_ptr()), "rlgpu_gae_rollout")
        return adv, tgt, ret
