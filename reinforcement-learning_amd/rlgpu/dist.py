"""Distributed pieces of the Learner: the rlgpu_collective the C++ Learner calls
(include/rlgpu_learner.h), bound to torch.distributed -- RCCL over xGMI on the GPUs (backend
"nccl"), gloo in the CPU tests.

Partitioning: rank g owns arenas [g*N, (g+1)*N); nothing on the env / inference / GAE path talks to
another rank.  The exchanges are the PPO ones, issued by the C++ Learner (host/learner.cpp):
  * gradient all-reduce (sum) of the flat fp32 grad buffer before clip_grad_norm_
    (PPOLearner.cpp:521-526); the loss scale uses the GLOBAL batch size (PPOLearner.cpp:374), so the
    summed gradient is the single-device gradient;
  * batch advantage moments (sum, sum of squares, count) in fp64 (PPOLearner.cpp:360-371),
    finished by rlgpu_moments_mean_std;
  * return samples for the WelfordStat (Learner.cpp:959-967), all-gathered so every rank holds the
    same return-std state;
  * max over ranks of the timed region (bench contract);
  * at start-up, rank 0's checkpoint (parameters, AdamW state, counters, return statistics, old
    policy versions) broadcast to every rank (rlgpu.learner.sync_from_rank0), so ranks without the
    checkpoint folder cannot start from diverged replicas.
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

_ALLREDUCE_F32 = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)
_ALLREDUCE_F64 = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)
_ALLGATHER_F32 = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)


class CCollective(ctypes.Structure):
    """rlgpu_collective (include/rlgpu_learner.h)."""
    _fields_ = [("user", ctypes.c_void_p), ("allreduce_sum_f32", _ALLREDUCE_F32),
                ("allreduce_sum_f64", _ALLREDUCE_F64), ("allgather_f32", _ALLGATHER_F32)]


def arena_range(rank, arenas_per_rank):
    return rank * arenas_per_rank, (rank + 1) * arenas_per_rank


def _host_view(ptr, n, dtype):
    ct = {np.float32: ctypes.c_float, np.float64: ctypes.c_double}[dtype]
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), shape=(n,))


class TorchCollective:
    """The rlgpu_collective callbacks over a torch.distributed process group.

    device: where the f32 gradient buffer lives ("cuda:k" in production; "cpu" when a test hands
    host pointers).  With the nccl backend host buffers travel through the device."""

    def __init__(self, group=None, device="cuda:0"):
        self.group = group
        self.device = torch.device(device)
        self.backend = dist.get_backend(group) if dist.is_initialized() else None
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self._c = None

    def _comm_dev(self):
        return self.device if self.backend == "nccl" else torch.device("cpu")

    def allreduce_sum_f32(self, ptr, n):
        if self.device.type == "cuda":
            from ._lib import alias
            t = alias(ptr, (n,), torch.float32, self.device)
            if self.backend == "nccl":
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            else:
                c = t.cpu()
                dist.all_reduce(c, op=dist.ReduceOp.SUM, group=self.group)
                t.copy_(c)
        else:
            a = _host_view(ptr, n, np.float32)
            c = torch.from_numpy(a.copy()).to(self._comm_dev())
            dist.all_reduce(c, op=dist.ReduceOp.SUM, group=self.group)
            a[:] = c.cpu().numpy()
        return 0

    def allreduce_sum_f64(self, ptr, n):
        a = _host_view(ptr, n, np.float64)
        c = torch.from_numpy(a.copy()).to(self._comm_dev())
        dist.all_reduce(c, op=dist.ReduceOp.SUM, group=self.group)
        a[:] = c.cpu().numpy()
        return 0

    def allgather_f32(self, in_ptr, n, out_ptr):
        src = torch.from_numpy(_host_view(in_ptr, n, np.float32).copy()).to(self._comm_dev())
        parts = [torch.empty_like(src) for _ in range(self.world)]
        dist.all_gather(parts, src, group=self.group)
        _host_view(out_ptr, n * self.world, np.float32)[:] = torch.cat(parts).cpu().numpy()
        return 0

    def c_struct(self):
        """The struct handed to rlgpu_learner_create (callbacks kept alive by this object)."""
        if self._c is None:
            def guard(f):
                def g(*a):
                    try:
                        return f(*a[1:])
                    except Exception as e:  # never unwind through C
                        import sys
                        print(f"rlgpu collective failed: {e!r}", file=sys.stderr)
                        return -1
                return g
            self._cb = (_ALLREDUCE_F32(guard(self.allreduce_sum_f32)), _ALLREDUCE_F64(guard(self.allreduce_sum_f64)),
                        _ALLGATHER_F32(guard(self.allgather_f32)))
            self._c = CCollective(None, *self._cb)
        return self._c


class RcclCollective:
    """The rlgpu_collective over a native RCCL communicator (include/rlgpu_learner.h rlgpu_rccl_*,
    host/rccl_collective.cpp): the C++ Learner's exchanges run in C++ on RCCL, no Python callback in
    the loop.  Rank 0's unique id reaches the other ranks through `group` (torch.distributed, any
    backend) -- or pass `unique_id` bytes from another channel."""

    def __init__(self, rank, world, stream=None, group=None, unique_id=None):
        from . import _lib
        L = _lib.lib()
        L.rlgpu_rccl_unique_id.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.rlgpu_rccl_collective_create.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                                   ctypes.POINTER(CCollective)]
        L.rlgpu_rccl_collective_destroy.argtypes = [ctypes.POINTER(CCollective)]
        uid = np.zeros(128, np.uint8)
        if unique_id is not None:
            uid[:] = np.frombuffer(bytes(unique_id), np.uint8)
        else:
            if rank == 0:
                _lib.check(L.rlgpu_rccl_unique_id(uid.ctypes.data, 128), "rlgpu_rccl_unique_id")
            if world > 1:
                t = torch.from_numpy(uid.astype(np.int64))
                broadcast_(t, group)
                uid[:] = t.numpy().astype(np.uint8)
        self.unique_id = uid.tobytes()
        self._c = CCollective()
        _lib.check(L.rlgpu_rccl_collective_create(uid.ctypes.data, rank, world, _lib.stream_ptr(stream),
                                                  ctypes.byref(self._c)), "rlgpu_rccl_collective_create")

    def c_struct(self):
        return self._c

    def close(self):
        if getattr(self, "_c", None) is not None and self._c.user:
            from . import _lib
            _lib.check(_lib.lib().rlgpu_rccl_collective_destroy(ctypes.byref(self._c)), "rlgpu_rccl_collective_destroy")

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def moments_mean_std(m3):
    """rlgpu_moments_mean_std: (mean, unbiased std) float32 from fp64 (sum, sum sq, count)."""
    from . import _lib
    L = _lib.lib()
    L.rlgpu_moments_mean_std.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    m = np.ascontiguousarray(m3, np.float64)
    out = np.zeros(2, np.float32)
    _lib.check(L.rlgpu_moments_mean_std(m.ctypes.data, out.ctypes.data), "rlgpu_moments_mean_std")
    return out


def broadcast_(t, group=None):
    """Rank 0's tensor into `t` on every rank, in place: RCCL for device tensors on nccl, whose host
    tensors (the header, version timestamps) travel through the current device; gloo through the
    host."""
    backend = dist.get_backend(group)
    if backend == "nccl":
        if t.device.type == "cuda":
            dist.broadcast(t, 0, group=group)
        else:  # RCCL cannot take host buffers
            d = t.to(torch.device("cuda", torch.cuda.current_device()))
            dist.broadcast(d, 0, group=group)
            t.copy_(d.cpu())
    elif t.device.type == "cpu":
        dist.broadcast(t, 0, group=group)
    else:
        c = t.cpu()
        dist.broadcast(c, 0, group=group)
        t.copy_(c)
    return t


def max_over_ranks(seconds, device=None, group=None):
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
