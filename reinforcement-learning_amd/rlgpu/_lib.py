"""ctypes binding of the product library rlgpu/librlgpu.so (built from csrc/*.hip for gfx950).

There is deliberately NO fallback: if the HIP library is missing or was not built,
every product entry point raises.  (The CPU oracle under /oracle is test infrastructure
and is never imported from here.)
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RLGPU_LIB: an alternative build of the same library (experiments, e.g. other compiler flags)
LIB_PATH = os.environ.get("RLGPU_LIB") or os.path.join(_HERE, "librlgpu.so")
_lib = None


class RLGPUError(RuntimeError):
    """A non-zero status from the C ABI (mirrors the reference's RG_ERR_CLOSE throw)."""


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RLGPUError(
                f"{LIB_PATH} not found: build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()')")
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.rlgpu_last_error.restype = ctypes.c_char_p
    return _lib


def last_error():
    """rlgpu_last_error() of this thread."""
    return lib().rlgpu_last_error().decode(errors="replace")


def check(status, what=""):
    if status != 0:
        msg = lib().rlgpu_last_error().decode(errors="replace")
        raise RLGPUError(f"{what} failed ({status}): {msg}")


def ptr(t):
    """Device/host pointer of a torch tensor (or None)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def require_gpu_tensor(t, name):
    if t is not None and not t.is_cuda:
        raise RLGPUError(f"{name} must be a device (HBM) tensor; the product path has no CPU fallback")


def alias(ptr, shape, dtype, device):
    """torch tensor aliasing library-owned device memory (no copy, no ownership)."""
    import torch
    n = int(np.prod(shape))
    elt = torch.empty((), dtype=dtype).element_size()

    class _Holder:
        __cuda_array_interface__ = {
            "shape": (n,), "typestr": {torch.float32: "<f4", torch.uint8: "|u1", torch.int32: "<i4",
                                       torch.int8: "|i1", torch.float64: "<f8", torch.int64: "<i8"}[dtype],
            "data": (ptr, False), "version": 2, "strides": (elt,)}

    t = torch.as_tensor(_Holder(), device=device)
    return t.view(*shape)
