"""The reference build's Bullet arithmetic (include/rlgpu_arith.h) -- the modes an EnvSet can follow and
this host's rsqrtss table, which the kernels index for btVector3::normalize in the x86 modes.

    MSVC_X64  build.ps1's build: SSE LinearMath (btScalar.h:113-137), _sse4_1_fma3 contact / friction rows
    GCC_X64   a GCC / Clang x86-64 build: SSE LinearMath (btScalar.h:217-223), _sse2 rows
    SCALAR    Bullet's scalar LinearMath and _scalar_reference rows
"""
import ctypes

import numpy as np

from . import _lib

MSVC_X64, GCC_X64, SCALAR = 0, 1, 2
NAMES = {MSVC_X64: "msvc_x64", GCC_X64: "gcc_x64", SCALAR: "scalar"}


def rsqrt_table():
    """(table uint32 [2 << bits], bits): this host's rsqrtss results for inputs of exponent 127 + p and
    mantissa top bits h at index (p << bits) | h (rlgpu_x86_rsqrt_table)."""
    L = _lib.lib()
    L.rlgpu_x86_rsqrt_table.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32)]
    bits = ctypes.c_int32()
    _lib.check(L.rlgpu_x86_rsqrt_table(None, 0, ctypes.byref(bits)), "rlgpu_x86_rsqrt_table")
    t = np.zeros(2 << bits.value, np.uint32)
    _lib.check(L.rlgpu_x86_rsqrt_table(t.ctypes.data, t.size, ctypes.byref(bits)), "rlgpu_x86_rsqrt_table")
    return t, bits.value


def rsqrtss_emulated(x, table=None):
    """The kernels' table lookup (dmath.hpp x86_rsqrtss) in numpy, for float32 arrays."""
    t, bits = rsqrt_table() if table is None else table
    u = np.ascontiguousarray(x, np.float32).view(np.uint32)
    e = (u >> 23) & 0xff
    m = u & 0x7fffff
    neg = (u >> 31) != 0
    E = e.astype(np.int64) - 127
    p = E & 1
    q = (E - p) // 2
    idx = (p.astype(np.uint32) << bits) | (m >> (23 - bits))
    r = t[np.minimum(idx, t.size - 1)].astype(np.int64) - q * (1 << 23)
    out = (r & 0xffffffff).astype(np.uint32)
    out = np.where(e == 0, (u & 0x80000000) | 0x7f800000, out)
    out = np.where((e != 0) & (e != 0xff) & neg, 0xffc00000, out)
    inf_nan = e == 0xff
    out = np.where(inf_nan & (m != 0), u | 0x400000, out)
    out = np.where(inf_nan & (m == 0), np.where(neg, 0xffc00000, 0), out)
    return out.astype(np.uint32).view(np.float32)


def rsqrtss_emulated_c(x):
    """The library's host copy of the emulation (rlgpu_x86_rsqrtss_emulated), element by element."""
    L = _lib.lib()
    L.rlgpu_x86_rsqrtss_emulated.argtypes = [ctypes.c_float]
    L.rlgpu_x86_rsqrtss_emulated.restype = ctypes.c_float
    x = np.asarray(x, np.float32).ravel()
    return np.array([L.rlgpu_x86_rsqrtss_emulated(float(v)) for v in x], np.float32)


def linear_math_queries(op, arith, inp):
    """rlgpu_linear_math_queries on the device: op 0 normalize, 1 setRotation, 2 getRotation, 3 quaternion
    product, 4 integrateTransform, 5 wheel-ray convex cast, 6 rsqrtss, 7 sin / cos / atan2 / asin / atan
    (include/rlgpu_arith.h), on a CUDA float32 tensor of rows of 24 floats -> [n, 12]."""
    import torch
    inp = inp.reshape(-1, 24).contiguous().float()
    out = torch.zeros((inp.shape[0], 12), dtype=torch.float32, device=inp.device)
    L = _lib.lib()
    L.rlgpu_linear_math_queries.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                            ctypes.c_void_p, ctypes.c_void_p]
    _lib.check(L.rlgpu_linear_math_queries(int(op), int(arith), inp.data_ptr(), inp.shape[0], out.data_ptr(),
                                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
               "rlgpu_linear_math_queries")
    return out
