"""ORACLE -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker / the timed CPU baseline.  The product (rlgpu) never
imports, links or executes anything here.  Built by oracle/Makefile into
oracle/build/liboracle.so (plain gcc/g++, strict IEEE float).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        _lib = ctypes.CDLL(LIB_PATH)
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def gae_flat(rews, terms, vals, trunc_vals, gamma, lam, return_std, clip_range):
    """oracle_gae_flat: GAE.cpp:7-208. Returns (adv, target, ret, clip_portion, status)."""
    rews = np.ascontiguousarray(rews, np.float32)
    terms = np.ascontiguousarray(terms, np.int8)
    vals = np.ascontiguousarray(vals, np.float32)
    tv = None if trunc_vals is None else np.ascontiguousarray(trunc_vals, np.float32)
    n = rews.size
    nt = 0 if tv is None else tv.size
    adv = np.empty(n, np.float32)
    tgt = np.empty(n, np.float32)
    ret = np.empty(n, np.float32)
    clip = ctypes.c_float(0)
    f = lib().oracle_gae_flat
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64] * 2 + [ctypes.c_float] * 4 + \
        [ctypes.c_void_p] * 3 + [ctypes.POINTER(ctypes.c_float)]
    st = f(_p(rews), _p(terms), _p(vals), _p(tv), n, nt, gamma, lam, return_std, clip_range,
           _p(adv), _p(tgt), _p(ret), ctypes.byref(clip))
    return adv, tgt, ret, clip.value, st


def gae_rollout(rews, terms, vals, trunc_vals, boot_vals, gamma, lam, return_std, clip_range):
    rews = np.ascontiguousarray(rews, np.float32)
    T, N = rews.shape
    terms = np.ascontiguousarray(terms, np.int8)
    vals = np.ascontiguousarray(vals, np.float32)
    tv = None if trunc_vals is None else np.ascontiguousarray(trunc_vals, np.float32)
    bv = None if boot_vals is None else np.ascontiguousarray(boot_vals, np.float32)
    adv = np.empty((T, N), np.float32)
    tgt = np.empty((T, N), np.float32)
    ret = np.empty((T, N), np.float32)
    f = lib().oracle_gae_rollout
    f.restype = None
    f.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int32] * 2 + [ctypes.c_float] * 4 + [ctypes.c_void_p] * 3
    f(_p(rews), _p(terms), _p(vals), _p(tv), _p(bv), T, N, gamma, lam, return_std, clip_range,
      _p(adv), _p(tgt), _p(ret))
    return adv, tgt, ret
