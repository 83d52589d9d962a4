"""RocketSim's arena byte stream (Arena::Serialize / Arena::DeserializeNew,
RS/Sim/Arena/Arena.cpp:572-671) for arena records (rlgpu.state.ARENA), over the host C++ of
include/rlgpu_arena_wire.h.  See that header for the format and what the reader accepts."""
import ctypes
import struct

import numpy as np

from . import _lib
from .state import ARENA

RS_VERSION_ID = 302020  # RLGPU_RS_VERSION_ID: RocketSim "2.1.1" (RS/Framework.h:3,100-106)
MAX_BYTES = 2076 + 4 * 68

_bound = False


def _bind():
    global _bound
    L = _lib.lib()
    if not _bound:
        vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32
        pu64 = ctypes.POINTER(u64)
        L.rlgpu_arena_serialized_size.argtypes = [vp, pu64]
        L.rlgpu_arena_serialize.argtypes = [vp, vp, u64, pu64]
        L.rlgpu_arena_deserialize.argtypes = [vp, u64, vp, pu64]
        L.rlgpu_envset_serialize_arena.argtypes = [vp, i32, vp, u64, pu64]
        L.rlgpu_envset_deserialize_arena.argtypes = [vp, i32, vp, u64, pu64]
        _bound = True
    return L


def _one(rec):
    a = np.ascontiguousarray(np.array(rec, dtype=ARENA).reshape(-1))
    if a.size != 1:
        raise _lib.RLGPUError("one arena record expected")
    return a


def serialized_size(rec):
    a = _one(rec)
    n = ctypes.c_uint64()
    _lib.check(_bind().rlgpu_arena_serialized_size(a.ctypes.data, ctypes.byref(n)), "rlgpu_arena_serialized_size")
    return n.value


def serialize(rec):
    """Arena::Serialize bytes of one arena record"""
    a = _one(rec)
    out = np.zeros(MAX_BYTES, np.uint8)
    w = ctypes.c_uint64()
    _lib.check(_bind().rlgpu_arena_serialize(a.ctypes.data, out.ctypes.data, out.size, ctypes.byref(w)),
               "rlgpu_arena_serialize")
    return out[:w.value].tobytes()


def deserialize(data, base=None):
    """Arena::DeserializeNew of the stream at the start of `data`: (record, bytes consumed).
    `base` (a record) supplies the RLGym bookkeeping the stream does not carry (zeros if None)."""
    a = np.zeros(1, ARENA) if base is None else _one(base).copy()
    buf = np.frombuffer(bytes(data), np.uint8)
    c = ctypes.c_uint64()
    _lib.check(_bind().rlgpu_arena_deserialize(buf.ctypes.data, buf.size, a.ctypes.data, ctypes.byref(c)),
               "rlgpu_arena_deserialize")
    return a[0], c.value


def to_file(path, data):
    """DataStreamOut::WriteToFile(path, writeVersionCheck = true) (DataStreamOut.h:46-59)"""
    with open(path, "wb") as f:
        f.write(struct.pack("<I", RS_VERSION_ID) + bytes(data))


def from_file(path):
    """DataStreamIn(path, versionCheck = true) (DataStreamIn.h:15-31): the stream after the version"""
    with open(path, "rb") as f:
        b = f.read()
    if len(b) < 4 or struct.unpack_from("<I", b)[0] != RS_VERSION_ID:
        raise _lib.RLGPUError(f"{path}: file is invalid or from a different version of RocketSim")
    return b[4:]


def envset_serialize(env, index):
    import torch
    torch.cuda.synchronize(env.device)
    out = np.zeros(MAX_BYTES, np.uint8)
    w = ctypes.c_uint64()
    _lib.check(_bind().rlgpu_envset_serialize_arena(env._h, index, out.ctypes.data, out.size, ctypes.byref(w)),
               "rlgpu_envset_serialize_arena")
    return out[:w.value].tobytes()


def envset_deserialize(env, index, data):
    import torch
    torch.cuda.synchronize(env.device)
    buf = np.frombuffer(bytes(data), np.uint8)
    c = ctypes.c_uint64()
    _lib.check(_bind().rlgpu_envset_deserialize_arena(env._h, index, buf.ctypes.data, buf.size, ctypes.byref(c)),
               "rlgpu_envset_deserialize_arena")
    return c.value
