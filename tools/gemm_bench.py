"""Microbenchmark + check of the f32 MFMA GEMM building block (rlgpu_gemm_f32) on the PPO shapes."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning_amd")]
from rlgpu import _lib  # noqa: E402

L = _lib.lib()
vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
L.rlgpu_gemm.argtypes = [i32, i32, i32, vp, i64, vp, i64, vp, i64, vp, i32, i32, i32, i32, vp]
dev = torch.device("cuda:0")
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def run(mode, la, lb, I, J, K, splits=1, reps=20):
    A = torch.randn((I, K) if la == 0 else (K, I), device=dev)
    B = torch.randn((J, K) if lb == 0 else (K, J), device=dev)
    C = torch.empty((splits, I, J), device=dev)
    args = (mode, la, lb, P(A), A.shape[1], P(B), B.shape[1], P(C), J, None, I, J, K, splits, _lib.stream_ptr())
    _lib.check(L.rlgpu_gemm(*args), "gemm")
    ref = (A if la == 0 else A.t()).double() @ (B.t() if lb == 0 else B).double()
    err = (C.sum(0).double() - ref).abs().max().item() / ref.abs().max().item()
    # the same product in torch fp32 (the reference's libtorch Linear arithmetic) against fp64
    tA = (A if la == 0 else A.t()).float()
    tB = (B.t() if lb == 0 else B).float()
    terr = ((tA @ tB).double() - ref).abs().max().item() / ref.abs().max().item()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        L.rlgpu_gemm(*args)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    tf = 2.0 * I * J * K / (us * 1e-6) / 1e12
    print(f"{('x6 ', 'f32', 'h3 ')[mode]} la={la} lb={lb} I={I:6d} J={J:4d} K={K:6d} splits={splits:3d}: {us:8.1f} us "
          f"{tf:7.1f} TF/s  max rel err vs fp64 {err:.1e} (torch fp32 {terr:.1e})")


SHAPES = [(0, 0, 50000, 512, 512), (0, 0, 50000, 512, 167), (0, 0, 50000, 90, 512),
          (0, 1, 50000, 512, 512), (0, 1, 50000, 512, 90),
          (1, 1, 512, 512, 50000, 49), (1, 1, 512, 167, 50000, 49), (1, 1, 90, 512, 50000, 49),
          (0, 0, 8192, 8192, 8192)]
# argv: modes (e.g. "2" or "0,2"), optionally shape indices ("0,5") and row counts replacing the
# 50000 of the picked shapes ("49152,50000": tile-round quantization)
modes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1, 2]
picks = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else range(len(SHAPES))
rows = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [None]
for i in picks:
    for r in rows:
        shp = tuple(r if (r is not None and v == 50000) else v for v in SHAPES[i])
        for mode in modes:
            run(mode, *shp)
