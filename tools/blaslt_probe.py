"""Library-GEMM yardstick for the H3 training GEMMs (timing only, not a product path).

An H3 product C = Ah Bh + Ah Bl + Al Bh is one fp16 GEMM over a 3x longer K ([Ah | Ah | Al] x [Bh; Bl; Bh]).
This times, on the PPO shapes, the engine's H3 kernel (rlgpu_gemm mode 2), torch's fp16 GEMM (hipBLASLt) over
K' = 3K, and torch's fp32 GEMM, each with HIP events over 20 launches.

usage: python tools/blaslt_probe.py
"""
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


def timed(fn, reps=20):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def probe(la, lb, I, J, K, splits=1):
    A = torch.randn((I, K) if la == 0 else (K, I), device=dev)
    B = torch.randn((J, K) if lb == 0 else (K, J), device=dev)
    C = torch.empty((splits, I, J), device=dev)
    args = (2, la, lb, P(A), A.shape[1], P(B), B.shape[1], P(C), J, None, I, J, K, splits, _lib.stream_ptr())
    h3 = timed(lambda: L.rlgpu_gemm(*args))
    tA = A if la == 0 else A.t()
    tB = B.t() if lb == 0 else B
    f32 = timed(lambda: torch.matmul(tA, tB))
    # fp16 over K' = 3K with the same transposition as the f32 operands
    a3 = torch.cat([tA, tA, tA], 1).half()
    b3 = torch.cat([tB, tB, tB], 0).half()
    if la == 1:
        a3 = a3.t().contiguous().t()
    if lb == 0:
        b3 = b3.t().contiguous().t()
    f16 = timed(lambda: torch.matmul(a3, b3))
    fl = 2.0 * I * J * K
    print(f"la={la} lb={lb} I={I:6d} J={J:4d} K={K:6d}: h3 {h3:7.1f} us ({3 * fl / h3 / 1e6:6.1f} TF/s eff)  "
          f"torch fp16 K'=3K {f16:7.1f} us ({3 * fl / f16 / 1e6:6.1f} TF/s)  torch fp32 {f32:7.1f} us "
          f"({fl / f32 / 1e6:6.1f} TF/s)", flush=True)


for shp in [(0, 0, 50000, 512, 512), (0, 1, 50000, 512, 512), (1, 1, 512, 512, 50000, 49),
            (0, 0, 50000, 512, 167), (0, 0, 50000, 90, 512), (0, 0, 8192, 8192, 8192)]:
    probe(*shp)
