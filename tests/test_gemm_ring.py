"""The LDS-DMA ring kernel of the forward / input-gradient training GEMMs (csrc/mlp_kernels.hpp
gemm_h3r, RLGPU_H3_RING) against the register-staged H3 kernel it replaces (gemm_x6, RLGPU_H3_RING=0):
the same split, product order and epilogue, so every output bit must agree -- on full tiles, ragged
row / column edges, K not a multiple of the 32- or 64-deep stage, and rows past the last tile.
Each ring setting runs in its own process (the library reads the switch once).
Reference arithmetic: torch.nn.Linear fp32 (PPOLearner.cpp:396-501's forward / backward GEMMs).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import ctypes, hashlib, json, os, sys
sys.path[:0] = [%(root)r, os.path.join(%(root)r, "reinforcement-learning_amd")]
import torch
from rlgpu import _lib
L = _lib.lib()
vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
L.rlgpu_gemm.argtypes = [i32, i32, i32, vp, i64, vp, i64, vp, i64, vp, i32, i32, i32, i32, vp]
dev = torch.device("cuda:0")
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
out = {}
for (I, J, K, bias) in [(50000, 512, 512, True), (1000, 90, 512, False), (4099, 512, 100, True), (257, 384, 168, True),
                        (128, 128, 64, False), (3, 1, 36, True)]:
    g = torch.Generator(device=dev).manual_seed(I * 7 + J * 3 + K)
    A = torch.randn((I, K), device=dev, generator=g) * 3.0
    B = torch.randn((J, K), device=dev, generator=g) * 0.05
    b = torch.randn((J,), device=dev, generator=g) if bias else None
    C = torch.full((I, J), float("nan"), device=dev)
    _lib.check(L.rlgpu_gemm(2, 0, 0, P(A), K, P(B), K, P(C), J, P(b), I, J, K, 1, _lib.stream_ptr()), "gemm")
    torch.cuda.synchronize()
    ref = A.double() @ B.double().t() + (b.double() if bias else 0)
    err = ((C.double() - ref).abs().max() / ref.abs().max()).item()
    out[f"{I}x{J}x{K}"] = [hashlib.sha256(C.cpu().numpy().tobytes()).hexdigest(), err]
print(json.dumps(out))
"""


def _run(ring):
    env = dict(os.environ, RLGPU_H3_RING=str(ring))
    r = subprocess.run([sys.executable, "-c", SCRIPT % {"root": ROOT}], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_ring_kernel_bit_identical_to_staged_kernel():
    base = _run(0)
    for shape, (_, err) in base.items():
        assert err < 1e-5, (shape, err)  # fp32-class (H3) accuracy of the reference path itself
    for ring in (1, 2, 3):
        got = _run(ring)
        for shape, (h, err) in base.items():
            assert got[shape][0] == h, f"RLGPU_H3_RING={ring}: {shape} differs from the staged kernel (err {got[shape][1]:.2e})"
