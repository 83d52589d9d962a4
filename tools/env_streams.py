"""Env collection split into K independent arena groups on K streams (the idea: a launch is its slowest
workgroup, so while one group's launch drains its tail the other groups' launches fill the idle SIMDs).

Steps K env sets of 4096 / K arenas (procedural SOCCAR mesh, disjoint arena streams) for `steps` env steps, each
group on its own HIP stream with its own random valid actions, and prints the wall time per step of all 4096
arenas for K = 1, 2, 4, 8.

usage: python tools/env_streams.py [steps=64] [arenas=4096]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning_amd")]
from rlgpu.env import EnvSet  # noqa: E402
from rlgpu.mesh import procedural_soccar  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 64
total = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
dev = torch.device("cuda:0")
mesh = procedural_soccar()
for K in (1, 2, 4, 8):
    n = total // K
    envs = [EnvSet(n, seed=1234, device=dev, mesh=mesh, arena_offset=g * n) for g in range(K)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(K)]
    gens = [torch.Generator(device=dev).manual_seed(7 + g) for g in range(K)]

    # a fixed cycle of random action sets per group (no per-step kernels besides the env step itself)
    pool = [[torch.randint(0, 90, (4 * n,), device=dev, dtype=torch.int32, generator=gens[g]) for _ in range(8)]
            for g in range(K)]
    torch.cuda.synchronize()

    def run(k):
        for i in range(k):
            for g in range(K):
                envs[g].step(pool[g][i % 8], True, stream=streams[g])
        torch.cuda.synchronize()

    run(8)  # warm-up (and past the kickoff)
    t0 = time.perf_counter()
    run(steps)
    ms = (time.perf_counter() - t0) * 1e3 / steps
    print(f"K={K}: {K} x {n} arenas on {K} streams: {ms:.3f} ms per env step of all {total} arenas "
          f"({total / ms * 1e3 / 1e6:.2f} M env-steps/s)", flush=True)
    del envs
