"""Env-kernel time per fused step against the arena count (latency- vs issue-bound check): a kernel
bound by per-wave latency takes about the same time while waves per SIMD grow; an issue-bound one
grows linearly."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning_amd")]
from rlgpu.env import EnvSet  # noqa: E402

dev = torch.device("cuda:0")
warm = int(os.environ.get("ENV_WARM", "8"))  # env steps before timing (late-episode states)
for n in [int(x) for x in (sys.argv[1:] or ["1024", "2048", "4096", "8192", "16384"])]:
    env = EnvSet(n, seed=1234, device=dev)
    gen = torch.Generator(device=dev).manual_seed(7)
    acts = torch.empty(4 * n, dtype=torch.int32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tot, steps = 0.0, 24
    for i in range(warm + steps):
        acts.copy_(torch.argmax(torch.rand((4 * n, 90), device=dev, generator=gen) * env.action_masks, 1))
        e0.record()
        env.step(acts, True)
        e1.record()
        torch.cuda.synchronize()
        if i >= warm:
            tot += e0.elapsed_time(e1)
    ms = tot / steps
    print(f"{n:6d} arenas: {ms:.3f} ms/step  {n / ms * 1e3 / 1e6:.2f} M env-steps/s", flush=True)
    del env
