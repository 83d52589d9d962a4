"""Learn-phase microbenchmark: rlgpu_ppo_minibatch on the bench's C2 model (policy / critic [512, 512],
LayerNorm + LeakyReLU, 167 obs, 90 actions) over 50,000-row minibatches of a 200,000-row synthetic
buffer, shuffled, then the optimizer step -- the PPOLearner::Learn inner loop (PPOLearner.cpp:396-501)
without the env.  Prints ms per minibatch (HIP events); run under rocprofv3 --kernel-trace --stats
for per-kernel durations.

usage: python tools/learn_bench.py [minibatches=24] [train_gemm=h3|x6|f32] [width=512] [depth=2]
(width 2048, depth 4 = the C5 leg's model)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning_amd")]
from rlgpu.ppo import GEMM_F16X3, GEMM_F32, GEMM_F32X6, PPO, kernel_timing, kernel_timing_read, permutation  # noqa: E402

nmb = int(sys.argv[1]) if len(sys.argv) > 1 else 24
mode = {"h3": GEMM_F16X3, "x6": GEMM_F32X6, "f32": GEMM_F32}[sys.argv[2] if len(sys.argv) > 2 else "h3"]
dev = torch.device("cuda:0")
N, MB = 200_000, 50_000
g = torch.Generator(device=dev).manual_seed(3)
obs = torch.randn((N, 167), device=dev, generator=g)
masks = (torch.rand((N, 90), device=dev, generator=g) < 0.7).to(torch.uint8)
masks[:, 0] = 1
acts = torch.multinomial(masks.float(), 1, generator=g).squeeze(1).to(torch.int32)
old = -torch.rand((N,), device=dev, generator=g) * 4
adv = torch.randn((N,), device=dev, generator=g)
tgt = torch.randn((N,), device=dev, generator=g)
width = int(sys.argv[3]) if len(sys.argv) > 3 else 512
depth = int(sys.argv[4]) if len(sys.argv) > 4 else 2
layers = (width,) * depth
p = PPO(max_rows=MB, seed=123, train_gemm=mode, policy_layers=layers, critic_layers=layers)
p.adv_normalizer(adv)
idx = permutation(N, 7, 0)


def run(k):
    for i in range(k):
        if i % (N // MB) == 0:
            p.zero_grad()
        p.minibatch(obs, masks, acts, old, adv, tgt, idx, (i % (N // MB)) * MB, MB, MB)
        if i % (N // MB) == N // MB - 1:
            p.optimizer_step()


run(4)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
run(nmb)
e1.record()
torch.cuda.synchronize()
print(f"learn_bench {layers}: {e0.elapsed_time(e1) / nmb:.3f} ms per 50k minibatch (+ optimizer step every {N // MB}), "
      f"mode {sys.argv[2] if len(sys.argv) > 2 else 'h3'}, {nmb} minibatches", flush=True)
print("metrics finite:", bool(np.isfinite(p.metrics.cpu().numpy()).all()))
kernel_timing(True)
run(8)
torch.cuda.synchronize()
for name, (ms, work, n) in kernel_timing_read().items():
    if n:
        g = "GEMM" in name
        print(f"  {name:34s} {n:4d} launches avg {ms * 1e3 / n:7.1f} us  "
              f"{work / (ms * 1e-3) / (1e12 if g else 1e9):7.1f} {'TF/s' if g else 'GB/s'}")
kernel_timing(False)
