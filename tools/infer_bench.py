"""Inference microbenchmark: rlgpu_ppo_infer_actions on one collection step (16,384 agents) and
rlgpu_ppo_infer_critic over a C2 rollout (129 x 16,384 rows), bf16 MFMA path."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning_amd")]
from rlgpu.ppo import PPO  # noqa: E402

dev = torch.device("cuda:0")
ppo = PPO(167, 90, (512, 512), (512, 512), max_rows=65536, seed=1, device=dev)
P = 16384
obs = torch.randn(P, 167, device=dev)
masks = torch.ones(P, 90, dtype=torch.uint8, device=dev)
roll = torch.randn(129 * P, 167, device=dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, fn, reps in (("infer_actions 16384", lambda: ppo.infer_actions(obs, masks, step=3), 50),
                       ("infer_critic 129x16384", lambda: ppo.infer_critic(roll), 3)):
    fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us")
