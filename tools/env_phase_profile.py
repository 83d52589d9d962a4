"""Per-phase cycle breakdown of the env kernel (rlgpu_envset_set_profile) at the C2 size."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning_amd")]
from rlgpu import _lib  # noqa: E402
from rlgpu.env import EnvSet  # noqa: E402

NAMES = ["T0 sleep/demo/snapshot", "T1 wheels static rays (16 lanes)", "T2 car logic + pads pre", "T3 gravity/predict",
         "T4 ball awake", "T5 narrowphase (queue GJK)", "T6 commit + solve (lane 0)", "T7 integrate", "T8 car post/finish",
         "T9 pad collide", "T10 pad post + ball finish", "prelude / halves", "builders", "obs rows", "resets", "store", "T6 commit loop", "T6 commit sort",
         "T5 deferred EPA (wave)", "T6 solve body setup", "T6 solve rows build", "T6 solve iterations", "T5 narrow pairs (grid walks)",
         "T1 wheel casts (wave)", "T1 wheel finish", "T2a car phase a", "T2b wheel friction"]
PH = list(range(23)) + [30, 31, 33, 34]  # the phase slots (env_kernel.hpp kProfPhases; slot 23 = penetration-solver calls)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 32
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 8  # env steps before profiling (late-episode states)
dev = torch.device("cuda:0")
mesh_name = sys.argv[4] if len(sys.argv) > 4 else "synthetic"
arith = int(sys.argv[5]) if len(sys.argv) > 5 else 0  # include/rlgpu_arith.h mode
if mesh_name == "procedural":
    from rlgpu.mesh import procedural_soccar
    env = EnvSet(n, seed=1234, device=dev, mesh=procedural_soccar(), arith=arith)
else:
    env = EnvSet(n, seed=1234, device=dev, arith=arith)
gen = torch.Generator(device=dev).manual_seed(7)
acts = torch.empty(4 * n, dtype=torch.int32, device=dev)
for i in range(warm):
    acts.copy_(torch.argmax(torch.rand((4 * n, 90), device=dev, generator=gen) * env.action_masks, 1))
    env.step(acts, True)
APW = int(os.environ.get("RLGPU_ENV_APW", "4"))  # arenas per workgroup of the built library (env_kernel.hpp)
wg = (n + APW - 1) // APW
KP, KW = 35, 64  # env_kernel.hpp kProfPhases, kProfWG
prof = torch.zeros(KW + wg * KP + n, dtype=torch.int64, device=dev)  # + per-arena penetration-solver calls
top32 = []  # per step: the mean phase vector of the 32 slowest workgroups
spread = []  # per step: (max WG cycles, mean WG cycles, phase vector of the slowest WG, mean phase vector)
L = _lib.lib()
L.rlgpu_envset_set_profile.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
_lib.check(L.rlgpu_envset_set_profile(env._h, ctypes.c_void_p(prof.data_ptr()), prof.numel()), "set_profile")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
tot_ms = 0.0
pen_rows = []  # per step: penetration-solver calls in all / the busiest / the slowest workgroup
arena_rows, slow_arenas = [], []  # per step: workgroups with >= 2 arenas calling it; the slowest one's per-arena calls
for i in range(steps):
    acts.copy_(torch.argmax(torch.rand((4 * n, 90), device=dev, generator=gen) * env.action_masks, 1))
    e0.record()
    env.step(acts, True)
    e1.record()
    torch.cuda.synchronize()
    tot_ms += e0.elapsed_time(e1)
    per = prof[KW:KW + wg * KP].view(wg, KP)[:, PH].double()
    tots = per.sum(1)
    k = int(tots.argmax())
    spread.append((tots.max().item(), tots.mean().item(), per[k].cpu(), per.mean(0).cpu()))
    top = tots.topk(min(32, wg)).indices  # the 32 slowest workgroups of this step (~3 % of them)
    top32.append(per[top].mean(0).cpu())
    pens = prof[KW:KW + wg * KP].view(wg, KP)[:, 23]
    pen_rows.append((int(pens.sum()), int(pens.max()), int(pens[k])))
    pa = prof[KW + wg * KP:].view(-1)
    pa = torch.nn.functional.pad(pa, (0, wg * APW - n)).view(wg, APW)
    arena_rows.append(((pa > 0).sum(1) >= 2).sum().item())  # workgroups with two or more arenas calling the solver
    slow_arenas.append(pa[k].cpu().tolist())
    prof[KW:].zero_()
c = prof.cpu().tolist()
total = sum(c[k] for k in PH)
print(f"{n} arenas, {steps} steps, {mesh_name} mesh, {tot_ms / steps:.3f} ms/step (profiled build)")
ticks = steps * 8
print(f"  per tick (workgroup 0, arena 0): candidates {c[24] / ticks / wg:.2f}, mode-1 ranks {c[27] / ticks / wg:.2f}, "
      f"refresh-needing ranks {c[25] / ticks / wg:.2f}, live ranks {c[26] / ticks / wg:.2f}")
for i, k in enumerate(PH):
    print(f"  {NAMES[i]:28s} {c[k] / total * 100:6.2f} %   {c[k] / wg / steps:12.0f} cycles/WG/step")

# The kernel ends with its slowest workgroup: per step, slowest vs mean workgroup, and where the
# slowest one spends the difference.
mx = sum(x[0] for x in spread) / len(spread)
mn = sum(x[1] for x in spread) / len(spread)
print(f"  slowest workgroup per step: {mx:.0f} cycles, mean workgroup {mn:.0f} (max / mean {mx / mn:.2f})")
slow = sum(x[2] for x in spread) / len(spread)
mean = sum(x[3] for x in spread) / len(spread)
order = sorted(range(len(PH)), key=lambda k: -(slow[k] - mean[k]).item())
for k in order[:8]:
    print(f"    {NAMES[k]:28s} slowest {slow[k].item():10.0f}  mean {mean[k].item():10.0f}  excess {slow[k].item() - mean[k].item():10.0f}")
pr = np.array(pen_rows)
print(f"  penetration-solver (EPA) calls per step: mean {pr[:, 0].mean():.1f} over all workgroups, busiest workgroup "
      f"{pr[:, 1].mean():.1f} (max {pr[:, 1].max()}), slowest workgroup {pr[:, 2].mean():.1f}")
print(f"  workgroups with two or more arenas calling the penetration solver, per step: {np.mean(arena_rows):.1f}; "
      f"the slowest workgroup's calls per arena, first steps: {slow_arenas[:6]}")
t32 = sum(top32) / len(top32)
print(f"  the 32 slowest workgroups per step (the launch's tail): mean {t32.sum().item():.0f} cycles; phases by excess over the mean")
for k in sorted(range(len(PH)), key=lambda k: -(t32[k] - mean[k]).item())[:8]:
    print(f"    {NAMES[k]:28s} top32 {t32[k].item():10.0f}  mean {mean[k].item():10.0f}  excess {t32[k].item() - mean[k].item():10.0f}")
