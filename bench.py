"""bench.py -- BASELINE.json metric on MI355X: env-steps/s (whole job) for the C2 workload
(4096 arenas per GPU, 2v2, tickSkip 8 / actionDelay 7, ExampleMain plugin set).

Contract (driver): python bench.py --gpus N --steps K --warmup W ; for N > 1 launched by
torch.distributed.run, one rank per GPU.  Rank 0 prints ONE JSON line.

A "step" here is one env step of every arena on every rank: the fused HIP env kernel
(7 + 1 physics ticks, rewards, terminals, obs, masks, reset-if-terminal) with the actions of
that step already resident in HBM.  Arenas shard across ranks with no data-path collective
(weak scaling); the barrier + max-over-ranks timing follows the contract.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-learning_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s peak
ARENAS_PER_GPU = 4096   # BASELINE configs[1] (C2)


def env_bytes_per_step(arena_state_size):
    """B_env = 2*S_arena + 16 (actions) + 2672 (obs) + 360 (masks) + 16 (rewards) + 1 (terminal)."""
    return 2 * arena_state_size + 16 + 4 * 167 * 4 + 4 * 90 + 16 + 1


def cpu_baseline(seconds=12.0, arenas=256):
    """The CPU restatement (oracle/, reference threading model: contiguous arena chunks over a
    pool) timed on this box's host cores on a bounded sample of the same workload."""
    import numpy as np
    import oracle
    cores = min(16, os.cpu_count() or 1)  # the box's CPU share is 16 (gpurun)
    env = oracle.EnvSet(arenas, seed=1234, threads=cores)
    rng = np.random.default_rng(7)
    steps = 0
    t0 = time.perf_counter()
    while True:
        m = env.masks.astype(bool)
        a = np.argmax(rng.random(m.shape) * m, axis=1).astype(np.int32)
        env.step(a, True)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": arenas * steps / el, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"{arenas} arenas x {steps} env steps (oracle/ CPU restatement, {cores} threads, "
                      f"random valid actions)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--arenas", type=int, default=ARENAS_PER_GPU)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from rlgpu.env import EnvSet, arena_state_size
    n = args.arenas
    env = EnvSet(n, seed=1234 + 1000003 * rank, device=dev)
    gen = torch.Generator(device=dev).manual_seed(7 + rank)
    P = 4 * n
    # actions for every step drawn up front (uniform over valid actions is mask-dependent, so
    # draw per-step uniforms now and pick inside the loop with one fused torch op)
    total = args.warmup + args.steps
    uni = torch.rand((min(total, 32), P, 90), device=dev, generator=gen)
    acts = torch.empty(P, dtype=torch.int32, device=dev)

    def one_step(i, e0=None, e1=None):
        acts.copy_(torch.argmax(uni[i % uni.shape[0]] * env.action_masks, dim=1))
        if e0 is not None:
            e0.record()
        env.step(acts, True)
        if e1 is not None:
            e1.record()

    for i in range(args.warmup):
        one_step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_step(args.warmup + i, *evs[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    value = world * n * args.steps / el
    b_env = env_bytes_per_step(arena_state_size())
    achieved = b_env * n / (kern_ms * 1e-3) / 1e9
    out = {
        "metric": "env-steps/sec (whole node) at 32768 arenas; PPO wall-clock per 1M steps",
        "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": el * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "C2 env collection: 4096 arenas/GPU 2v2, tickSkip 8 / actionDelay 7, "
                               "AdvancedObs+DefaultAction+13 rewards, uniform valid actions",
                   "arenas_per_gpu": n, "agents_per_gpu": P, "parallelism": f"arena-sharded x{world}"},
        "agent_steps_per_s": 4 * value,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "rl::env_kernel", "kernel_ms": kern_ms, "bytes_per_env_step": b_env},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
