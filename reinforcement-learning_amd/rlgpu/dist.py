"""Distributed pieces of the Learner, written against torch.distributed so the same
code runs over RCCL on the GPUs (backend "nccl") and over gloo in the CPU tests.

Partitioning: rank g owns arenas [g*N, (g+1)*N); nothing on the env / inference / GAE path talks to
another rank.  The exchanges are the PPO ones:
  * gradient all-reduce (sum) of the flat fp32 grad buffer before clip_grad_norm_
    (PPOLearner.cpp:521-526); the loss scale uses the GLOBAL batch size (PPOLearner.cpp:374), so the
    summed gradient is the single-device gradient;
  * batch advantage moments (sum, sum of squares, count) in fp64 (PPOLearner.cpp:360-371);
  * return samples for the WelfordStat (Learner.cpp:959-967), all-gathered so every rank holds the
    same return-std state;
  * max over ranks of the timed region (bench contract).
"""
import torch
import torch.distributed as dist


def arena_range(rank, arenas_per_rank):
    return rank * arenas_per_rank, (rank + 1) * arenas_per_rank


def allreduce_grads(flat_grads, group=None):
    """In-place sum of the flat gradient buffer over ranks (one collective, 3 MB at C2)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(flat_grads, op=dist.ReduceOp.SUM, group=group)
    return flat_grads


def global_mean_std(x, group=None):
    """(mean, unbiased std) of x over all ranks' elements, fp64 accumulation -> float32 [2]."""
    s = torch.stack([x.double().sum(), (x.double() ** 2).sum(),
                     torch.tensor(float(x.numel()), dtype=torch.float64, device=x.device)])
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(s, op=dist.ReduceOp.SUM, group=group)
    n = s[2]
    mean = s[0] / n
    var = (s[1] - s[0] * mean) / (n - 1)
    return torch.stack([mean, torch.sqrt(torch.clamp(var, min=0.0))]).float()


def gather_samples(samples, group=None):
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return samples
    out = [torch.empty_like(samples) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, samples, group=group)
    return torch.cat(out)


def max_over_ranks(seconds, device=None, group=None):
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
