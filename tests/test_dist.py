"""Multi-rank logic of the Learner on CPU with gloo, world size 2.

The C++ Learner (host/learner.cpp) issues its exchanges through an rlgpu_collective; on the GPUs
bench.py / rlgpu.learner bind it to rlgpu.dist.TorchCollective over RCCL.  Here the same
TorchCollective runs over gloo with host buffers, called exactly as the C++ Learner calls it
(through its ctypes C callbacks).  Checks: gradient all-reduce with global-batch loss scaling equals
the single-device gradient of the whole batch; global advantage (mean, std) from all-reduced fp64
moments (rlgpu_moments_mean_std, the C++ finish) equals the single-device one; return samples
gathered identically on every rank; max-over-ranks timing; arena sharding is a partition.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.LayerNorm(16), torch.nn.LeakyReLU(),
                               torch.nn.Linear(16, 3))


def _loss(m, x, y, global_batch):
    # the reference scales each minibatch loss by mb / batchSize (PPOLearner.cpp:374)
    return torch.nn.functional.mse_loss(m(x), y) * (x.shape[0] / global_batch)


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "reinforcement-learning_amd"))
    from rlgpu import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(1)
        X, Y = torch.randn(64, 6, generator=g), torch.randn(64, 3, generator=g)
        lo, hi = D.arena_range(rank, 32)
        m = _model()
        # each rank: two minibatches of its shard, accumulate, then all-reduce
        for a in range(lo, hi, 16):
            _loss(m, X[a:a + 16], Y[a:a + 16], 64).backward()
        flat = np.ascontiguousarray(torch.cat([p.grad.reshape(-1) for p in m.parameters()]).numpy())
        coll = D.TorchCollective(device="cpu")
        c = coll.c_struct()  # the C callbacks the C++ Learner receives
        assert c.allreduce_sum_f32(None, flat.ctypes.data, flat.size) == 0
        adv = torch.randn(1000, generator=torch.Generator().manual_seed(10 + rank)).double()
        mom = np.array([adv.sum().item(), (adv * adv).sum().item(), float(adv.numel())])
        assert c.allreduce_sum_f64(None, mom.ctypes.data, 3) == 0
        st = D.moments_mean_std(mom)
        mine = np.full(3, float(rank), np.float32)
        smp = np.zeros(3 * world, np.float32)
        assert c.allgather_f32(None, mine.ctypes.data, 3, smp.ctypes.data) == 0
        t = D.max_over_ranks(0.5 + rank)
        q.put((rank, flat, st, smp, t))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_gloo_reductions():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    # single-device reference over the whole batch
    g = torch.Generator().manual_seed(1)
    X, Y = torch.randn(64, 6, generator=g), torch.randn(64, 3, generator=g)
    m = _model()
    _loss(m, X, Y, 64).backward()
    want = torch.cat([p.grad.reshape(-1) for p in m.parameters()]).numpy()
    for r in res:
        np.testing.assert_allclose(r[1], want, rtol=1e-5, atol=1e-7)
    advs = torch.cat([torch.randn(1000, generator=torch.Generator().manual_seed(10 + r)) for r in range(world)])
    np.testing.assert_allclose(res[0][2], [advs.mean().item(), advs.double().std().item()], rtol=1e-5, atol=1e-7)
    np.testing.assert_array_equal(res[0][2], res[1][2])
    np.testing.assert_array_equal(res[0][3], [0, 0, 0, 1, 1, 1])
    np.testing.assert_array_equal(res[1][3], res[0][3])
    assert res[0][4] == res[1][4] == 1.5


def test_arena_sharding_is_a_partition():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "reinforcement-learning_amd"))
    from rlgpu.dist import arena_range
    seen = []
    for r in range(8):
        lo, hi = arena_range(r, 4096)
        seen.extend(range(lo, hi))
    assert seen == list(range(32768))


def test_batch_ranges_match_experience_buffer():
    """ExperienceBuffer::GetAllBatchesShuffled (ExperienceBuffer.cpp:117-162) batch boundaries."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "reinforcement-learning_amd"))
    from rlgpu.learner import batch_ranges
    assert batch_ranges(100_000, 100_000) == [(0, 100_000)]            # ExampleMain: batch = tsPerItr
    assert batch_ranges(250, 100) == [(0, 100), (100, 250)]            # remainder folded (overbatching)
    assert batch_ranges(250, 100, False) == [(0, 100), (100, 200)]     # remainder dropped
    assert batch_ranges(300, 100) == [(0, 100), (100, 200), (200, 300)]
    assert batch_ranges(50, 100) == [(0, 50)]                          # fewer than one batch
    assert batch_ranges(50, 100, False) == []
    assert batch_ranges(0, 100) == []


def test_return_samples_come_from_finished_trajectories():
    """rlgpu_sample_finished_rows: the reference samples returns of combinedTraj, which holds
    finished trajectories only (Learner.cpp:823-861, 959-967).  Every drawn row (t, p) has t <= the
    column's last trajectory end; the count is min(n, #eligible); the draws are reproducible and
    cover the eligible set roughly uniformly; no finished trajectory -> no samples."""
    import numpy as np
    from rlgpu.learner import last_ends, sample_finished_rows
    T, P = 16, 12
    rng = np.random.default_rng(3)
    terms = np.zeros((T, P), np.int8)
    terms[rng.random((T, P)) < 0.08] = 1
    terms[5, 3], terms[15, 4], terms[0, 6] = 2, 1, 1
    terms[:, 0] = 0  # column 0: an unfinished trajectory only
    ends = last_ends(terms)
    assert ends[0] == -1 and ends[4] == 15 and ends[6] >= 0
    for p in range(P):
        nz = np.nonzero(terms[:, p])[0]
        assert ends[p] == (nz.max() if nz.size else -1)
    eligible = {t * P + p for p in range(P) for t in range(ends[p] + 1)}
    rows = sample_finished_rows(123, 0, 7, ends, 150)
    assert rows.size == min(150, len(eligible))
    assert set(rows.tolist()) <= eligible
    assert np.array_equal(rows, sample_finished_rows(123, 0, 7, ends, 150))      # reproducible
    assert not np.array_equal(rows, sample_finished_rows(123, 0, 8, ends, 150))  # per-iteration draws
    big = sample_finished_rows(1, 0, 0, ends, 200_000)
    assert big.size == len(eligible)  # capped at the eligible count (torch::randint over tReturns)
    many = np.concatenate([sample_finished_rows(1, 0, it, ends, 150) for it in range(400)])
    cnt = np.bincount(many, minlength=T * P)[sorted(eligible)]
    assert cnt.min() > 0 and cnt.max() < 3 * cnt.mean()
    assert sample_finished_rows(1, 0, 0, np.full(P, -1, np.int32), 150).size == 0


class _FakeStats:
    def __init__(self):
        self.total_steps = self.iteration = self.return_n = 0
        self.return_mean = self.return_m2 = 0.0


class _FakePPO:
    """The slice of rlgpu.ppo.PPO that sync_from_rank0 touches, on CPU tensors."""

    def __init__(self, n, policy):
        self.params, self.m, self.v = torch.zeros(n), torch.zeros(n), torch.zeros(n)
        self.policy, self.step, self.refreshed = policy, 0, False

    def optimizer_state(self):
        return self.step, self.m, self.v

    def set_optimizer_step(self, s):
        self.step = s

    def refresh_half(self):
        self.refreshed = True

    def model_slice(self, model):
        return self.params[:self.policy]

    def policy_version(self):
        return self.params[:self.policy]


class _FakeLearner:
    def __init__(self, rank, loaded=True):
        from rlgpu.versions import PolicyVersionManager
        self.ppo = _FakePPO(10, 4)
        self.versions = PolicyVersionManager(self.ppo)
        self.st = _FakeStats()
        self.last_checkpoint = None
        if rank == 0 and not loaded:  # no checkpoint, but policy_versions/ held two versions
            self.versions.add_version(100, torch.full((4,), 1.0))
            self.versions.add_version(200, torch.full((4,), 2.0))
        elif rank == 0:  # what checkpoint.load + load_versions leave on rank 0
            self.last_checkpoint = "/ckpt/300"
            self.ppo.params.copy_(torch.arange(10.0))
            self.ppo.m.fill_(0.5)
            self.ppo.v.fill_(0.25)
            self.ppo.step = 7
            self.st.total_steps, self.st.iteration, self.st.return_n = 300, 3, 450
            self.st.return_mean, self.st.return_m2 = 1.25, 9.5
            self.versions.add_version(100, torch.full((4,), 1.0))
            self.versions.add_version(200, torch.full((4,), 2.0))

    def _stats(self):
        return self.st

    def _set_stats(self, st):
        self.st = st


def _sync_worker(rank, world, port, q, case="loaded"):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "reinforcement-learning_amd"))
    from rlgpu.learner import sync_from_rank0
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = _FakeLearner(rank, loaded=case == "loaded")
        if case == "error":  # rank 0's load raised: every rank raises, none hangs
            try:
                sync_from_rank0(L, None, ValueError("truncated archive") if rank == 0 else None)
                q.put((rank, "no error"))
            except RuntimeError as e:
                q.put((rank, "raised" if "failed to load" in str(e) else repr(e)))
            return
        sync_from_rank0(L)
        s = L.st
        q.put((rank, L.ppo.params.tolist(), L.ppo.m.tolist(), L.ppo.v.tolist(), L.ppo.step, L.ppo.refreshed,
               (s.total_steps, s.iteration, s.return_n, s.return_mean, s.return_m2),
               [(x.timesteps, x.params.tolist()) for x in L.versions.versions]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_checkpoint_state_broadcast_from_rank0():
    """Only rank 0 reads the checkpoint folder; sync_from_rank0 hands its parameters, AdamW state,
    counters, return statistics and old policy versions to every other rank (world size 2, gloo)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sync_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert res[1][1:] == res[0][1:]
    assert res[1][1] == list(np.arange(10.0)) and res[1][4] == 7 and res[1][5]
    assert res[1][6] == (300, 3, 450, 1.25, 9.5)
    assert res[1][7] == [(100, [1.0] * 4), (200, [2.0] * 4)]


def _run_sync(case):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sync_worker, args=(r, world, port, q, case)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    return res


@pytest.mark.timeout(120)
def test_checkpoint_load_error_raises_on_every_rank():
    """a failing rank-0 load is broadcast in the header, so all ranks raise together."""
    assert _run_sync("error") == [(0, "raised"), (1, "raised")]


@pytest.mark.timeout(120)
def test_versions_broadcast_without_checkpoint():
    """rank 0's policy versions reach the other ranks even when no checkpoint was loaded."""
    res = _run_sync("versions")
    assert res[1][7] == res[0][7] == [(100, [1.0] * 4), (200, [2.0] * 4)]
    assert res[1][6] == (0, 0, 0, 0.0, 0.0) and not res[1][5]


@pytest.mark.gpu
def test_native_rccl_collective_single_rank():
    """rlgpu_rccl_* (host/rccl_collective.cpp): a one-rank RCCL communicator on the learner's stream;
    the three callbacks the C++ Learner calls -- device f32 all-reduce, host f64 all-reduce, host f32
    all-gather -- return their inputs (sum / gather over one rank).  Two ranks cannot share one GPU
    under RCCL ("Duplicate GPU detected"), so the multi-rank path runs on the driver's 8-GPU node."""
    import ctypes
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "reinforcement-learning_amd"))
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rlgpu.dist import RcclCollective
    c = RcclCollective(0, 1)
    s = c.c_struct()
    x = torch.arange(1000, dtype=torch.float32, device="cuda:0")
    assert s.allreduce_sum_f32(s.user, x.data_ptr(), x.numel()) == 0
    torch.cuda.synchronize()
    assert torch.equal(x.cpu(), torch.arange(1000, dtype=torch.float32))
    m = np.array([1.5, -2.25, 3.0])
    assert s.allreduce_sum_f64(s.user, m.ctypes.data, 3) == 0
    np.testing.assert_array_equal(m, [1.5, -2.25, 3.0])
    a = np.float32([1, 2, 3, 4])
    out = np.zeros(4, np.float32)
    assert s.allgather_f32(s.user, a.ctypes.data, 4, out.ctypes.data) == 0
    np.testing.assert_array_equal(out, a)
    c.close()
    assert not c.c_struct().user
