"""Data parallelism through the real C++ Learner (host/learner.cpp), ranks on one GPU over gloo.

* 2 ranks x 64 arenas equal 1 rank x 128 arenas: the arenas' and the sampler's random streams are global
  (rlgpu_envset_config.arena_offset, rlgpu_ppo_config.sample_row_offset), and the return samples are drawn
  over the job's rows with one generator, so the two jobs collect the same rollouts and feed the
  WelfordStat the same returns (identical statistics); the parameters after the iterations agree to fp32
  summation order (the minibatches of the two jobs hold different rows; AdamW's first steps move each
  parameter by +-lr, so a flipped sign of a near-zero gradient component shows as a 2 lr difference).
  PPOLearner.cpp:360-374,521-526; SURVEY.md 8e.
* the trajectory mode (experience_mode 1) with a rank that finishes no trajectory in an iteration: it
  still joins the return-sample all-gather and every batch's all-reduces, so nothing hangs
  and the ranks stay identical.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, kw, iters):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "reinforcement-learning_amd"))
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rlgpu.learner import Learner, LearnerConfig
        k = dict(kw)
        per_rank = k.pop("per_rank", {})
        k.update(per_rank.get(rank, {}))
        L = Learner(LearnerConfig(train_against_old_versions=False, **k), device="cuda:0", rank=rank, world=world)
        out = {"rank": rank, "rewards": [], "ret": [], "grads": []}
        # the all-reduced flat gradient of each batch, before clip_grad_norm_ / AdamW (rlgpu_learner_set_grad_hook)
        L.set_grad_hook(lambda g, epoch, batch: out["grads"].append((epoch, batch, g.cpu().numpy().copy())))
        for _ in range(iters):
            L.iterate()
            torch.cuda.synchronize()
            if k.get("experience_mode", 0) == 0:
                out["rewards"].append(L.rewards.cpu().numpy().copy())
            out["ret"].append((L.return_stat.n, L.return_stat.mean, L.return_stat.m2))
        out["params"] = L.ppo.flat().cpu().numpy().copy()
        out["steps"] = L.total_steps
        q.put(out)
    finally:
        if world > 1:
            dist.destroy_process_group()


def _run(world, kw, iters):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, kw, iters)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time
    res, deadline = [], time.time() + 280
    try:
        while len(res) < world:  # a rank that dies must fail the test now, not after the queue's timeout
            try:
                res.append(q.get(timeout=5))
            except queue.Empty:
                dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
                assert not dead, f"a rank exited with {dead}"
                assert time.time() < deadline, "ranks did not finish in time"
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    return sorted(res, key=lambda r: r["rank"])


@pytest.mark.timeout(400)
def test_two_ranks_equal_one_rank(gpu):
    """One iteration from the same initial parameters: the rollouts and return statistics are identical; the
    first batch's all-reduced gradient (before clip_grad_norm_ / AdamW, the whole rollout in both jobs) agrees
    normwise to 1e-5 -- the same rows, summed in a different order -- and the parameters after the update agree
    to fp32 summation order.  (A second iteration would infer with those
    slightly different parameters, so its sampled actions -- and rollouts -- may differ where two actions
    are nearly tied.)"""
    import torch  # noqa: F401
    kw = dict(num_arenas=64, rollout_len=16, mini_batch_size=1024, seed=5)
    two = _run(2, kw, 1)
    one = _run(1, dict(kw, num_arenas=128), 1)[0]
    # the same rollouts: rank r's players are players [256 r, 256 (r + 1)) of the one-rank job
    got = np.concatenate([two[0]["rewards"][0], two[1]["rewards"][0]], axis=1)
    np.testing.assert_array_equal(got.view(np.uint32), one["rewards"][0].view(np.uint32))
    # the same return statistics (the same samples in the same order), bit for bit
    assert two[0]["ret"][0] == two[1]["ret"][0] == one["ret"][0], (two[0]["ret"][0], one["ret"][0])
    assert two[0]["steps"] == two[1]["steps"] == one["steps"]
    # the gradient both jobs clip and step first: the sum over the ranks of each rank's rows' gradients
    (e2, b2, g2), (e1, b1, g1) = two[0]["grads"][0], one["grads"][0]
    assert (e2, b2) == (e1, b1) == (0, 0)
    np.testing.assert_array_equal(g2, two[1]["grads"][0][2])  # every rank steps the same reduced gradient
    assert len(two[0]["grads"]) == len(one["grads"])
    rel = float(np.linalg.norm(g2.astype(np.float64) - g1) / np.linalg.norm(g1.astype(np.float64)))
    print(f"first all-reduced gradient, 2 x 64 vs 1 x 128 arenas: ||diff|| / ||g|| = {rel:.3g}")
    assert np.linalg.norm(g1) > 0 and rel <= 1e-5, rel
    np.testing.assert_array_equal(two[0]["params"], two[1]["params"])
    d = np.abs(two[0]["params"] - one["params"])
    lr = 2.5e-4
    close = d <= 1e-6 + 1e-5 * np.abs(one["params"])
    print(f"2 x 64 vs 1 x 128 arenas: {close.mean():.5f} of {d.size} parameters within 1e-5, max |diff| {d.max():.3g}")
    assert d.max() <= 4 * lr * 1.01
    assert close.mean() >= 0.98


@pytest.mark.timeout(400)
def test_trajectory_mode_rank_without_finished_rows(gpu):
    """Rank 0's episodes (4.5 s = 67 steps, inside its 80-row step store) cannot end in the few collection
    steps rank 1's 0.2 s episodes need to fill an iteration, so rank 0 brings no rows; rank 1 does.  Both
    ranks run 3 iterations to the end with the same parameters and return statistics."""
    kw = dict(num_arenas=16, experience_mode=1, experience_capacity=80, ts_per_itr=512, mini_batch_size=512, seed=7,
              per_rank={0: dict(max_episode_duration=4.5), 1: dict(max_episode_duration=0.2)})
    res = _run(2, kw, 3)
    np.testing.assert_array_equal(res[0]["params"], res[1]["params"])
    assert res[0]["ret"] == res[1]["ret"]
    assert res[1]["ret"][-1][0] > 0  # rank 1's samples reached both ranks' statistics


def test_bench_two_ranks_under_torchrun(gpu):
    """The driver's multi-GPU launch, rehearsed on one GPU: `python -m torch.distributed.run --nproc-per-node 2
    bench.py --gpus 2` (gloo, since RCCL refuses two ranks on one device; on a node the same command runs the
    native RCCL collective).  Rank 0 prints ONE JSON line: n_gpus 2, value = 2 ranks x arenas x T x steps over
    the max-over-ranks wall time."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    arenas, T, steps = 64, 16, 2
    env = dict(os.environ, RLGPU_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", str(steps), "--warmup",
           "1", "--arenas", str(arenas), "--rollout", str(T), "--no-legs", "--no-cpu-baseline", "--mesh", "synthetic"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == steps and out["scaling"] == "weak"
    assert out["config"]["parallelism"] == "arena-sharded dp2"
    assert "gloo" in out["config"]["collective"]
    want = 2 * arenas * T * steps / (out["ms_per_step"] * steps / 1e3)
    assert abs(out["value"] - want) <= 1e-6 * want, (out["value"], want)
    assert out["roofline"]["units_per_launch"] == arenas
