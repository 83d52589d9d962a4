"""GAE: oracle pinned by closed forms + golden vectors (CPU); HIP kernels vs oracle (GPU).

Reference: GGL::GAE::Compute, GigaLearnCPP/src/private/GigaLearnCPP/PPO/GAE.cpp:7-208.
Tolerances: the [T,N] rollout kernel is bit-exact (same operation order, no FMA
contraction); the flat kernel reassociates the recursion as an affine scan, so it is
checked at rtol 1e-5 (north-star float tolerance) with an absolute floor scaled by the
magnitude of the terms.
"""
import glob
import os

import numpy as np
import pytest

import oracle
from conftest import ROOT

GOLDEN = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "gae_flat_*.npz")))


def closed_form(rews, vals, gamma, lam):
    """Single episode ending NORMAL: A_t = sum_k (g*l)^k delta_{t+k}."""
    n = len(rews)
    nxt = np.append(vals[1:], 0.0)
    delta = rews + gamma * nxt - vals
    adv = np.array([sum((gamma * lam) ** k * delta[t + k] for k in range(n - t)) for t in range(n)])
    ret = np.array([sum(gamma ** k * rews[t + k] for k in range(n - t)) for t in range(n)])
    return adv, ret


def test_oracle_closed_form_single_episode():
    rng = np.random.default_rng(0)
    r = rng.standard_normal(40).astype(np.float32)
    v = rng.standard_normal(40).astype(np.float32)
    t = np.zeros(40, np.int8)
    t[-1] = 1
    adv, tgt, ret, cp, st = oracle.gae_flat(r, t, v, None, 0.99, 0.95, 1.0, 0.0)
    ea, er = closed_form(r.astype(np.float64), v.astype(np.float64), 0.99, 0.95)
    np.testing.assert_allclose(adv, ea, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ret, er, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(tgt, v + adv)
    assert st == 0 and cp == 0.0


def test_oracle_truncation_bootstrap_and_normalisation():
    # two episodes: [0..2] truncated (bootstrap 5.0), [3..4] normal
    r = np.array([1, 2, 3, 4, 5], np.float32)
    v = np.array([0.5, 0.25, 0.0, 1.0, 2.0], np.float32)
    t = np.array([0, 0, 2, 0, 1], np.int8)
    g, l, std, clip = 0.9, 0.5, 2.0, 1.2
    adv, tgt, ret, cp, st = oracle.gae_flat(r, t, v, np.array([5.0], np.float32), g, l, std, clip)
    n = np.clip(r / std, -clip, clip)
    d2 = n[2] + g * 5.0 - v[2]
    d1 = n[1] + g * v[2] - v[1]
    d0 = n[0] + g * v[1] - v[0]
    d4 = n[4] - v[4]
    d3 = n[3] + g * v[4] - v[3]
    exp_adv = [d0 + g * l * (d1 + g * l * d2), d1 + g * l * d2, d2, d3 + g * l * d4, d4]
    np.testing.assert_allclose(adv, exp_adv, rtol=1e-6)
    # returns use RAW rewards (GAE.cpp:183-185) and stop at either terminal type
    np.testing.assert_allclose(ret, [1 + g * (2 + g * 3), 2 + g * 3, 3, 4 + g * 5, 5], rtol=1e-6)
    raw = np.abs(r / std).sum()
    assert cp == pytest.approx((raw - np.abs(n).sum()) / raw, rel=1e-6)
    assert st == 0


def test_oracle_truncation_count_mismatch_is_error():
    r = np.ones(4, np.float32)
    t = np.array([2, 0, 2, 1], np.int8)
    *_, st = oracle.gae_flat(r, t, r, np.ones(1, np.float32), 0.99, 0.95, 1.0, 0.0)
    assert st == -1


def test_oracle_empty():
    e = np.zeros(0, np.float32)
    adv, tgt, ret, cp, st = oracle.gae_flat(e, np.zeros(0, np.int8), e, None, 0.99, 0.95, 1.0, 0.0)
    assert adv.size == 0 and cp == 0.0 and st == 0


@pytest.mark.parametrize("path", GOLDEN)
def test_oracle_matches_golden(path):
    z = np.load(path)
    g, l, std, clip = [float(x) for x in z["params"]]
    adv, tgt, ret, cp, st = oracle.gae_flat(z["rews"], z["terms"], z["vals"], z["trunc_vals"], g, l, std, clip)
    np.testing.assert_array_equal(adv, z["adv"])
    np.testing.assert_array_equal(ret, z["ret"])
    np.testing.assert_array_equal(tgt, z["target"])
    assert np.float32(cp) == z["clip_portion"]


def test_oracle_rollout_equals_flat_per_column():
    rng = np.random.default_rng(3)
    T, N = 33, 7
    r = rng.standard_normal((T, N)).astype(np.float32)
    v = rng.standard_normal((T, N)).astype(np.float32)
    t = (rng.random((T, N)) < 0.08).astype(np.int8)
    a, tg, rt = oracle.gae_rollout(r, t, v, None, None, 0.99, 0.95, 3.0, 2.0)
    for n in range(N):
        fa, ft, fr, _, _ = oracle.gae_flat(r[:, n], t[:, n], v[:, n], None, 0.99, 0.95, 3.0, 2.0)
        np.testing.assert_array_equal(a[:, n], fa)
        np.testing.assert_array_equal(rt[:, n], fr)


# ---------------------------------------------------------------- GPU parity (C ABI)

def _flat_case(m, seed):
    from tests_util import synth_gae
    return synth_gae(m, seed)


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN)
def test_gpu_flat_matches_golden(gpu, path):
    import torch
    from rlgpu import GAE
    z = np.load(path)
    g, l, std, clip = [float(x) for x in z["params"]]
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    adv, tgt, ret, cp = GAE.compute(d(z["rews"]), d(z["terms"]), d(z["vals"]), d(z["trunc_vals"]), g, l, std, clip)
    scale = np.abs(z["adv"]).max() + 1
    np.testing.assert_allclose(adv.cpu().numpy(), z["adv"], rtol=1e-5, atol=1e-5 * scale)
    np.testing.assert_allclose(ret.cpu().numpy(), z["ret"], rtol=1e-5, atol=1e-5 * (np.abs(z["ret"]).max() + 1))
    np.testing.assert_allclose(tgt.cpu().numpy(), z["target"], rtol=1e-5, atol=1e-5 * scale)
    assert cp == pytest.approx(float(z["clip_portion"]), rel=1e-4, abs=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("m", [1, 7, 2047, 2048, 2049, 4095, 4096, 4097, 8191, 8192, 8193, 12289, 1 << 21, 1 << 24])
def test_gpu_flat_sizes_and_edges(gpu, m):
    import torch
    from rlgpu import GAE
    from tests_util import synth_gae
    r, t, v, tv = synth_gae(m, 11 + m)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    adv, tgt, ret, cp = GAE.compute(d(r), d(t), d(v), d(tv) if tv.size else None, 0.99, 0.95, 1.7, 5.0)
    ea, et, er, ecp, st = oracle.gae_flat(r, t, v, tv, 0.99, 0.95, 1.7, 5.0)
    assert st == 0
    np.testing.assert_allclose(adv.cpu().numpy(), ea, rtol=1e-5, atol=1e-5 * (np.abs(ea).max() + 1))
    np.testing.assert_allclose(ret.cpu().numpy(), er, rtol=1e-5, atol=1e-5 * (np.abs(er).max() + 1))
    assert cp == pytest.approx(ecp, rel=1e-4, abs=1e-6)


@pytest.mark.gpu
def test_gpu_flat_tile_boundaries_unaligned_and_deterministic(gpu):
    """The flat scan's 8192-element tiles (1024-element rounds in the apply pass): one episode running across
    tiles with no terminal, truncations on a tile's / round's first and last elements and on adjacent steps, and the same inputs one element off 16-byte
    alignment (the scalar-access variant); two calls agree bit for bit (a fixed composition order)."""
    import torch
    from rlgpu import GAE
    m = 3 * 8192 + 1024 + 77
    rng = np.random.default_rng(3)
    r = rng.standard_normal(m).astype(np.float32)
    v = rng.standard_normal(m).astype(np.float32)
    t = np.zeros(m, np.int8)
    for i in (1023, 1024, 2047, 2048, 4096, 8191, 8192, 8193, 12288 + 4095, 16383, 16384, 16385, 24575, 24576, m - 1):
        t[i] = 2
    t[9000] = 1
    tv = rng.standard_normal(int((t == 2).sum())).astype(np.float32)
    ea, et, er, ecp, st = oracle.gae_flat(r, t, v, tv, 0.99, 0.95, 1.7, 5.0)
    assert st == 0
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)  # noqa: E731
    outs = []
    for off in (0, 1):
        pad = lambda a: np.concatenate([np.zeros(off, a.dtype), a])  # noqa: E731
        rr, tt, vv = d(pad(r))[off:], d(pad(t))[off:], d(pad(v))[off:]
        for _ in range(2):
            adv, tgt, ret, cp = GAE.compute(rr, tt, vv, d(tv), 0.99, 0.95, 1.7, 5.0)
            np.testing.assert_allclose(adv.cpu().numpy(), ea, rtol=1e-5, atol=1e-5 * (np.abs(ea).max() + 1))
            np.testing.assert_allclose(ret.cpu().numpy(), er, rtol=1e-5, atol=1e-5 * (np.abs(er).max() + 1))
            np.testing.assert_allclose(tgt.cpu().numpy(), et, rtol=1e-5, atol=1e-5 * (np.abs(et).max() + 1))
            assert cp == pytest.approx(ecp, rel=1e-4, abs=1e-6)
            outs.append((adv.cpu().numpy(), ret.cpu().numpy(), cp))
    for a, b in ((0, 1), (2, 3)):
        np.testing.assert_array_equal(outs[a][0], outs[b][0])
        np.testing.assert_array_equal(outs[a][1], outs[b][1])
        assert outs[a][2] == outs[b][2]


@pytest.mark.gpu
def test_gpu_flat_trunc_mismatch_raises(gpu):
    import torch
    from rlgpu import GAE, RLGPUError
    r = torch.ones(4, device=gpu)
    t = torch.tensor([2, 0, 2, 1], dtype=torch.int8, device=gpu)
    with pytest.raises(RLGPUError, match="truncation count mismatch"):
        GAE.compute(r, t, r, torch.ones(1, device=gpu), 0.99, 0.95, 1.0, 0.0)


@pytest.mark.gpu
@pytest.mark.parametrize("T,N", [(128, 16384), (1, 5), (37, 1000)])
def test_gpu_rollout_bit_exact(gpu, T, N):
    import torch
    from rlgpu import GAE
    rng = np.random.default_rng(T * 7 + N)
    r = rng.standard_normal((T, N)).astype(np.float32)
    v = rng.standard_normal((T, N)).astype(np.float32)
    u = rng.random((T, N))
    t = np.where(u < 1 / 128, 1, np.where(u < 1 / 128 + 1 / 512, 2, 0)).astype(np.int8)
    tv = rng.standard_normal((T, N)).astype(np.float32)
    bv = rng.standard_normal(N).astype(np.float32)
    d = lambda a: torch.from_numpy(a).to(gpu)
    adv, tgt, ret = GAE.compute_rollout(d(r), d(t), d(v), d(tv), d(bv), 0.99, 0.95, 2.0, 10.0)
    ea, et, er = oracle.gae_rollout(r, t, v, tv, bv, 0.99, 0.95, 2.0, 10.0)
    np.testing.assert_array_equal(adv.cpu().numpy(), ea)
    np.testing.assert_array_equal(tgt.cpu().numpy(), et)
    np.testing.assert_array_equal(ret.cpu().numpy(), er)


def test_c1_cpu_loop_runs():
    """oracle/ppo_cpu.py (the timed C1 CPU baseline leg of bench.py) completes an iteration."""
    from oracle.ppo_cpu import run_c1
    r = run_c1(seconds=0.01, arenas=4, rollout=4, threads=2)
    assert r["iterations"] >= 1 and r["agent_steps"] == 4 * 4 * 4 * r["iterations"]
    assert r["ppo_s_per_1M_agent_steps"] > 0


def test_clip_portion_follows_the_reference_unroll():
    """GAE.cpp:113-162: |r/std| summed in groups of 8 (left to right, each group then added to the
    running float total), the remainder one by one -- restated exactly, so the clipped-reward portion
    carries the reference's rounding (values chosen so a plain sequential sum rounds differently)."""
    r = np.float32([2e8, 0, 0, 0, 0, 0, 0, 0] + [6] * 8 + [7, 5, 2])
    std, clip = 2.0, 1e7
    m = r.size
    _, _, _, cp, st = oracle.gae_flat(r, np.zeros(m, np.int8), np.zeros(m, np.float32), None, 0.99, 0.95, std, clip)
    n = r * np.float32(1 / std)
    c = np.clip(n, -clip, clip)

    def ref_sum(x):
        tot = np.float32(0)
        for g in range(0, 16, 8):
            s = np.float32(0) + x[g]
            for k in range(1, 8):
                s = np.float32(s + x[g + k])
            tot = np.float32(tot + s)
        for v in x[16:]:
            tot = np.float32(tot + v)
        return tot

    def seq_sum(x):
        tot = np.float32(0)
        for v in x:
            tot = np.float32(tot + v)
        return tot
    tot, totc = ref_sum(np.abs(n)), ref_sum(np.abs(c))
    assert st == 0 and np.float32(cp) == np.float32((tot - totc) / max(tot, np.float32(1e-7)))
    assert ref_sum(np.abs(n)) != seq_sum(np.abs(n))  # the order is observable on this input
