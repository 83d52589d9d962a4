"""Action sampling (PPOLearner::InferActionsFromModels, GigaLearnCPP/src/private/GigaLearnCPP/PPO/
PPOLearner.cpp:78-184): the GPU sampler against the CPU oracle (oracle/sampler_ref.c).  The draw is the
reference's CPU sampler (PPOLearner.cpp:157-178: sequential running sum of the clamped probs, the first
column with r <= running, cols - 1 when none, log(max(1e-12, p))); the softmax is in the kernel's
operation order.  Given the same 16-bit logits, masks and Philox uniforms the action indices and log
probs must agree BIT FOR BIT (north_star: discrete action indices bit-exact) -- for the fused inference
kernel, the layer-by-layer path, max_rows chunking, a shared head and fp16.

CPU part: the shared exp / log kernels against libm (known answers), the oracle's draw against a numpy
transcription of the reference loop on the same probs and uniforms, and the sampler's semantics
(argmax, masks, frequencies).
"""
import numpy as np
import pytest

import oracle


def test_detmath_exp_log_known_answers():
    """rs_expf / rs_logf within 2 ulp of the correctly rounded value over the sampler's ranges."""
    rng = np.random.default_rng(0)
    x = np.concatenate([-rng.random(200_000).astype(np.float32) * 87.0, rng.random(20_000).astype(np.float32) * 88.0,
                        np.float32([0.0, -1e-30, 1e-30, -87.0, 88.0])])
    ex, _ = oracle.detmath_exp_log(x)
    want = np.exp(x.astype(np.float64)).astype(np.float32)
    ulp = np.abs(ex.view(np.int32).astype(np.int64) - want.view(np.int32).astype(np.int64))
    assert ulp.max() <= 2, ulp.max()
    assert oracle.detmath_exp_log(np.float32([-1e10, -100.0]))[0].tolist() == [0.0, 0.0]
    p = np.concatenate([rng.random(200_000).astype(np.float32), np.float32([1e-11, 1.0, 0.5, 2.0, 1e-38, 3e-39])])
    _, lg = oracle.detmath_exp_log(p)
    want = np.log(p.astype(np.float64)).astype(np.float32)
    ulp = np.abs(lg.view(np.int32).astype(np.int64) - want.view(np.int32).astype(np.int64))
    assert ulp.max() <= 2, ulp.max()
    assert lg[p == 1.0][0] == 0.0


def _bf16_bits(x):
    """Round-to-nearest-even f32 -> bf16 bit patterns."""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def test_oracle_sampler_semantics():
    rng = np.random.default_rng(1)
    n, A = 3000, 90
    logits = _bf16_bits(rng.standard_normal((n, A)) * 2)
    masks = (rng.random((n, A)) < 0.5).astype(np.uint8)
    masks[:, 7] = 1
    masks[0] = 0
    masks[0, 42] = 1  # a single valid action
    a, lp = oracle.sample_actions(logits, masks, False, 42, 3)
    assert (masks[np.arange(n), a] == 1).all() and a[0] == 42 and lp[0] == 0.0
    z = (logits.astype(np.uint32) << 16).view(np.float32).astype(np.float64) + np.where(masks, 0, -1e10)
    pr = np.exp(z - z.max(1, keepdims=True))
    pr = np.clip(pr / pr.sum(1, keepdims=True), 1e-11, 1)
    np.testing.assert_allclose(lp, np.log(pr[np.arange(n), a]), rtol=1e-5, atol=2e-6)
    ad, _ = oracle.sample_actions(logits, masks, True, 42, 3)
    np.testing.assert_array_equal(ad, pr.argmax(1))
    # one row, many draws (different steps): frequencies follow the probabilities
    one = np.repeat(logits[1:2], 20000, 0)
    m1 = np.repeat(masks[1:2], 20000, 0)
    aa, _ = oracle.sample_actions(one, m1, False, 9, 5)
    freq = np.bincount(aa, minlength=A) / aa.size
    assert np.abs(freq - pr[1] / pr[1].sum()).max() < 0.015
    # the global row counter: a chunk at row0 draws what the whole batch draws for those rows
    b, _ = oracle.sample_actions(logits[1000:], masks[1000:], False, 42, 3, row0=1000)
    np.testing.assert_array_equal(b, a[1000:])


def reference_cpu_draw(pr, r):
    """PPOLearner.cpp:157-178 in float32: running += p in column order, first j with r <= running, else the
    last column; log(std::max(1e-12f, p))."""
    n, A = pr.shape
    act = np.full(n, A - 1, np.int64)
    for i in range(n):
        running = np.float32(0)
        for j in range(A):
            running = np.float32(running + pr[i, j])
            if r[i] <= running:
                act[i] = j
                break
    p = pr[np.arange(n), act]
    return act, np.log(np.maximum(np.float32(1e-12), p).astype(np.float64)).astype(np.float32)


def test_oracle_draw_is_the_reference_cpu_loop():
    """Zero disagreement with the reference's CPU inverse CDF on 16,384 rows x 4 steps given the same
    probs and uniforms, including rows whose uniform lands past the probs' rounded
    total (picked = the last column, as the reference does)."""
    rng = np.random.default_rng(3)
    n, A = 16384, 90
    logits = _bf16_bits(rng.standard_normal((n, A)) * 3)
    masks = (rng.random((n, A)) < 0.6).astype(np.uint8)
    masks[:, 0] = 1
    for step in (0, 1, 2, 12345):
        a, lp = oracle.sample_actions(logits, masks, False, 77, step)
        pr, r = oracle.sampler_probs(logits, masks, 77, step)
        ra, rlp = reference_cpu_draw(pr, r)
        np.testing.assert_array_equal(a, ra)
        np.testing.assert_allclose(lp, rlp, rtol=3e-7, atol=1e-7)  # rs_logf vs libm log: <= 2 ulp
    # a uniform past every running sum takes the last column (here: masked) -- the reference's fallback
    pr = np.full((1, A), np.float32(1e-11))
    pr[0, 0] = np.float32(0.5)
    ra, _ = reference_cpu_draw(pr, np.float32([0.75]))
    assert ra[0] == A - 1


def test_skill_steps_draw_their_own_uniforms():
    """The skill matches sample at steps 2^40 + k (rlgpu/skill.py); the step's high 32 bits are folded into the
    Philox key (ppo_kernels.hpp sample_key), so their uniforms differ from the rollout's at step k on the same rows
    (a uint32 counter alone made them identical)."""
    rng = np.random.default_rng(5)
    n, A = 4096, 90
    logits = _bf16_bits(rng.standard_normal((n, A)))
    masks = np.ones((n, A), np.uint8)
    for k in (0, 3, 1000):
        _, r0 = oracle.sampler_probs(logits, masks, 77, k)
        _, r1 = oracle.sampler_probs(logits, masks, 77, 2**40 + k)
        assert (r0 != r1).mean() > 0.99
        _, r2 = oracle.sampler_probs(logits, masks, 77, k)
        np.testing.assert_array_equal(r0, r2)


def _gpu_logits16(p, o, fp16):
    """The policy's 16-bit logits exactly as the sampler reads them (forward(..., half=True) returns
    their exact f32 values)."""
    f = p.forward(0, o, half=True).cpu().numpy()
    return f.astype(np.float16).view(np.uint16) if fp16 else (f.view(np.uint32) >> 16).astype(np.uint16)


@pytest.mark.gpu
@pytest.mark.parametrize("kw,fp16,fused,chunk", [
    (dict(), False, True, False),
    (dict(), False, False, False),
    (dict(), False, True, True),
    (dict(shared_layers=(384, 384), policy_layers=(384,) * 3, critic_layers=(384,) * 3), False, True, False),
    (dict(policy_layers=(256, 256)), True, True, False),
    (dict(policy_layers=(256, 256)), True, False, True)],
    ids=["c2-fused", "c2-layer", "c2-fused-chunked", "shared-head", "fp16-fused", "fp16-layer-chunked"])
def test_sampler_bit_exact_vs_oracle(gpu, monkeypatch, kw, fp16, fused, chunk):
    """16,384 rows (C2's agents per GPU) over several steps: sampled and argmax indices bit-exact, log
    probs bit-exact (and within 1e-6 relative + a few ulp of 1 absolute of float64 log softmax)."""
    import torch
    from rlgpu.ppo import PPO
    from test_ppo import make_batch
    if not fused:
        monkeypatch.setenv("RLGPU_FUSED_INFER", "0")
    n = 16384
    p = PPO(max_rows=6000 if chunk else n, seed=31, infer_fp16=fp16, **kw)
    rng = np.random.default_rng(7)
    obs, masks, *_ = make_batch(rng, n)
    masks[::97] = 0
    masks[::97, 11] = 1  # rows with one valid action
    o, m = torch.from_numpy(obs).to(gpu), torch.from_numpy(masks).to(gpu)
    logits = np.concatenate([_gpu_logits16(p, o[i:i + p.max_rows], fp16) for i in range(0, n, p.max_rows)])
    for det in (True, False):
        for step in (0, 1, 77, 2**31 + 5, 2**40 + 5):  # 2^40 + k: the skill matches' step range
            a, lp = p.infer_actions(o, m, step=step, deterministic=det)
            wa, wlp = oracle.sample_actions(logits, masks, det, p.cfg.seed, step, 0, fp16)
            ga, glp = a.cpu().numpy(), lp.cpu().numpy()
            bad = np.nonzero(ga != wa)[0]
            assert bad.size == 0, (step, det, bad[:5], ga[bad[:5]], wa[bad[:5]])
            np.testing.assert_array_equal(glp.view(np.uint32), wlp.view(np.uint32))
    lf = logits.view(np.float16).astype(np.float64) if fp16 else (logits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    z = lf + np.where(masks, 0, -1e10)
    pr = np.exp(z - z.max(1, keepdims=True))
    pr = np.clip(pr / pr.sum(1, keepdims=True), 1e-11, 1)
    ref = np.log(pr[np.arange(n), ga])
    assert np.all(np.abs(glp - ref) <= 1e-6 * np.abs(ref) + 5e-7), np.abs(glp - ref).max()


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(), dict(shared_layers=(384, 384), policy_layers=(384,) * 3, critic_layers=(384,) * 3)],
                         ids=["c2", "shared-head"])
def test_fp32_inference_bit_exact_vs_oracle(gpu, kw):
    """PPOLearnerConfig::useHalfPrecision = false (RLGPU_INFER_F32, Models.cpp:36-68's fp32 branch): the policy's
    fp32 logits (the training forward) sampled by the same sampler -- actions and log probs bit-exact to the
    oracle sampler on those fp32 logits; the critic's values equal the fp32 forward; self-play inference is
    refused by name."""
    import torch
    from rlgpu.ppo import PPO
    from test_ppo import make_batch
    n = 12000
    p = PPO(max_rows=5000, seed=41, infer_fp16=2, **kw)
    rng = np.random.default_rng(9)
    obs, masks, *_ = make_batch(rng, n)
    masks[::89] = 0
    masks[::89, 5] = 1
    o, m = torch.from_numpy(obs).to(gpu), torch.from_numpy(masks).to(gpu)
    logits = np.concatenate([p.forward(0, o[i:i + 5000]).cpu().numpy() for i in range(0, n, 5000)])
    assert logits.dtype == np.float32
    for det in (True, False):
        for step in (0, 3, 2**31 + 1):
            a, lp = p.infer_actions(o, m, step=step, deterministic=det)
            wa, wlp = oracle.sample_actions(logits, masks, det, p.cfg.seed, step, 0)
            np.testing.assert_array_equal(a.cpu().numpy(), wa)
            np.testing.assert_array_equal(lp.cpu().numpy().view(np.uint32), wlp.view(np.uint32))
    v = p.infer_critic(o).cpu().numpy().ravel()
    want = np.concatenate([p.forward(1, o[i:i + 5000]).cpu().numpy().ravel() for i in range(0, n, 5000)])
    np.testing.assert_array_equal(v.view(np.uint32), want.view(np.uint32))
    # the fp32 logits differ from the bf16 path's (it is not the 16-bit inference under another name)
    assert not np.array_equal(logits, p.forward(0, o[:5000], half=True).cpu().numpy())
    from rlgpu._lib import RLGPUError
    p.set_version(p.policy_version())
    with pytest.raises(RLGPUError, match="fp32 inference"):
        p.infer_actions_mixed(o, m, torch.zeros(n, dtype=torch.uint8, device=gpu), step=0)
