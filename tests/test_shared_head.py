"""The shared head (PPOLearnerConfig::sharedHead) through the whole PPO stack: create, training
forward / minibatch backward, AdamW, 16-bit inference (fused and layer-by-layer), self-play versions
and the Learner with ExampleMain's own topology.

Reference: PPOLearner::MakeModels (GigaLearnCPP/src/private/GigaLearnCPP/PPO/PPOLearner.cpp:42-74:
shared head = [Linear -> LayerNorm -> LeakyReLU] x k without an output layer, policy / critic take its
last width), InferPolicyProbsFromModels / InferCritic (:90-91, :188-191: shared head first), Learn
(:395-398 one shared forward per minibatch, :403/:474 both heads read it, :498 one backward of
ppoLoss + criticLoss, :526 clip_grad_norm_ of the shared head), SetLearningRates (:652-663: shared LR
= min(policy, critic)), run_out.log:25-39 (ExampleMain's [384, 384] / [384] x 3 and parameter counts).

The checker is a plain PyTorch fp32 restatement of those lines (libtorch is unpinned);
tolerances as tests/test_ppo.py.
"""
import numpy as np
import pytest

from test_ppo import assert_grads_close, make_batch

EXAMPLE = dict(shared_layers=(384, 384), policy_layers=(384, 384, 384), critic_layers=(384, 384, 384))
SMALL = dict(shared_layers=(96, 64), policy_layers=(80,), critic_layers=(48, 40))


def _ref_minibatch(shared, pol, crit, obs, masks, acts, old_logp, adv, target, batch_size, clip=0.2, ent_scale=0.035):
    """PPOLearner::Learn minibatch body with a shared head (PPOLearner.cpp:395-498), fp32 torch."""
    import math

    import torch
    n = obs.shape[0]
    bsr = n / float(batch_size)
    feats = shared(obs)
    logits = pol(feats) + -1e10 * masks.bool().logical_not()
    probs = torch.softmax(logits, -1).clamp(1e-11, 1.0)
    logp = probs.gather(-1, acts.long().unsqueeze(-1)).squeeze(-1).log()
    ent = (-(probs.log() * probs).sum(-1) / math.log(probs.shape[1])).mean()
    ratio = (logp - old_logp).exp()
    pl = -torch.min(ratio * adv, ratio.clamp(1 - clip, 1 + clip) * adv).mean()
    closs = torch.nn.functional.mse_loss(crit(feats).flatten(), target) * bsr
    ((pl - ent * ent_scale) * bsr + closs).backward()


def test_shared_param_counts_known_answer_cpu():
    """run_out.log:36-39 through the Python model description (no GPU)."""
    from rlgpu.ppo import param_count
    assert param_count(167, 0, [384, 384], out=0) == 213_888
    assert param_count(384, 90, [384] * 3) == 480_474
    assert param_count(384, 1, [384] * 3, out=1) == 446_209


@pytest.mark.gpu
def test_engine_param_counts_example_main(gpu):
    """rlgpu_ppo_create with ExampleMain's topology holds exactly the reference's parameter counts,
    and its torch modules are the reference's module lists."""
    from rlgpu.ppo import PPO
    p = PPO(max_rows=256, seed=1, **EXAMPLE)
    assert [p.model_range(m)[1] for m in (0, 1, 2)] == [480_474, 446_209, 213_888]
    assert p.flat().numel() == 1_140_571  # "[Total]: 1,140,571"
    assert len(p.torch_module(2)) == 6  # (Linear, LayerNorm, LeakyReLU) x 2, no output Linear
    nosh = PPO(max_rows=64, seed=1)
    assert nosh.model_range(2)[1] == 0


@pytest.mark.gpu
def test_shared_forward_fp32_matches_torch(gpu):
    import torch
    from rlgpu.ppo import PPO
    p = PPO(max_rows=1024, seed=3, **EXAMPLE)
    x = torch.randn(700, 167)
    for m in (0, 1, 2):
        want = p.torch_chain(m)(x).detach()
        got = p.forward(m, x.to(gpu)).cpu()
        np.testing.assert_allclose(got.numpy(), want.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 2], ids=["x6", "f32", "h3"])
@pytest.mark.parametrize("arch,n,slope", [(EXAMPLE, 700, 1.0), (EXAMPLE, 1029, 0.01), (SMALL, 333, 1.0)])
def test_shared_minibatch_grads_match_torch(gpu, mode, arch, n, slope):
    """Gradients of policy, critic and shared head (the sum of both heads' input gradients) against
    the torch restatement; kink-free slope 1.0 to rel 1e-4 on every element, LeakyReLU 0.01 to the
    Frobenius bound of tests/test_ppo.py."""
    import torch
    from rlgpu.ppo import PPO
    rng = np.random.default_rng(n + mode)
    p = PPO(max_rows=2048, seed=7, leaky_slope=slope, train_gemm=mode, **arch)
    sh, pol, crit = p.torch_module(2), p.torch_module(0), p.torch_module(1)
    obs, masks, acts, old, adv, tgt = make_batch(rng, n)
    T = lambda a: torch.from_numpy(a)  # noqa: E731
    advn = ((adv - adv.mean()) / (adv.std(ddof=1) + 1e-8)).astype(np.float32)
    _ref_minibatch(sh, pol, crit, T(obs), T(masks), T(acts), T(old), T(advn), T(tgt), n)
    d = [T(v).to(gpu) for v in (obs, masks, acts, old, adv, tgt)]
    p.adv_normalizer(d[4])
    p.zero_grad()
    p.minibatch(*d, None, 0, n, n)
    got = p.flat(grads=True).cpu()
    if slope == 1.0:
        assert_grads_close(got, pol, crit, sh, rel_tol=1e-4, frac=1.0)
    else:
        assert_grads_close(got, pol, crit, sh)


@pytest.mark.gpu
def test_shared_optimizer_step_matches_torch_adamw(gpu):
    """clip_grad_norm_ per model (the shared head too, PPOLearner.cpp:526) and AdamW with the shared
    head at min(policyLR, criticLR) (:652-663), three steps against torch."""
    import torch
    from rlgpu.ppo import PPO
    rng = np.random.default_rng(21)
    p = PPO(max_rows=1024, seed=15, policy_lr=1e-3, critic_lr=5e-4, **SMALL)
    sh, pol, crit = p.torch_module(2), p.torch_module(0), p.torch_module(1)
    opts = [torch.optim.AdamW(pol.parameters(), lr=1e-3), torch.optim.AdamW(crit.parameters(), lr=5e-4),
            torch.optim.AdamW(sh.parameters(), lr=5e-4)]
    T = lambda a: torch.from_numpy(a)  # noqa: E731
    for _ in range(3):
        obs, masks, acts, old, adv, tgt = make_batch(rng, 400)
        advn = ((adv - adv.mean()) / (adv.std(ddof=1) + 1e-8)).astype(np.float32)
        for o in opts:
            o.zero_grad(set_to_none=True)
        _ref_minibatch(sh, pol, crit, T(obs), T(masks), T(acts), T(old), T(advn), T(tgt), 400)
        for m in (pol, crit, sh):
            torch.nn.utils.clip_grad_norm_(m.parameters(), 0.5)
        for o in opts:
            o.step()
        d = [T(v).to(gpu) for v in (obs, masks, acts, old, adv, tgt)]
        p.adv_normalizer(d[4])
        p.minibatch(*d, None, 0, 400, 400)
        p.optimizer_step()
    want = torch.cat([q.detach().reshape(-1) for m in (pol, crit, sh) for q in m.parameters()])
    got = p.flat().cpu()
    diff = np.abs(got.numpy() - want.numpy())
    tight = diff <= 1e-4 * np.abs(want.numpy()) + 2e-6
    assert tight.mean() > 0.9999, tight.mean()
    assert diff.max() < 0.1 * 1e-3, diff.max()
    assert p.read_metrics()["Shared Head Grad Norm"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("arch,fp16", [(EXAMPLE, False), (SMALL, True)])
def test_shared_fused_inference_matches_layer_path(gpu, monkeypatch, arch, fp16):
    """The fused inference kernel runs the 3-model chain (shared head -> policy / critic) in one launch,
    bit-identical to the layer-by-layer path; an old version carries its own shared head."""
    import torch
    from rlgpu.ppo import PPO
    n = 2000 + 13
    p = PPO(max_rows=n, seed=11, infer_fp16=fp16, **arch)
    rng = np.random.default_rng(5)
    obs, masks, *_ = make_batch(rng, n)
    o, m = torch.from_numpy(obs).to(gpu), torch.from_numpy(masks).to(gpu)
    old_rows = torch.from_numpy((rng.random(n) < 0.5).astype(np.uint8)).to(gpu)
    v = p.policy_version()
    assert v.numel() == p.model_range(0)[1] + p.model_range(2)[1]
    p.set_version(v * 0.5)

    def run():
        torch.cuda.synchronize()
        res = [p.forward(0, o, half=True).cpu(), p.forward(2, o, half=True).cpu(), p.infer_critic(o).cpu()]
        for det in (False, True):
            a, lp = p.infer_actions(o, m, step=5, deterministic=det)
            res += [a.cpu(), lp.cpu()]
        a, lp = p.infer_actions_mixed(o, m, old_rows, step=9)
        res += [a.cpu(), lp.cpu()]
        torch.cuda.synchronize()
        return res

    fused = run()
    monkeypatch.setenv("RLGPU_FUSED_INFER", "0")
    layer = run()
    for nm, f, l in zip(["logits", "shared", "values", "actions", "logp", "argmax", "logp_det", "mixed", "mixed_logp"],
                        fused, layer):
        assert torch.equal(f, l), (nm, (f != l).sum().item())
    # the 16-bit chain is close to the fp32 torch chain
    x = torch.from_numpy(obs[:300])
    for mi in (0, 1):
        want = p.torch_chain(mi)(x).detach().numpy()
        got = (fused[0][:300] if mi == 0 else fused[2][:300, None]).numpy()
        assert np.abs(got - want).max() <= 3e-2 * np.abs(want).max() + 1e-3, mi


@pytest.mark.gpu
def test_shared_version_roundtrip_and_checkpoint(gpu, tmp_path):
    """A Learner with ExampleMain's topology: one iteration moves all three models; the checkpoint
    holds POLICY.lt, CRITIC.lt and SHARED_HEAD.lt plus the optimizer state of all three, and a new
    Learner resumes bit-identically; the self-play version holds policy + shared head and its folder
    POLICY.lt + SHARED_HEAD.lt (PolicyVersionManager.cpp:64-104, ModelSet::Save of GetPolicyModels)."""
    import os

    import torch
    from rlgpu.learner import Learner, LearnerConfig
    folder = str(tmp_path / "ck")
    cfg = LearnerConfig(num_arenas=16, rollout_len=16, mini_batch_size=512, seed=9, checkpoint_folder=folder,
                        ts_per_save=0, **EXAMPLE)
    L = Learner(cfg, device=gpu)
    before = [L.ppo.model_slice(m).clone() for m in (0, 1, 2)]
    L.iterate()
    for m in (0, 1, 2):
        assert not torch.equal(before[m], L.ppo.model_slice(m)), m
    ck = L.last_checkpoint
    for name in ("POLICY.lt", "CRITIC.lt", "SHARED_HEAD.lt"):
        assert os.path.exists(os.path.join(ck, name)), name
    v = L.versions.versions[0]
    assert torch.equal(v.params, L.ppo.policy_version())
    L.save()
    vdir = os.path.join(folder, "policy_versions", str(v.timesteps))
    assert sorted(os.listdir(vdir)) == ["POLICY.lt", "SHARED_HEAD.lt", "STATS.json"]
    L2 = Learner(cfg, device=gpu)
    assert torch.equal(L2.ppo.flat(), L.ppo.flat())
    s1, m1, v1 = L.ppo.optimizer_state()
    s2, m2, v2 = L2.ppo.optimizer_state()
    assert s1 == s2 and torch.equal(m1, m2) and torch.equal(v1, v2)
    assert torch.equal(L2.versions.versions[0].params, v.params)
    x = L.obs[0][:64].contiguous()
    assert torch.equal(L.ppo.forward(0, x, half=True), L2.ppo.forward(0, x, half=True))
