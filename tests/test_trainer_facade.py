"""The trainer-side drop-in (facade/GigaLearn.hpp): GGL::Learner(EnvCreateFn, LearnerConfig, StepCallbackFn) with
Start / Save / Load, as src/ExampleMain.cpp:592-598 uses it (GL/public/GigaLearnCPP/Learner.h:11-57).

  * rlgpu_train (host/example_main.cpp, the facade with registry plugins) writes a numbered checkpoint that the
    Python loader and the libtorch readers read, and a Load + Save round trip reproduces it exactly.
"""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "reinforcement-learning_amd", "rlgpu")
TRAIN = os.path.join(BIN, "rlgpu_train")


def test_host_uniform_draws():
    from rlgpu.learner import host_uniform
    u = [host_uniform(123, 1, k) for k in range(2000)]
    assert all(0.0 <= x < 1.0 for x in u)
    assert u == [host_uniform(123, 1, k) for k in range(2000)]
    assert abs(np.mean(u) - 0.5) < 0.03
    assert host_uniform(123, 2, 5) != host_uniform(123, 1, 5) != host_uniform(124, 1, 5)


def _ckpt_dir(base):
    dirs = sorted(int(d) for d in os.listdir(base) if d.isdigit())
    assert dirs, os.listdir(base)
    return os.path.join(base, str(dirs[-1])), dirs[-1]


@pytest.mark.gpu
def test_rlgpu_train_checkpoint_round_trip(gpu, tmp_path):
    import torch
    from safetensors.torch import load_file
    from rlgpu import checkpoint as ck
    a, b = tmp_path / "a", tmp_path / "b"
    args = ["--arenas", "32", "--rollout", "16", "--seed", "11"]
    r = subprocess.run([TRAIN, *args, "--iterations", "2", "--checkpoint-folder", str(a), "--self-play"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    fa, ts = _ckpt_dir(a)
    per = 16 * 4 * 32  # one iteration's steps; an old-version iteration (self-play) counts only the new team's half
    assert ts in (2 * per, per + per // 2), ts
    assert sorted(os.listdir(fa)) == sorted(["RUNNING_STATS.json", "POLICY.lt", "CRITIC.lt", "SHARED_HEAD.lt",
                                             "POLICY_OPTIM.lt", "CRITIC_OPTIM.lt", "SHARED_HEAD_OPTIM.lt",
                                             "RLGPU_OPTIM.safetensors"])
    assert os.listdir(a / "policy_versions"), "no policy version saved"
    r = subprocess.run([TRAIN, *args, "--checkpoint-folder", str(a), "--self-play", "--resave-to", str(b)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    fb, tsb = _ckpt_dir(b)
    assert tsb == ts
    assert json.load(open(os.path.join(fa, "RUNNING_STATS.json"))) == json.load(open(os.path.join(fb, "RUNNING_STATS.json")))
    for f in ("POLICY.lt", "CRITIC.lt", "SHARED_HEAD.lt"):
        x = torch.cat([t.reshape(-1) for t in ck.read_model_state(os.path.join(fa, f))])
        y = torch.cat([t.reshape(-1) for t in ck.read_model_state(os.path.join(fb, f))])
        assert torch.equal(x, y), f
    sa, sb = load_file(os.path.join(fa, "RLGPU_OPTIM.safetensors")), load_file(os.path.join(fb, "RLGPU_OPTIM.safetensors"))
    assert sa.keys() == sb.keys() and all(torch.equal(sa[k], sb[k]) for k in sa)
    assert int(sa["step"][0]) == 2 * 2  # 2 iterations x 2 epochs x 1 batch
    # the libtorch archives hold the same moments (AdamW::save read back by AdamW::load)
    shapes = {"policy": [(384, 384), (384,), (384,), (384,)] * 3 + [(90, 384), (90,)],
              "critic": [(384, 384), (384,), (384,), (384,)] * 3 + [(1, 384), (1,)],
              "shared_head": [(384, 167), (384,), (384,), (384,), (384, 384), (384,), (384,), (384,)]}
    for name, sh in shapes.items():
        step, m, v = ck.read_optim_archive(os.path.join(fa, name.upper() + "_OPTIM.lt"), sh)
        assert step == 4
        np.testing.assert_array_equal(m, sa[name + ".exp_avg"].numpy())
        np.testing.assert_array_equal(v, sa[name + ".exp_avg_sq"].numpy())
    # the Python binding loads the C++ checkpoint (Learner ctor -> checkpoint.load)
    from rlgpu.learner import Learner, LearnerConfig
    L = Learner(LearnerConfig(num_arenas=32, rollout_len=16, seed=11, shared_layers=(384, 384), policy_layers=(384,) * 3,
                              critic_layers=(384,) * 3, checkpoint_folder=str(a), train_against_old_versions=True),
                device=gpu)
    assert L.total_steps == ts and len(L.versions.versions) >= 1
    pol = torch.cat([t.reshape(-1) for t in ck.read_model_state(os.path.join(fa, "POLICY.lt"))])
    o, c = L.ppo.model_range(0)
    assert torch.equal(L.ppo.params[o:o + c].cpu(), pol)
    L.close()


@pytest.mark.gpu
def test_rlgpu_train_fp32_inference(gpu):
    """PPOLearnerConfig::useHalfPrecision = false through the trainer facade (rlgpu_train --fp32-inference): the
    Learner runs its inference on the fp32 training forward (RLGPU_INFER_F32) and trains; with self-play the
    config is refused by name (old versions are 16-bit copies only)."""
    args = ["--arenas", "16", "--rollout", "8", "--seed", "3", "--c2-model", "--fp32-inference"]
    r = subprocess.run([TRAIN, *args, "--iterations", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run([TRAIN, *args, "--iterations", "1", "--self-play"], capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "useHalfPrecision" in r.stdout + r.stderr, r.stdout + r.stderr
