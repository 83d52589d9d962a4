"""Checkpoint format compatibility (rlgpu/checkpoint.py).  CPU only.

Anchor: libtorch itself.  tools/lt_load_check.cpp restates GGL::Model's Sequential and loads our
<NAME>.lt with torch::load(seq, stream) exactly as Model::Load does (Models.cpp:130-166); it also
writes a module with torch::save(seq, stream) (Model::Save, Models.cpp:116-120) for the reverse
direction.  The harness is compiled here against the installed libtorch (skipped if that fails).
"""
import json
import os
import subprocess

import numpy as np
import pytest

from rlgpu import checkpoint as ckpt
from rlgpu.learner import WelfordStat
from rlgpu.ppo import make_sequential

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    import torch.utils.cpp_extension as ext
    out = tmp_path_factory.mktemp("lt") / "lt_load_check"
    inc = sum([["-I", p] for p in ext.include_paths()], [])
    libs = ext.library_paths()
    cmd = ["g++", "-std=c++17", "-O1", os.path.join(ROOT, "tools", "lt_load_check.cpp"), *inc,
           "-L" + libs[0], "-ltorch", "-ltorch_cpu", "-lc10", "-Wl,-rpath," + libs[0], "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        pytest.skip("cannot build the libtorch harness: " + r.stderr[-400:])
    return str(out)


ARCH = dict(obs=167, out=90, ln=1, layers=(64, 48))


def _args():
    return [str(ARCH["obs"]), str(ARCH["out"]), str(ARCH["ln"])] + [str(h) for h in ARCH["layers"]]


def test_model_file_loads_in_libtorch(harness, tmp_path):
    import torch
    torch.manual_seed(3)
    seq = make_sequential(ARCH["obs"], ARCH["out"], ARCH["layers"], True)
    with torch.no_grad():  # non-trivial LayerNorm affine parameters
        for m in seq:
            if isinstance(m, torch.nn.LayerNorm):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    p = str(tmp_path / "POLICY.lt")
    ckpt.write_model(seq, p)
    x = np.random.default_rng(0).standard_normal((7, ARCH["obs"])).astype(np.float32)
    x.tofile(tmp_path / "x.f32")
    r = subprocess.run([harness, "load", p, str(tmp_path / "x.f32"), "7", str(tmp_path / "y.f32"), *_args()],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    y = np.fromfile(tmp_path / "y.f32", np.float32).reshape(7, ARCH["out"])
    with torch.no_grad():
        want = seq(torch.from_numpy(x)).numpy()
    np.testing.assert_allclose(y, want, rtol=1e-5, atol=1e-6)


def test_libtorch_written_model_loads_here(harness, tmp_path):
    import torch
    n = sum(p.numel() for p in make_sequential(ARCH["obs"], ARCH["out"], ARCH["layers"], True).parameters())
    flat = np.random.default_rng(1).standard_normal(n).astype(np.float32)
    flat.tofile(tmp_path / "p.f32")
    p = str(tmp_path / "CRITIC.lt")
    r = subprocess.run([harness, "save", str(tmp_path / "p.f32"), p, *_args()], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    got = torch.cat([t.reshape(-1) for t in ckpt.read_model_state(p)]).numpy()
    np.testing.assert_array_equal(got, flat)


def test_size_mismatch_is_refused(harness, tmp_path):
    seq = make_sequential(ARCH["obs"], ARCH["out"], (32, 48), True)
    p = str(tmp_path / "POLICY.lt")
    ckpt.write_model(seq, p)
    np.zeros((1, ARCH["obs"]), np.float32).tofile(tmp_path / "x.f32")
    r = subprocess.run([harness, "load", p, str(tmp_path / "x.f32"), "1", str(tmp_path / "y.f32"), *_args()],
                       capture_output=True, text=True)
    assert r.returncode != 0


def test_numbered_dirs_and_paths(tmp_path):
    for n in ("100", "2000", "abc", "12x"):
        (tmp_path / n).mkdir()
    (tmp_path / "300").write_text("file, not a dir")
    assert ckpt.numbered_dirs(str(tmp_path)) == {100, 2000}
    assert ckpt.numbered_dirs(str(tmp_path / "missing")) == set()
    assert ckpt.model_path("d", "policy") == os.path.join("d", "POLICY.lt")
    assert ckpt.model_path("d", "critic", "_optim") == os.path.join("d", "CRITIC_OPTIM.lt")


def test_welford_stat_reference_rules():
    w = WelfordStat()
    assert w.std() == 1.0 and w.get_mean() == 0.0
    w.add([3.0])
    assert w.std() == 1.0  # count < 2
    w.add([3.0])
    assert w.std() == 1.0  # variance 0 -> 1 (WelfordStat.h:43-47)
    xs = np.random.default_rng(0).standard_normal(500).astype(np.float32)
    v = WelfordStat()
    v.add(xs)
    assert abs(v.std() - np.std(xs.astype(np.float64), ddof=1)) < 1e-9
    j = json.loads(json.dumps(v.to_json()))
    assert set(j) == {"mean", "var", "count"}
    u = WelfordStat()
    u.read_json(j)
    assert (u.n, u.mean, u.m2) == (v.n, v.mean, v.m2)


def test_model_reader_executes_nothing(tmp_path):
    """read_model_state admits only tensor rebuilds, OrderedDict and inert module stand-ins: an archive
    whose data.pkl names any other global is refused before anything runs (user-supplied
    POLICY.lt / policy_versions archives are untrusted input)."""
    import pickle
    import zipfile
    marker = tmp_path / "ran"

    class Evil:
        def __reduce__(self):
            return (os.system, (f"touch {marker}",))

    p = str(tmp_path / "POLICY.lt")
    with zipfile.ZipFile(p, "w") as z:
        z.writestr("POLICY/data.pkl", pickle.dumps(Evil(), protocol=2))
    with pytest.raises(pickle.UnpicklingError):
        ckpt.read_model_state(p)
    assert not marker.exists()
    with zipfile.ZipFile(str(tmp_path / "x.lt"), "w") as z:
        z.writestr("x/other.bin", b"")
    with pytest.raises(ValueError):
        ckpt.read_model_state(str(tmp_path / "x.lt"))


def test_model_reader_matches_parameters(tmp_path):
    """The code-free reader returns exactly the module's parameters() in order."""
    import torch
    torch.manual_seed(5)
    seq = make_sequential(ARCH["obs"], ARCH["out"], ARCH["layers"], True)
    p = str(tmp_path / "POLICY.lt")
    ckpt.write_model(seq, p)
    got = ckpt.read_model_state(p)
    want = list(seq.parameters())
    assert [t.shape for t in got] == [w.shape for w in want]
    for g, w in zip(got, want):
        assert torch.equal(g, w.detach())


def test_shared_head_file_loads_in_libtorch(harness, tmp_path):
    """SHARED_HEAD.lt (Models.h:114-128, the shared head of PPOLearner::MakeModels: hidden layers,
    no output Linear) loads into libtorch's Sequential built with addOutputLayer = false, and a
    libtorch-written shared head reads back here."""
    import torch
    torch.manual_seed(4)
    seq = make_sequential(ARCH["obs"], None, (64, 32), True)
    p = str(tmp_path / "SHARED_HEAD.lt")
    assert ckpt.model_path(str(tmp_path), "shared_head") == p
    ckpt.write_model(seq, p)
    x = np.random.default_rng(2).standard_normal((5, ARCH["obs"])).astype(np.float32)
    x.tofile(tmp_path / "x.f32")
    args = [str(ARCH["obs"]), "0", "1", "64", "32"]
    r = subprocess.run([harness, "load", p, str(tmp_path / "x.f32"), "5", str(tmp_path / "y.f32"), *args],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    y = np.fromfile(tmp_path / "y.f32", np.float32).reshape(5, 32)
    with torch.no_grad():
        np.testing.assert_allclose(y, seq(torch.from_numpy(x)).numpy(), rtol=1e-5, atol=1e-6)
    n = sum(q.numel() for q in seq.parameters())
    flat = np.random.default_rng(3).standard_normal(n).astype(np.float32)
    flat.tofile(tmp_path / "p.f32")
    q = str(tmp_path / "LT_SHARED_HEAD.lt")
    r = subprocess.run([harness, "save", str(tmp_path / "p.f32"), q, *args], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    got = torch.cat([t.reshape(-1) for t in ckpt.read_model_state(q)]).numpy()
    np.testing.assert_array_equal(got, flat)


def _shapes():
    import torch
    from rlgpu.ppo import make_sequential
    seq = make_sequential(ARCH["obs"], ARCH["out"], ARCH["layers"], bool(ARCH["ln"]))
    return [tuple(p.shape) for p in seq.parameters()]


def test_reference_optimizer_archive_reads(harness, tmp_path):
    """A reference-written <NAME>_OPTIM.lt (libtorch AdamW after 3 steps, saved as Model::Save does,
    Models.cpp:122-125) reads back through rlgpu's reader -- libtorch's AdamW::load, as Model::Load
    (Models.cpp:177-180) -- with the exact step and moments, mapped by parameter order."""
    import numpy as np
    from rlgpu.checkpoint import OPTIM_TOOL, read_optim_archive
    if not os.path.exists(OPTIM_TOOL):
        pytest.skip("rlgpu_optim_lt not built")
    p, dump = str(tmp_path / "POLICY_OPTIM.lt"), str(tmp_path / "dump.bin")
    r = subprocess.run([harness, "optim", p, dump, "3", *_args()], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    raw = open(dump, "rb").read()
    shapes = _shapes()
    n = sum(int(np.prod(s)) for s in shapes)
    want_step, want = int(np.frombuffer(raw[:8], np.int64)[0]), np.frombuffer(raw[8:], np.float32)
    step, m, v = read_optim_archive(p, shapes)
    assert step == want_step == 3
    np.testing.assert_array_equal(m, want[:n])
    np.testing.assert_array_equal(v, want[n:])


def test_optimizer_archive_round_trip(tmp_path):
    """rlgpu's <NAME>_OPTIM.lt writer (libtorch AdamW::save) and reader (AdamW::load) round-trip the
    step and both moments bit for bit."""
    import numpy as np
    from rlgpu.checkpoint import OPTIM_TOOL, read_optim_archive, write_optim_archive
    if not os.path.exists(OPTIM_TOOL):
        pytest.skip("rlgpu_optim_lt not built")
    shapes = _shapes()
    n = sum(int(np.prod(s)) for s in shapes)
    rng = np.random.default_rng(2)
    m, v = rng.standard_normal(n).astype(np.float32), rng.random(n).astype(np.float32)
    p = str(tmp_path / "CRITIC_OPTIM.lt")
    write_optim_archive(p, shapes, 41, 2.5e-4, (0.9, 0.999), 1e-8, 1e-2, m, v)
    step, m2, v2 = read_optim_archive(p, shapes)
    assert step == 41
    np.testing.assert_array_equal(m2, m)
    np.testing.assert_array_equal(v2, v)


def test_optimizer_archive_without_reader_raises(tmp_path, monkeypatch):
    """A checkpoint holding <NAME>_OPTIM.lt but no RLGPU_OPTIM.safetensors, loaded by a build without
    rlgpu_optim_lt: the load fails instead of silently resetting the saved AdamW moments."""
    import json
    import torch
    seq = make_sequential(ARCH["obs"], ARCH["out"], ARCH["layers"], True)
    d = tmp_path / "100"
    d.mkdir()
    ckpt.write_model(seq, str(d / "POLICY.lt"))
    (d / "POLICY_OPTIM.lt").write_bytes(b"PK\x03\x04 not empty")
    (d / ckpt.STATS_FILE).write_text(json.dumps({"total_timesteps": 100, "total_iterations": 1}))
    n = sum(p.numel() for p in seq.parameters())

    class _PPO:
        models = (0,)
        params = torch.zeros(n)

        def model_sizes(self, mi):
            return [p.numel() for p in seq.parameters()]

        def model_range(self, mi):
            return 0, n

        def refresh_half(self):
            pass

        def optimizer_state(self):
            return 0, torch.ones(n), torch.ones(n)

        def set_optimizer_step(self, step):
            assert step == 0

    class _Learner:
        total_steps = iteration = 0
        return_stat = None
        ppo = _PPO()

    monkeypatch.setattr(ckpt, "OPTIM_TOOL", str(tmp_path / "no_such_tool"))
    with pytest.raises(RuntimeError, match="holds optimizer state"):
        ckpt.load(_Learner(), str(tmp_path))
    # an empty archive is the reference's "cannot use": that model's optimizer resets, with a warning
    (d / "POLICY_OPTIM.lt").write_bytes(b"")
    L = _Learner()
    with pytest.warns(UserWarning, match="optimizer will be reset"):
        ckpt.load(L, str(tmp_path))
    assert L.ppo.optimizer_state()[1].sum() == n  # a fresh tensor each call: nothing else touched
