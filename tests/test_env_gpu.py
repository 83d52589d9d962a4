"""Arena-set parity: the HIP env kernel (rlgpu.EnvSet over include/rlgpu_env.h) against the
CPU oracle (oracle.EnvSet, oracle/rsim_ref.cpp + oracle/env_ref.cpp).

Both sides restate RocketSim Arena::Step + RLGymCPP EnvSet::StepFirstHalf/StepSecondHalf
(GigaLearnCPP/RLGymCPP/src/RLGymCPP/EnvSet/EnvSet.cpp:113-273) with strict IEEE float and
deterministic trig, so the bar is BIT-EXACT on every field of the arena record, the obs rows,
the action masks, the rewards and the terminal codes, step after step.
"""
import numpy as np
import pytest

import oracle
from tests_util import arena_diff, random_actions

pytestmark = pytest.mark.gpu


def _mk(n, seed, gpu):
    from rlgpu.env import EnvSet
    return EnvSet(n, seed=seed, device=gpu), oracle.EnvSet(n, seed=seed)


def _state(env):
    from rlgpu.state import ARENA
    return np.frombuffer(env.get_arenas().tobytes(), ARENA)


def _check(g, o, what):
    import torch
    torch.cuda.synchronize()
    d = arena_diff(_state(g), _state(o))
    assert not d, f"{what}: arena state differs\n" + "\n".join(d)
    go = g.obs.cpu().numpy()
    bad = np.nonzero((go.view(np.uint32) != o.obs.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, f"{what}: obs rows differ {bad[:8]} max|d|={np.abs(go - o.obs).max()}"
    np.testing.assert_array_equal(g.action_masks.cpu().numpy(), o.masks, err_msg=what + ": masks")


def _check_step(g, o, what):
    _check(g, o, what)
    np.testing.assert_array_equal(g.rewards.cpu().numpy().view(np.uint32), o.rewards.view(np.uint32),
                                  err_msg=what + ": rewards")
    np.testing.assert_array_equal(g.terminals.cpu().numpy(), o.terminals, err_msg=what + ": terminals")


def test_env_create_reset_parity(gpu):
    g, o = _mk(37, 11, gpu)
    _check(g, o, "create")


def test_env_trajectory_parity(gpu):
    import torch
    n, steps = 48, 200
    g, o = _mk(n, 5, gpu)
    rng = np.random.default_rng(0)
    saw = set()
    for t in range(steps):
        a = random_actions(o.masks, rng)
        o.step(a, True)
        g.step(torch.from_numpy(a).to(gpu), True)
        saw.update(np.unique(o.terminals).tolist())
        _check_step(g, o, f"step {t}")
    assert 2 in saw or 1 in saw, "trajectory never terminated; extend it"


def test_env_two_half_api_matches_fused(gpu):
    import torch
    n = 16
    g, o = _mk(n, 3, gpu)
    rng = np.random.default_rng(1)
    for t in range(30):
        a = random_actions(o.masks, rng)
        o.step_first_half()
        o.step_second_half(a)
        o.reset()
        g.step_first_half()
        g.step_second_half(torch.from_numpy(a).to(gpu))
        g.reset()
        _check(g, o, f"two-half step {t}")


def test_env_perturbed_contacts_parity(gpu):
    """Ball thrown at cars / walls / ceiling from random states: exercises car-ball,
    ball-world (special contacts), car-car bumps and demos, wall rides."""
    import torch
    from rlgpu.state import ARENA
    n = 64
    g, o = _mk(n, 21, gpu)
    rng = np.random.default_rng(2)
    for t in range(20):
        a = random_actions(o.masks, rng)
        o.step(a, True)
    st = np.frombuffer(o.get_arenas().tobytes(), ARENA).copy()
    # ball velocities toward the cars, random spins; cars given speed toward each other
    for i in range(n):
        c = st["cars"][i]["body"]["pos"][i % 4]
        b = st["ball"][i]["pos"]
        d = c - b
        st["ball"][i]["vel"] = (d / (np.linalg.norm(d) + 1e-6) * rng.uniform(10, 110)).astype(np.float32)
        st["ball"][i]["angvel"] = rng.uniform(-6, 6, 3).astype(np.float32)
        for k in range(4):
            other = st["cars"][i]["body"]["pos"][(k + 1) % 4]
            dd = other - st["cars"][i]["body"]["pos"][k]
            st["cars"][i]["body"]["vel"][k] = (dd / (np.linalg.norm(dd) + 1e-6) * rng.uniform(0, 46)).astype(np.float32)
    buf = np.frombuffer(st.tobytes(), np.uint8)
    o.set_arenas(buf)
    g.set_arenas(buf)
    for t in range(40):
        a = random_actions(o.masks, rng)
        o.step(a, True)
        g.step(torch.from_numpy(a).to(gpu), True)
        _check_step(g, o, f"perturbed step {t}")


def _stacked_states(st, rng):
    """Cars parked on the ball and on each other, high above the floor: their wheel rays end on the ball's
    sphere or another car's box (btSubsimplexConvexCast, btCollisionWorld.cpp:277-310)."""
    n = st.shape[0]
    for i in range(n):
        x, y = rng.uniform(-30, 30), rng.uniform(-40, 40)
        st["ball"]["pos"][i] = (x, y, 6.0)
        st["ball"]["vel"][i] = 0
        st["ball"]["angvel"][i] = rng.uniform(-1, 1, 3)
        for k in range(4):
            body = st["cars"]["body"][i, k]
            body["vel"] = rng.uniform(-0.2, 0.2, 3)
            body["angvel"] = rng.uniform(-0.3, 0.3, 3)
            a = rng.uniform(-0.2, 0.2)
            body["rot"] = np.array([np.cos(a), -np.sin(a), 0, np.sin(a), np.cos(a), 0, 0, 0, 1], np.float32)
        cars = st["cars"]["body"]["pos"][i]
        cars[0] = (x + rng.uniform(-0.4, 0.4), y + rng.uniform(-0.4, 0.4), 6.0 + 1.825 + rng.uniform(0.35, 0.7))
        cars[1] = (x + 12, y, 5.0)
        cars[2] = (x + 12 + rng.uniform(-0.5, 0.5), y + rng.uniform(-0.5, 0.5), 5.0 + rng.uniform(0.9, 1.3))
        cars[3] = (x - 12, y + rng.uniform(-2, 2), 0.4)
    return st


def test_env_wheel_rays_on_dynamic_bodies_parity(gpu):
    import torch
    from rlgpu.state import ARENA
    n = 64
    g, o = _mk(n, 31, gpu)
    rng = np.random.default_rng(5)
    st = _stacked_states(np.frombuffer(o.get_arenas().tobytes(), ARENA).copy(), rng)
    buf = np.frombuffer(st.tobytes(), np.uint8)
    o.set_arenas(buf)
    g.set_arenas(buf)
    elevated_contacts = 0
    for t in range(30):
        a = random_actions(o.masks, rng)
        o.step(a, False)
        g.step(torch.from_numpy(a).to(gpu), False)
        _check_step(g, o, f"stacked step {t}")
        s = _state(o)
        high = s["cars"]["body"]["pos"][..., 2] > 2.5
        elevated_contacts += int((s["cars"]["wheel_contact"].any(-1) & high).sum())
    assert elevated_contacts > 0, "no wheel ray reached the ball or a car"
    print(f"wheel contacts of cars standing on the ball / a car: {elevated_contacts}")


def test_env_custom_mesh_parity(gpu):
    """A dense 8-object collision mesh loaded from .cmf images (bumpy heightfield floor, side
    ramps, back walls; 3.5k triangles): wheel rays, ball and car contacts against the uniform-grid
    index on the GPU must equal the oracle's scan of every triangle in index order, with one
    manifold per (body, mesh object) pair."""
    import warnings

    import torch
    from rlgpu.env import EnvSet
    from rlgpu.mesh import ArenaMesh, cmf_bytes
    from rlgpu.state import ARENA
    from tests_util import procedural_arena_mesh
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        mesh = ArenaMesh.from_cmf([cmf_bytes(v, t) for v, t in procedural_arena_mesh()])
    n = 48
    g, o = EnvSet(n, seed=9, device=gpu, mesh=mesh), oracle.EnvSet(n, seed=9, mesh=mesh, threads=4)
    _check(g, o, "create")
    rng = np.random.default_rng(4)
    for t in range(10):
        a = random_actions(o.masks, rng)
        o.step(a, True)
        g.step(torch.from_numpy(a).to(gpu), True)
        _check_step(g, o, f"mesh step {t}")
    st = np.frombuffer(o.get_arenas().tobytes(), ARENA).copy()
    for i in range(n):  # throw the ball at the ramps / back walls, launch cars
        d = rng.normal(size=3)
        d[2] = abs(d[2])
        st["ball"][i]["vel"] = (d / np.linalg.norm(d) * rng.uniform(40, 110)).astype(np.float32)
        for k in range(4):
            st["cars"][i]["body"]["vel"][k] = rng.uniform(-40, 40, 3).astype(np.float32) * [1, 1, 0.3]
    buf = np.frombuffer(st.tobytes(), np.uint8)
    o.set_arenas(buf)
    g.set_arenas(buf)
    for t in range(50):
        a = random_actions(o.masks, rng)
        o.step(a, True)
        g.step(torch.from_numpy(a).to(gpu), True)
        _check_step(g, o, f"mesh perturbed step {t}")


@pytest.mark.parametrize("pen_slots", [None, 0])
def test_env_procedural_soccar_mesh_parity(gpu, pen_slots, monkeypatch):
    """The bench's SOCCAR-sized workload mesh (rlgpu.mesh.procedural_soccar: 16 objects, 8,800
    triangles -- quarter pipes, rounded corners, goal boxes): cars driven and balls thrown into the
    curved transitions and goals, bit-exact vs the oracle's scan of every triangle.  The run goes through
    the penetration solver (counted by the env set's profile counters); pen_slots = 0 takes the deferred
    queries' restart path (no saved pair-GJK state) instead of the resume path."""
    import ctypes
    import torch
    from rlgpu import _lib
    from rlgpu.env import EnvSet
    from rlgpu.mesh import procedural_soccar
    from rlgpu.state import ARENA
    mesh = procedural_soccar()
    assert (mesh.num_objects, mesh.num_tris) == (16, 8800)
    n = 64
    if pen_slots is not None:
        monkeypatch.setenv("RLGPU_DEBUG_PEN_SAVE_SLOTS", str(pen_slots))
    g, o = EnvSet(n, seed=21, device=gpu, mesh=mesh), oracle.EnvSet(n, seed=21, mesh=mesh, threads=8)
    prof = torch.zeros(64 + 35 * (n // 4) + n, dtype=torch.int64, device=gpu)
    L = _lib.lib()
    L.rlgpu_envset_set_profile.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
    _lib.check(L.rlgpu_envset_set_profile(g._h, ctypes.c_void_p(prof.data_ptr()), prof.numel()), "set_profile")
    _check(g, o, "create")
    rng = np.random.default_rng(8)
    st = np.frombuffer(o.get_arenas().tobytes(), ARENA).copy()
    for i in range(n):  # aim every ball at a transition, corner or goal; send cars at the walls
        tgt = np.float32([rng.choice([-1, 1]) * rng.uniform(3000, 4096), rng.choice([-1, 1]) * rng.uniform(3500, 5900),
                          rng.uniform(0, 2000)]) / 50.0
        d = tgt - st["ball"][i]["pos"]
        st["ball"][i]["vel"] = (d / np.linalg.norm(d) * rng.uniform(50, 110)).astype(np.float32)
        for k in range(4):
            v = rng.normal(size=3) * [1, 1, 0.2]
            st["cars"][i]["body"]["vel"][k] = (v / np.linalg.norm(v) * rng.uniform(20, 46)).astype(np.float32)
    buf = np.frombuffer(st.tobytes(), np.uint8)
    o.set_arenas(buf)
    g.set_arenas(buf)
    for t in range(60):
        a = random_actions(o.masks, rng)
        o.step(a, True)
        g.step(torch.from_numpy(a).to(gpu), True)
        _check_step(g, o, f"procedural soccar step {t}")
    torch.cuda.synchronize()
    pen = int(prof[28])
    assert pen > 0 and int(prof[64 + 35 * (n // 4):].sum()) == pen, pen  # the penetration solver ran
    _lib.check(L.rlgpu_envset_set_profile(g._h, None, 0), "set_profile")


@pytest.mark.parametrize("n", [1, 6, 39])
def test_env_ragged_workgroup_parity(gpu, n):
    """Arena counts that leave the last workgroup partly empty (1 of 4, 2 of 4, 3 of 4 arenas): the
    workgroup-wide phases (the wheel rays' casts, the queued box-triangle queries, the deferred penetration
    queries) deal only over the valid arenas, on the procedural SOCCAR mesh with balls and cars thrown at
    its transitions, bit-exact for 80 steps."""
    import torch
    from rlgpu.env import EnvSet
    from rlgpu.mesh import procedural_soccar
    from rlgpu.state import ARENA
    mesh = procedural_soccar()
    g, o = EnvSet(n, seed=31 + n, device=gpu, mesh=mesh), oracle.EnvSet(n, seed=31 + n, mesh=mesh, threads=4)
    _check(g, o, "create")
    rng = np.random.default_rng(n)
    st = np.frombuffer(o.get_arenas().tobytes(), ARENA).copy()
    for i in range(n):
        tgt = np.float32([rng.choice([-1, 1]) * rng.uniform(3000, 4096), rng.choice([-1, 1]) * rng.uniform(3500, 5900),
                          rng.uniform(0, 2000)]) / 50.0
        d = tgt - st["ball"][i]["pos"]
        st["ball"][i]["vel"] = (d / np.linalg.norm(d) * rng.uniform(50, 110)).astype(np.float32)
        for k in range(4):
            v = rng.normal(size=3) * [1, 1, 0.2]
            st["cars"][i]["body"]["vel"][k] = (v / np.linalg.norm(v) * rng.uniform(20, 46)).astype(np.float32)
    buf = np.frombuffer(st.tobytes(), np.uint8)
    o.set_arenas(buf)
    g.set_arenas(buf)
    for t in range(80):
        a = random_actions(o.masks, rng)
        o.step(a, True)
        g.step(torch.from_numpy(a).to(gpu), True)
        _check_step(g, o, f"ragged n={n} step {t}")


def test_env_reset_arenas_mask(gpu):
    import torch
    n = 12
    g, o = _mk(n, 9, gpu)
    rng = np.random.default_rng(3)
    for t in range(5):
        a = random_actions(o.masks, rng)
        o.step(a, True)
        g.step(torch.from_numpy(a).to(gpu), True)
    m = (np.arange(n) % 3 == 0).astype(np.uint8)
    o.reset_arenas(m)
    g.reset_arenas(torch.from_numpy(m).to(gpu))
    _check(g, o, "reset_arenas")


def test_env_step_outputs_append(gpu):
    """rlgpu_envset_step's experience-append outputs equal the state buffers."""
    import torch
    from rlgpu.env import StepOutputs
    n = 8
    g, o = _mk(n, 4, gpu)
    obs_out = torch.empty((4 * n, 167), device=gpu)
    mask_out = torch.empty((4 * n, 90), dtype=torch.uint8, device=gpu)
    rew_out = torch.empty(4 * n, device=gpu)
    term_out = torch.empty(4 * n, dtype=torch.int8, device=gpu)
    a = torch.zeros(4 * n, dtype=torch.int32, device=gpu)
    g.step(a, True, StepOutputs.of(obs_out, mask_out, rew_out, term_out))
    torch.cuda.synchronize()
    assert torch.equal(obs_out, g.obs) and torch.equal(rew_out, g.rewards) and torch.equal(mask_out, g.action_masks)
    assert torch.equal(term_out.view(n, 4)[:, 0].to(torch.uint8), g.terminals)


def test_env_output_only_rows(gpu):
    """rlgpu_envset_set_output_only: the appended rows (obs, masks, rewards, codes, truncation obs) equal a normal
    set's bit for bit through truncations (max episode length) and terminal resets (NoTouch after 8 s), and the
    set's own obs / masks / trunc buffers keep the values they had before the steps (the C++ Learner's single
    copy per env step)."""
    import torch
    from rlgpu.env import EnvSet, StepOutputs

    def bufs(n):
        return (torch.empty((4 * n, 167), device=gpu), torch.empty((4 * n, 90), dtype=torch.uint8, device=gpu),
                torch.empty(4 * n, device=gpu), torch.empty(4 * n, dtype=torch.int8, device=gpu),
                torch.zeros((4 * n, 167), device=gpu))
    rng = np.random.default_rng(2)
    saw = {1: 0, 2: 0}
    for n, L, steps in ((24, 29, 90), (64, 0, 160)):  # truncations; then episodes ended by NoTouch (120 steps)
        A = EnvSet(n, seed=9, device=gpu, max_episode_steps=L)
        B = EnvSet(n, seed=9, device=gpu, max_episode_steps=L)
        B.set_output_only(True)
        obs0, masks0, trunc0 = B.obs.clone(), B.action_masks.clone(), B.trunc_obs.clone()
        for t in range(steps):
            a = torch.from_numpy(random_actions(A.action_masks.cpu().numpy(), rng)).to(gpu)
            oa, ob = bufs(n), bufs(n)
            A.step(a, True, StepOutputs.of(*oa))
            B.step(a, True, StepOutputs.of(*ob))
            torch.cuda.synchronize()
            for x, y in zip(oa, ob):
                assert torch.equal(x.view(torch.uint8) if x.dtype != torch.uint8 else x,
                                   y.view(torch.uint8) if y.dtype != torch.uint8 else y), f"step {t}"
            assert torch.equal(A.rewards, B.rewards) and torch.equal(A.terminals, B.terminals)
            for c in (1, 2):
                saw[c] += int((oa[3] == c).sum())
        assert torch.equal(B.obs, obs0) and torch.equal(B.action_masks, masks0) and torch.equal(B.trunc_obs, trunc0)
        # a step without rows still writes the set's buffers
        a = torch.zeros(4 * n, dtype=torch.int32, device=gpu)
        A.step(a, True)
        B.step(a, True)
        torch.cuda.synchronize()
        assert torch.equal(A.obs, B.obs) and torch.equal(A.action_masks, B.action_masks)
    assert saw[1] > 0 and saw[2] > 0, saw


def test_env_max_episode_truncation_parity(gpu):
    """Learner maxEpisodeLength (Learner.cpp:848-850): trajectories cut TRUNCATED without an arena
    reset; codes and trunc obs rows bit-exact vs the oracle."""
    import torch
    from rlgpu.env import EnvSet, StepOutputs
    n, L = 24, 37
    g = EnvSet(n, seed=8, device=gpu, max_episode_steps=L)
    o = oracle.EnvSet(n, seed=8, max_episode_steps=L)
    rng = np.random.default_rng(5)
    term_out = torch.empty(4 * n, dtype=torch.int8, device=gpu)
    trunc = torch.zeros((4 * n, 167), device=gpu)
    saw = 0
    for t in range(130):
        a = random_actions(o.masks, rng)
        o.step(a, True)
        g.step(torch.from_numpy(a).to(gpu), True, StepOutputs.of(terminals=term_out, trunc_obs=trunc))
        _check_step(g, o, f"step {t}")
        np.testing.assert_array_equal(term_out.cpu().numpy(), o.traj_terms, err_msg=f"traj terms step {t}")
        saw += int((o.traj_terms == 2).sum())
        sel = o.traj_terms == 2
        if sel.any():
            np.testing.assert_array_equal(trunc.cpu().numpy()[sel], o.trunc_obs[sel])
    assert saw > 0


def test_env_full_size_invariants(gpu):
    """BASELINE config C2 size (4096 arenas): finite obs, >=1 legal action per player,
    terminal codes in {0,1,2}, deterministic across two identical sets."""
    import torch
    n = 4096
    from rlgpu.env import EnvSet
    g1 = EnvSet(n, seed=77, device=gpu)
    g2 = EnvSet(n, seed=77, device=gpu)
    gen = torch.Generator(device=gpu).manual_seed(0)
    for t in range(24):
        u = torch.rand((4 * n, 90), device=gpu, generator=gen) * g1.action_masks.float()
        a = u.argmax(1).to(torch.int32)
        g1.step(a, True)
        g2.step(a, True)
    torch.cuda.synchronize()
    assert torch.isfinite(g1.obs).all()
    assert (g1.action_masks.sum(1) > 0).all()
    assert int(g1.terminals.max()) <= 2
    assert torch.equal(g1.obs, g2.obs) and torch.equal(g1.rewards, g2.rewards)
    assert np.array_equal(g1.get_arenas(), g2.get_arenas()) or not arena_diff(_state(g1), _state(g2))


def test_env_rejects_host_actions(gpu):
    import torch
    from rlgpu import RLGPUError
    from rlgpu.env import EnvSet
    g = EnvSet(2, device=gpu)
    with pytest.raises(RLGPUError):
        g.step(torch.zeros(8, dtype=torch.int32), True)
