"""Car hitbox vs car hitbox: btBoxBoxDetector / ODE dBoxBox2 as RocketSim runs it (btBoxBoxCollisionAlgorithm
.cpp:44-71 -> btBoxBoxDetector.cpp:267-767).

CPU: the oracle restatement (oracle/boxbox_ref.hpp) against known answers -- separated boxes give no point
(dBoxBox2 reports overlap only, no breaking-threshold margin), two aligned boxes overlapping face to face
give 4 points at the analytic depth with the face normal, a tilted box resting on another's face gives
its penetrating corners, crossed edges give one edge-edge point.  Parity unpinned beyond these (the
reference cannot be built here).
GPU: the device restatement (csrc/boxbox.hpp, rlgpu_box_box_queries) bit for bit against the oracle on
20,000 seeded overlapping poses (face-face with culling to 4, face-edge, edge-edge).
"""
import numpy as np
import pytest

import oracle
from test_gjk import _canon, _rand_rot


def _q(Ra, ca, Rb, cb):
    return oracle.box_box(np.asarray(Ra, np.float32)[None], np.asarray(ca, np.float32)[None],
                          np.asarray(Rb, np.float32)[None], np.asarray(cb, np.float32)[None])[0]


def test_separated_gives_nothing():
    impl, margin, half = oracle.car_box_shape()
    I = np.eye(3, dtype=np.float32)
    out = _q(I, [0, 0, 0], I, [2 * half[0] + 0.001, 0, 0])
    assert out[0] == 0
    out = _q(I, [0, 0, 0], I, [2 * half[0] + 0.01, 0.3, 0])  # within Bullet's 0.02 threshold: still none
    assert out[0] == 0


def test_face_face_overlap_four_points():
    impl, margin, half = oracle.car_box_shape()
    I = np.eye(3, dtype=np.float32)
    d = 0.05
    out = _q(I, [0, 0, 0], I, [0, 0, 2 * half[2] - d])  # B on top of A, overlapping by d
    assert out[0] == 4
    pts = out[1:].reshape(4, 7)
    assert np.allclose(pts[:, 6], -d, atol=2e-6)
    assert np.allclose(np.abs(pts[:, 2]), 1) and np.all(pts[:, :2] == 0)
    # normal on B (the upper box) points from B to A: -z
    assert np.all(pts[:, 2] == -1)


def test_tilted_box_corner_points_and_culling():
    rng = np.random.default_rng(1)
    impl, margin, half = oracle.car_box_shape()
    I = np.eye(3, dtype=np.float32)
    c, s_ = np.cos(0.3), np.sin(0.3)
    Rb = np.array([[c, -s_, 0], [s_, c, 0], [0, 0, 1]], np.float32)  # yawed, lying flat on A
    out = _q(I, [0, 0, 0], Rb, [0.2, 0.1, 2 * half[2] - 0.02])
    assert out[0] == 4  # the clipped polygon has up to 8 points; culled to 4
    assert np.allclose(out[1:].reshape(4, 7)[:, 6], -0.02, atol=2e-6)


def test_edge_edge_single_point():
    impl, margin, half = oracle.car_box_shape()
    I = np.eye(3, dtype=np.float32)
    a = np.pi / 4
    # B rolled 45 deg about x and yawed 45 deg: its lower edge crosses A's top face diagonally
    Rx = np.array([[1, 0, 0], [0, np.cos(a), -np.sin(a)], [0, np.sin(a), np.cos(a)]])
    Rz = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    Ry = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    Rb = (Rz @ Rx @ Ry).astype(np.float32)
    found = False
    for z in np.linspace(0.5, 1.6, 60):
        out = _q(I, [0, 0, 0], Rb, [0.9, 0.6, z])
        if out[0] == 1:
            found = True
            assert out[7] < 0
            assert abs(np.linalg.norm(out[1:4]) - 1) < 1e-5
    assert found


def make_pairs(n, seed):
    rng = np.random.default_rng(seed)
    impl, margin, half = oracle.car_box_shape()
    Ra, Rb = _rand_rot(rng, n), _rand_rot(rng, n)
    flat = rng.random(n) < 0.35  # cars on the ground: yaw-only rotations (face-face, culling)
    yaw = rng.uniform(-np.pi, np.pi, (2, n))
    for R, y in ((Ra, yaw[0]), (Rb, yaw[1])):
        c, s = np.cos(y[flat]), np.sin(y[flat])
        R[flat] = 0
        R[flat, 0, 0], R[flat, 0, 1], R[flat, 1, 0], R[flat, 1, 1], R[flat, 2, 2] = c, -s, s, c, 1
    ca = rng.uniform(-5, 5, (n, 3)).astype(np.float32)
    d = rng.standard_normal((n, 3))
    d[flat, 2] *= 0.2
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    cb = (ca + d * rng.uniform(0.2, 2.2, (n, 1))).astype(np.float32)
    return Ra, ca, Rb, cb


def test_oracle_pairs_cover_all_codes():
    out = oracle.box_box(*make_pairs(6000, 3))
    cnt = out[:, 0]
    assert (cnt == 0).sum() > 200 and (cnt == 1).sum() > 200 and (cnt == 4).sum() > 200 and ((cnt == 2) | (cnt == 3)).sum() > 50


@pytest.mark.gpu
def test_device_box_box_bit_exact(gpu):
    import torch
    from rlgpu.mesh import box_box_queries
    args = make_pairs(20000, 11)
    want = oracle.box_box(*args)
    got = box_box_queries(*[torch.from_numpy(a).to(gpu) for a in args]).cpu().numpy()
    bad = np.nonzero(np.any(_canon(got) != _canon(want), axis=1))[0]
    assert (want[:, 0] > 0).sum() > 5000
    assert len(bad) == 0, f"{len(bad)} of {len(want)} differ; first {bad[:5]}: got {got[bad[:1]]} want {want[bad[:1]]}"
