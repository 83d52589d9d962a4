"""Car hitbox vs mesh triangle narrowphase: Bullet's GJK / EPA query as RocketSim runs it
(btConvexConcaveCollisionAlgorithm.cpp:71-138 -> btConvexConvexAlgorithm.cpp:268-513 ->
btGjkPairDetector.cpp:686-959 with btVoronoiSimplexSolver and btGjkEpaPenetrationDepthSolver / btGjkEpa2).

CPU: the oracle restatement (oracle/gjk_ref.hpp) against known answers -- the Octane btBoxShape after
setSafeMargin, a box resting on / sunk into a large triangle (depth = analytic signed distance, normal =
the face normal to f32 GJK accuracy), separation beyond the threshold, the early out, and that the
penetration solver (EPA) takes over exactly where btGjkPairDetector's degenerate catch says (core distance
below 0.01).  Parity unpinned beyond these: the reference cannot be built here.
GPU: the device restatement (csrc/gjk.hpp, rlgpu_box_triangle_queries) bit for bit against the oracle
on 20,000 seeded poses spanning separated, touching, shallow and deep (EPA) contacts on faces, edges
and vertices of small and large triangles, for each work-set policy (HBM, LDS first, and the env kernel's
deferred queries run by the whole wavefront with the polytope in its registers, gjk.hpp epa_wave).
"""
import numpy as np
import pytest

import oracle


def _rand_rot(rng, n):
    q = rng.standard_normal((n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    x, y, z, w = q.T
    R = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                  2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                  2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], 1)
    return R.reshape(n, 3, 3).astype(np.float32)


def make_cases(n, seed=0):
    """Seeded box / triangle poses: triangle sizes 0.05-20 bt units, box placed against a point on the
    triangle (inside, or out past an edge / vertex) at signed gaps -0.6..+0.15 along the face normal."""
    rng = np.random.default_rng(seed)
    impl, margin, half = oracle.car_box_shape()
    R = _rand_rot(rng, n)
    # a fraction of boxes axis-aligned (cars on flat ground / walls hit the simplex corner cases)
    flat = rng.random(n) < 0.2
    R[flat] = np.eye(3, dtype=np.float32)
    size = np.exp(rng.uniform(np.log(0.05), np.log(20.0), n)).astype(np.float32)
    tri = (rng.standard_normal((n, 3, 3)) * size[:, None, None]).astype(np.float32)
    base = rng.uniform(-30, 30, (n, 1, 3)).astype(np.float32)
    tri = tri + base
    nrm = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    bary = rng.dirichlet([1, 1, 1], n)
    out = rng.random(n) < 0.3  # past an edge or vertex
    bary[out] = bary[out] * rng.uniform(1.0, 1.6, (out.sum(), 1)) - rng.uniform(0, 0.4, (out.sum(), 3))
    p = np.einsum("nk,nkj->nj", bary, tri)
    ext = np.abs(np.einsum("nij,ni->nj", R, nrm)) @ half  # box extent along the normal (R rows -> R^T n)
    gap = rng.uniform(-0.6, 0.15, n)
    side = np.where(rng.random(n) < 0.5, 1.0, -1.0)
    centre = (p + nrm * side[:, None] * (ext + gap)[:, None]).astype(np.float32)
    cbt = np.full(n, 0.02 * 50 / 50, np.float32)  # the car's contact breaking threshold scale (bullet units)
    return R, centre, tri, cbt


def test_car_box_shape_safe_margin():
    impl, margin, half = oracle.car_box_shape()
    hs = np.float32(np.array([120.507, 86.6994, 38.6591], np.float32) * np.float32(1 / 50)) / np.float32(2)
    # setSafeMargin: 0.1 x the smallest half extent (z) is below CONVEX_DISTANCE_MARGIN 0.04
    assert margin == np.float32(np.float32(0.1) * hs[2]) and margin < 0.04
    assert np.allclose(half, hs, rtol=0, atol=2e-7)
    assert np.all(impl < half) and np.allclose(half - impl, margin, atol=1e-7)


def _flat_case(h, R=None, cbt=0.02):
    tri = np.array([[[-50, -50, 0], [50, -50, 0], [0, 60, 0]]], np.float32)
    R = np.eye(3, dtype=np.float32)[None] if R is None else R[None].astype(np.float32)
    return oracle.box_triangle(R, np.array([[0.1, 0.2, h]], np.float32), tri, np.array([cbt], np.float32))


def test_resting_and_sunk_box_known_depth():
    impl, margin, half = oracle.car_box_shape()
    for gap, epa in [(0.01, False), (0.001, False), (-0.01, False), (-0.03, True), (-0.1, True), (-0.3, True)]:
        out, counts = _flat_case(half[2] + gap)
        assert out[0, 0] == 1.0
        assert abs(out[0, 7] - gap) < 2e-6, (gap, out[0])
        assert np.allclose(out[0, 1:4], [0, 0, 1], atol=5e-4)  # f32 GJK direction
        assert abs(out[0, 6]) < 1e-6  # the point lies on the triangle (body B)
        # btGjkPairDetector.cpp:847-851: the penetration solver runs when the core (margin-free)
        # distance falls below 0.01
        assert bool(counts[1]) == epa, (gap, counts)


def test_separated_and_early_out():
    impl, margin, half = oracle.car_box_shape()
    out, counts = _flat_case(half[2] + 0.03)  # beyond the 0.02 threshold: the normal early out
    assert out[0, 0] == 0 and counts[0] == 0
    out, counts = _flat_case(half[2] + 0.015)  # inside the threshold: a point with positive depth
    assert out[0, 0] == 1 and abs(out[0, 7] - 0.015) < 2e-6
    out, counts = _flat_case(-(half[2] - 0.01))  # box below the triangle, 0.01 into it from the back
    assert out[0, 0] == 1 and out[0, 3] < -0.999 and abs(out[0, 7] + 0.01) < 2e-6


def test_oracle_cases_cover_all_regimes():
    R, c, t, cbt = make_cases(4000, seed=1)
    out, counts = oracle.box_triangle(R, c, t, cbt)
    hit = out[:, 0] == 1
    assert 0.3 < hit.mean() < 0.95
    d = out[hit, 7]
    assert (d < -0.1).sum() > 50 and ((d > -0.02) & (d < 0.02)).sum() > 50
    assert counts[1] > 200  # penetration solver (EPA) exercised
    assert np.all(np.abs(np.linalg.norm(out[hit, 1:4], axis=1) - 1) < 1e-5)


def _canon(a):
    a = np.ascontiguousarray(a, np.float32).copy()
    a[np.isnan(a)] = np.nan  # one NaN pattern on both sides
    return a.view(np.uint32)


@pytest.mark.gpu
def test_device_box_triangle_bit_exact(gpu):
    import torch
    from rlgpu.mesh import box_triangle_queries
    R, c, t, cbt = make_cases(20000, seed=7)
    want, counts = oracle.box_triangle(R, c, t, cbt)
    assert counts[1] > 1000
    args = [torch.from_numpy(a).to(gpu) for a in (R, c, t, cbt)]
    # full-capacity HBM sets; small LDS sets with the HBM rerun; the env kernel's deferred wave-mode EPA
    for lds_first in (False, True, "wave", "wave-overflow"):
        got = box_triangle_queries(*args, lds_first=lds_first).cpu().numpy()
        bad = np.nonzero(np.any(_canon(got) != _canon(want), axis=1))[0]
        assert len(bad) == 0, f"lds_first={lds_first}: {len(bad)} of {len(R)} differ; first {bad[:5]}: " \
                              f"got {got[bad[:2]]} want {want[bad[:2]]}"
