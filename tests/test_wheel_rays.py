"""Wheel rays against the ball and other cars: btCollisionWorld::rayTestSingleInternal's convex branch
(btCollisionWorld.cpp:277-310) -> btSubsimplexConvexCast::calcTimeOfImpact (btSubSimplexConvexCast.cpp:30-153)
of the ray's point shape against the ball's btSphereShape or a car compound's btBoxShape child.

CPU: the oracle's restatement (oracle/gjk_ref.hpp ray_convex_cast) against the closed-form ray / sphere and
ray / oriented-box intersections -- the same hits, fractions within the cast's convergence tolerance (it stops
once the simplex is within sqrt(1e-4) = 0.01 bullet units of the body), normals the face / radial direction.
GPU: the kernels' cast (csrc/gjk.hpp, rlgpu_linear_math_queries op 5) bit for bit against the oracle in every
arithmetic mode; whole-arena parity with cars parked on the ball and on each other is
tests/test_env_gpu.py::test_env_wheel_rays_on_dynamic_bodies_parity.
"""
import numpy as np
import pytest

import oracle

BALL_R = np.float32(91.25 * 0.02)
CAR_HALF = (np.array([120.507, 86.6994, 38.6591], np.float32) * np.float32(0.02)) * np.float32(0.5)


def _rot(rng, n):
    q = rng.standard_normal((n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    x, y, z, w = q.T
    R = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                  2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                  2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], 1)
    return R.astype(np.float32)


def _rays(n, seed, sphere):
    """Wheel-like rays (length 0.3-0.9) aimed near a body: hits, misses, grazing rays, rays starting inside."""
    rng = np.random.default_rng(seed)
    x = np.zeros((n, 24), np.float32)
    x[:, :9] = _rot(rng, n)
    o = rng.uniform(-40, 40, (n, 3)).astype(np.float32)
    x[:, 15:18] = o
    reach = BALL_R if sphere else np.float32(np.linalg.norm(CAR_HALF))
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    start_r = rng.uniform(0.3, 1.3, (n, 1)) * reach + rng.uniform(0.0, 0.6, (n, 1))
    frm = o + d * start_r
    aim = o + rng.uniform(-1.0, 1.0, (n, 3)) * reach * rng.choice([0.2, 0.8, 1.2], (n, 1))
    u = aim - frm
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    to = frm + u * rng.uniform(0.3, 0.9, (n, 1))
    x[:, 9:12] = frm
    x[:, 12:15] = to
    if sphere:
        x[:, 21] = BALL_R
    else:
        x[:, 18:21] = CAR_HALF
    return x


def _analytic(x, sphere):
    frm, to, o = x[:, 9:12].astype(np.float64), x[:, 12:15].astype(np.float64), x[:, 15:18].astype(np.float64)
    d = to - frm
    n = len(x)
    hit = np.zeros(n, bool)
    f = np.full(n, np.nan)
    nrm = np.zeros((n, 3))
    if sphere:
        oc = frm - o
        a = (d * d).sum(1)
        b = (oc * d).sum(1)
        c = (oc * oc).sum(1) - float(BALL_R) ** 2
        disc = b * b - a * c
        ok = (c > 0) & (disc >= 0) & (b < 0)
        t = (-b - np.sqrt(np.maximum(disc, 0))) / a
        hit = ok & (t >= 0) & (t <= 1)
        f = np.where(hit, t, np.nan)
        p = frm + d * np.nan_to_num(f)[:, None] - o
        nrm = p / np.maximum(np.linalg.norm(p, axis=1, keepdims=True), 1e-30)
        return hit, f, nrm
    R = x[:, :9].reshape(n, 3, 3).astype(np.float64)
    lo = np.einsum("nji,nj->ni", R, frm - o)
    ld = np.einsum("nji,nj->ni", R, d)
    h = CAR_HALF.astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        t1 = (-h - lo) / ld
        t2 = (h - lo) / ld
    tn = np.minimum(t1, t2)
    tf = np.maximum(t1, t2)
    tmin = tn.max(1)
    tmax = tf.min(1)
    inside = (np.abs(lo) <= h).all(1)
    hit = (tmin <= tmax) & (tmin >= 0) & (tmin <= 1) & ~inside
    f = np.where(hit, tmin, np.nan)
    ax = tn.argmax(1)
    sgn = -np.sign(ld[np.arange(n), ax])
    ln = np.zeros((n, 3))
    ln[np.arange(n), ax] = sgn
    nrm = np.einsum("nij,nj->ni", R, ln)
    return hit, f, nrm


@pytest.mark.parametrize("sphere", (True, False))
def test_oracle_convex_cast_agrees_with_closed_form(sphere):
    x = _rays(40000, 1 if sphere else 2, sphere)
    out = oracle.linear_math(5, 0, x)
    got_hit = out[:, 0] > 0
    hit, f, nrm = _analytic(x, sphere)
    # rays whose closed-form answer is clear: the signed distance to the body along the segment starts and
    # ends away from the surface and either stays clearly outside or goes clearly inside (the cast converges
    # to within 0.01 of the surface: grazing rays, and rays starting within that of it, are Bullet's call)
    frm, to, o = x[:, 9:12].astype(np.float64), x[:, 12:15].astype(np.float64), x[:, 15:18].astype(np.float64)
    d = to - frm
    L = np.linalg.norm(d, axis=1)
    R = x[:, :9].reshape(-1, 3, 3).astype(np.float64)
    t = np.linspace(0, 1, 257)
    pts = frm[:, None, :] + d[:, None, :] * t[None, :, None] - o[:, None, :]
    if sphere:
        sd = np.linalg.norm(pts, axis=2) - float(BALL_R)
    else:
        lp = np.einsum("nji,ntj->nti", R, pts)
        q = np.abs(lp) - CAR_HALF.astype(np.float64)
        sd = np.linalg.norm(np.maximum(q, 0), axis=2) + np.minimum(q.max(2), 0)
    tol = 0.03
    clear = (sd[:, 0] > tol) & (np.abs(sd[:, -1]) > tol) & ((sd.min(1) < -tol) | (sd.min(1) > tol))
    # the ray test keeps a cast only below the closest fraction so far (1 for the first body,
    # btCollisionWorld.cpp:291): a "hit" past the ray's end is no hit
    got_hit &= out[:, 1] < 1.0
    agree = got_hit[clear] == hit[clear]
    assert agree.mean() > 0.995, f"hit / miss agree on {agree.mean():.4f} of {clear.sum()} clear rays"
    both = got_hit & hit & clear
    assert both.sum() > 1000
    # the cast stops once its point is within sqrt(1e-4) = 0.01 of the body: the reported point lies outside
    # the surface by at most that much, whatever the incidence angle
    hp = frm[both] + d[both] * out[both, 1:2].astype(np.float64) - o[both]
    if sphere:
        sdh = np.linalg.norm(hp, axis=1) - float(BALL_R)
    else:
        qh = np.abs(np.einsum("nji,nj->ni", R[both], hp)) - CAR_HALF.astype(np.float64)
        sdh = np.linalg.norm(np.maximum(qh, 0), axis=1) + np.minimum(qh.max(1), 0)
    assert sdh.min() > -2e-4 and sdh.max() < 0.0102, (sdh.min(), sdh.max())
    err = np.abs(out[both, 1] - f[both]) * L[both]
    cosn = (out[both, 2:5] * nrm[both]).sum(1)
    # the cast's normal is its last separating direction: radial on the sphere, the face normal on a box face,
    # a blend of the faces near a box edge or corner
    assert np.median(cosn) > 0.999 and (cosn > 0.99).mean() > (0.99 if sphere else 0.95), (np.median(cosn), (cosn > 0.99).mean())
    print(f"{'sphere' if sphere else 'box'}: {both.sum()} hits, hit point outside the surface by <= {sdh.max():.4g}, "
          f"distance along the ray to the exact hit p99 {np.percentile(err, 99):.4g} max {err.max():.4g}, "
          f"normal within 8 deg of the closed form's: {(cosn > 0.99).mean():.4f}")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", (0, 1, 2))
def test_device_convex_cast_equals_oracle(gpu, mode):
    import torch
    from rlgpu import arith
    for sphere in (True, False):
        x = _rays(20000, 10 + mode, sphere)
        want = oracle.linear_math(5, mode, x)[:, :5]
        got = arith.linear_math_queries(5, mode, torch.from_numpy(x).to(gpu)).cpu().numpy()[:, :5]
        bad = np.nonzero((got.view(np.uint32) != want.view(np.uint32)).any(axis=1))[0]
        assert bad.size == 0, f"mode {mode} sphere {sphere}: {bad.size} rows differ: {got[bad[:2]]} vs {want[bad[:2]]}"
        assert (want[:, 0] > 0).mean() > 0.1
