import numpy as np


def synth_gae(m, seed, p_normal=1 / 128, p_trunc=1 / 512):
    """SURVEY.md 8(d) GAE microbenchmark distribution (r, V ~ N(0,1); NORMAL 1/128; TRUNC 1/512)."""
    rng = np.random.default_rng(seed)
    rews = rng.standard_normal(m).astype(np.float32)
    vals = rng.standard_normal(m).astype(np.float32)
    u = rng.random(m)
    terms = np.zeros(m, np.int8)
    terms[u < p_normal] = 1
    terms[(u >= p_normal) & (u < p_normal + p_trunc)] = 2
    nt = int((terms == 2).sum())
    tv = rng.standard_normal(nt).astype(np.float32)
    return rews, terms, vals, tv


def arena_diff(a, b, limit=20):
    """Field-by-field bit comparison of two structured ARENA arrays (rlgpu.state.ARENA).

    Returns a list of "arena i: path (max |diff|)" strings, empty when bit-identical.
    Floats are compared by bit pattern (NaN-safe, -0 != +0)."""
    out = []

    def walk(x, y, path):
        if x.dtype.names:
            for n in x.dtype.names:
                walk(x[n], y[n], path + "." + n)
            return
        xa, ya = np.ascontiguousarray(x), np.ascontiguousarray(y)
        if xa.dtype.kind == "f":
            bad = xa.view(np.uint32) != ya.view(np.uint32)
        else:
            bad = xa != ya
        if bad.ndim > 1:
            bad_arena = bad.reshape(bad.shape[0], -1).any(axis=1)
        else:
            bad_arena = bad
        for i in np.nonzero(bad_arena)[0][:limit]:
            xi, yi = np.asarray(xa[i], np.float64), np.asarray(ya[i], np.float64)
            with np.errstate(invalid="ignore"):
                d = np.nanmax(np.abs(xi - yi)) if xi.size else 0.0
            out.append(f"arena {i}: {path[1:]} max|diff|={d:.3g} got={np.ravel(xi)[:6]} want={np.ravel(yi)[:6]}")

    walk(a, b, "")
    return out[:limit] if limit else out


def random_actions(masks, rng):
    """One valid DefaultAction index per player, uniform over the mask (masks [P, 90] uint8)."""
    m = np.asarray(masks, bool)
    u = rng.random(m.shape) * m
    return np.argmax(u, axis=1).astype(np.int32)


def procedural_arena_mesh(nx=36, ny=48, seed=0):
    """A dense multi-object collision mesh for parity tests (bullet units), in place of the absent
    SOCCAR .cmf files: a bumpy heightfield over the floor (z 0..16 uu) split into 4 quadrant objects,
    plus 45-degree ramps along both side walls (2 objects) and a back-wall panel pair per goal end
    (2 objects).  Returns (vertices [V, 3], triangles [T, 3]) per object as a list, ready for
    rlgpu.mesh.cmf_bytes."""
    rng = np.random.default_rng(seed)
    s = 1.0 / 50.0
    objs = []
    xs = np.linspace(-3800, 3800, nx + 1)
    ys = np.linspace(-4900, 4900, ny + 1)
    ph = rng.random(2) * 6.0
    hx, hy = nx // 2, ny // 2
    for qx, qy in ((0, 0), (1, 0), (0, 1), (1, 1)):
        ix = np.arange(qx * hx, (qx + 1) * hx + 1 if qx else hx + 1)
        iy = np.arange(qy * hy, (qy + 1) * hy + 1 if qy else hy + 1)
        X, Y = np.meshgrid(xs[ix], ys[iy], indexing="ij")
        Z = 8 + 8 * np.sin(X / 300 + ph[0]) * np.cos(Y / 410 + ph[1])
        V = np.stack([X, Y, Z], -1).reshape(-1, 3) * s
        W = len(iy)
        T = []
        for a in range(len(ix) - 1):
            for b in range(W - 1):
                p00, p01, p10, p11 = a * W + b, a * W + b + 1, (a + 1) * W + b, (a + 1) * W + b + 1
                T += [(p00, p10, p11), (p00, p11, p01)]
        objs.append((V.astype(np.float32), np.array(T, np.int32)))
    for side in (-1, 1):  # side-wall ramps: from (x = side*3700, z=0) up to (x = side*4096, z=396)
        V, T = [], []
        for k, y in enumerate(np.linspace(-4800, 4800, 17)):
            V += [(side * 3700, y, 0), (side * 4096, y, 396)]
            if k:
                i = 2 * k
                T += [(i - 2, i, i + 1), (i - 2, i + 1, i - 1)] if side > 0 else [(i - 2, i + 1, i), (i - 2, i - 1, i + 1)]
        objs.append((np.array(V, np.float32) * s, np.array(T, np.int32)))
    for end in (-1, 1):  # back walls with a goal mouth (x in [-893, 893], z < 643)
        V = np.array([(-4096, end * 5120, 0), (-893, end * 5120, 0), (-893, end * 5120, 2044), (-4096, end * 5120, 2044),
                      (893, end * 5120, 0), (4096, end * 5120, 0), (4096, end * 5120, 2044), (893, end * 5120, 2044),
                      (-893, end * 5120, 643), (893, end * 5120, 643)], np.float32) * s
        T = np.array([(0, 1, 2), (0, 2, 3), (4, 5, 6), (4, 6, 7), (8, 9, 7), (8, 7, 2)], np.int32)
        objs.append((V, T))
    return objs


def mesh_from_objects(objs):
    """(tris [N, 9], object_ntris [K]) of a list of (vertices, triangles)."""
    tris = [v[t].reshape(-1, 9) for v, t in objs]
    return np.concatenate(tris).astype(np.float32), np.array([len(t) for t in tris], np.int32)
