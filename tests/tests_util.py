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
