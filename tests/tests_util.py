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
