"""Generates tests/golden/gae_*.npz from the CPU oracle (oracle/gae_ref.c).

The reference ships no GAE fixtures, so these vectors are produced
by the restatement itself; the restatement is pinned independently by the closed-form
cases in tests/test_gae.py.  Re-run: python tests/golden/make_gae_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402


def synth(m, seed, p_normal=1 / 128, p_trunc=1 / 512):
    # SURVEY.md 8(d) GAE microbenchmark distribution
    rng = np.random.default_rng(seed)
    rews = rng.standard_normal(m).astype(np.float32)
    vals = rng.standard_normal(m).astype(np.float32)
    u = rng.random(m)
    terms = np.zeros(m, np.int8)
    terms[u < p_normal] = 1
    terms[(u >= p_normal) & (u < p_normal + p_trunc)] = 2
    terms[-1] = 1
    nt = int((terms == 2).sum())
    tv = rng.standard_normal(nt).astype(np.float32)
    return rews, terms, vals, tv


def main():
    cases = [(4096, 7, 0.99, 0.95, 1.0, 0.0), (5000, 8, 0.99, 0.95, 2.5, 10.0), (3001, 9, 0.9, 0.8, 0.5, 1.0)]
    for i, (m, seed, g, l, std, clip) in enumerate(cases):
        rews, terms, vals, tv = synth(m, seed)
        adv, tgt, ret, cp, st = oracle.gae_flat(rews, terms, vals, tv, g, l, std, clip)
        assert st == 0
        np.savez_compressed(os.path.join(HERE, f"gae_flat_{i}.npz"), rews=rews, terms=terms, vals=vals,
                            trunc_vals=tv, params=np.array([g, l, std, clip], np.float32),
                            adv=adv, target=tgt, ret=ret, clip_portion=np.float32(cp))
    print("wrote", len(cases), "cases")


if __name__ == "__main__":
    main()
