"""Device box-triangle query cost (rlgpu_box_triangle_queries): kernel time per launch for query sets that
stay in GJK vs sets that all need the penetration solver (EPA), at a few lane counts."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning_amd"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
from rlgpu.mesh import box_triangle_queries  # noqa: E402
from test_gjk import make_cases  # noqa: E402

dev = torch.device("cuda:0")
R, c, t, cbt = make_cases(40000, seed=3)
out, _ = oracle.box_triangle(R, c, t, cbt)
# classify each query by whether the oracle used the penetration solver
pen = np.zeros(len(R), bool)
for i in range(len(R)):
    _, cnt = oracle.box_triangle(R[i:i + 1], c[i:i + 1], t[i:i + 1], cbt[i:i + 1])
    pen[i] = cnt[1] > 0
sets = {"empty": np.zeros(0, int), "gjk-only": np.nonzero(~pen & (out[:, 0] == 1))[0], "penetration": np.nonzero(pen)[0],
        "no-hit": np.nonzero(out[:, 0] == 0)[0]}
for name, idx in sets.items():
    for n in (1, 16, 64, 1024):
        sel = np.resize(idx, n) if len(idx) else np.resize(np.nonzero(out[:, 0] == 0)[0], n)
        args = [torch.from_numpy(np.ascontiguousarray(a[sel])).to(dev) for a in (R, c, t, cbt)]
        for _ in range(3):
            box_triangle_queries(*args)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tm = {}
        for mode in (True, False, "wave"):
            box_triangle_queries(*args, lds_first=mode)
            torch.cuda.synchronize()
            e0.record()
            reps = 10
            for _ in range(reps):
                box_triangle_queries(*args, lds_first=mode)
            e1.record()
            torch.cuda.synchronize()
            tm[mode] = e0.elapsed_time(e1) / reps * 1e3
        print(f"{name:12s} n={n:5d}: {tm[True]:9.1f} us per launch LDS-first, {tm[False]:9.1f} us HBM only, "
              f"{tm['wave']:9.1f} us wave-mode EPA (incl. scratch alloc)", flush=True)
