"""GAE microbenchmark on its own (bench.py's gae_micro inputs): HIP events around rlgpu_gae_flat /
rlgpu_gae_rollout calls at M = 2^lg; run under rocprofv3 --kernel-trace --stats for the per-kernel split.

usage: python tools/gae_bench.py [lg=24] [reps=50]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reinforcement-learning_amd")]
from bench import gae_inputs  # noqa: E402
from rlgpu.gae import GAE  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 24
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda:0")
r, t, v, tv = gae_inputs(lg)
dr, dv, dt = (torch.from_numpy(x).to(dev) for x in (r, v, t))
dtv = torch.from_numpy(tv).to(dev)
T = 128
N = r.size // T
boot = torch.zeros(N, device=dev)
trv = torch.zeros(r.size, device=dev)
outs = [torch.empty(r.size, device=dev) for _ in range(3)]
for name, call in (("flat", lambda: GAE.compute(dr, dt, dv, dtv, 0.99, 0.95, 1.7, 200.0)),
                   ("rollout", lambda: GAE.compute_rollout(dr.view(T, N), dt.view(T, N), dv.view(T, N), trv.view(T, N),
                                                           boot, 0.99, 0.95, 1.7, 200.0))):
    call()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    for i in range(reps):
        ev[2 * i].record()
        call()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    ms = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps))
    med = ms[len(ms) // 2]
    print(f"{name} M=2^{lg}: median {med * 1e3:.1f} us, {21 * r.size / med / 1e6:.0f} GB/s algorithmic")
