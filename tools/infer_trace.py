"""Phase timestamps of the fused inference kernel (infer::mlp_infer) per workgroup.

python tools/infer_trace.py [rows] -- policy action sampling over `rows` rows (default 16384, the
C2 collection step) and the critic over 50000 rows; prints per-phase medians (us) across
workgroups, from wall_clock64 marks (100 MHz) written by thread 0 of each workgroup.
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "reinforcement-learning_amd"))
from rlgpu import _lib  # noqa: E402
from rlgpu.ppo import PPO  # noqa: E402

NAMES = {0: "start", 1: "obs staged", 2: "L0 mfma", 8: "L0 epilogue", 3: "L0 ln", 4: "L1 mfma", 9: "L1 epilogue",
         5: "L1 ln", 6: "L2 mfma", 10: "L2 epilogue", 12: "out start", 13: "out mfma", 14: "logits staged",
         15: "sampled", 7: "probs", 11: "picks"}
ORDER = [0, 1, 2, 8, 3, 4, 9, 5, 6, 10, 12, 13, 14, 7, 11, 15]


def report(tag, tr, nblk):
    t = tr[:nblk * 16].reshape(nblk, 16).astype(np.int64)
    t0 = t[:, 0].min()
    marks = [p for p in ORDER if (t[:, p] > 0).all()]
    print(f"{tag}: {nblk} WGs, kernel span {(t[:, marks[-1]].max() - t0) / 100:.1f} us, "
          f"WG start spread {(t[:, 0].max() - t0) / 100:.1f} us")
    prev = marks[0]
    for p in marks[1:]:
        d = (t[:, p] - t[:, prev]) / 100.0
        print(f"  {NAMES.get(prev, prev):>18} -> {NAMES.get(p, p):<18} median {np.median(d):7.2f} us  max {d.max():7.2f}")
        prev = p
    tot = (t[:, marks[-1]] - t[:, 0]) / 100.0
    print(f"  per-WG total median {np.median(tot):.2f} us, max {tot.max():.2f}")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    lib = _lib.lib()
    lib.rlgpu_debug_infer_trace.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    p = PPO(max_rows=50_000, seed=1)
    g = torch.Generator().manual_seed(0)
    obs = torch.randn(max(n, 50_000), 167, generator=g).cuda()
    masks = (torch.rand(n, 90, generator=g) < 0.6).to(torch.uint8).cuda()
    masks[:, 0] = 1
    tr = torch.zeros(800 * 16, dtype=torch.int64, device="cuda")
    for _ in range(5):
        p.infer_actions(obs[:n], masks)
        p.infer_critic(obs[:50_000])
    torch.cuda.synchronize()
    for tag, fn, rows in (("policy sample", lambda: p.infer_actions(obs[:n], masks), n),
                          ("critic values", lambda: p.infer_critic(obs[:50_000]), 50_000)):
        tr.zero_()
        lib.rlgpu_debug_infer_trace(ctypes.c_void_p(tr.data_ptr()), tr.numel())
        fn()
        torch.cuda.synchronize()
        lib.rlgpu_debug_infer_trace(None, 0)
        report(tag, tr.cpu().numpy(), (rows + 63) // 64)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(20):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        print(f"  {tag}: {ev[0].elapsed_time(ev[1]) / 20 * 1000:.1f} us per call (untraced)")


if __name__ == "__main__":
    main()
