"""Timeline analysis of a rocprofv3 kernel trace (run_kernel_trace.csv) of bench.py: splits the last
PPO iteration into phases (collect = env_kernel span, learn = after the last gae kernel) and reports,
for the learn phase, wall time, GPU-busy time (union over streams), per-stream busy time and the
kernel classes on it."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]) for r in rows]
ks.sort()
gae = [k for k in ks if "gae_rollout" in k[2]]
last_gae_end = gae[-1][1]
learn = [k for k in ks if k[0] >= last_gae_end and "trampoline" not in k[2] or (k[0] >= last_gae_end)]
learn = [k for k in ks if k[0] >= last_gae_end]
t0, t1 = learn[0][0], max(k[1] for k in learn)
print(f"learn wall {(t1 - t0) / 1e6:.2f} ms, kernels {len(learn)}")
# union busy
busy, cur_s, cur_e = 0, None, None
for s, e, _, _ in learn:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"GPU busy (union) {busy / 1e6:.2f} ms")
by_stream = defaultdict(int)
by_name = defaultdict(lambda: [0, 0])
for s, e, n, st in learn:
    by_stream[st] += e - s
    key = n.split("(")[0][:60]
    by_name[key][0] += e - s
    by_name[key][1] += 1
for st, v in by_stream.items():
    print(f"stream {st}: kernel time {v / 1e6:.2f} ms")
for n, (v, c) in sorted(by_name.items(), key=lambda x: -x[1][0])[:20]:
    print(f"  {n:60s} {c:5d} {v / 1e6:8.2f} ms")
