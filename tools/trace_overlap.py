"""Concurrency of env-kernel launches in a rocprofv3 kernel trace: for the env kernels, the queue each ran on,
their durations, and how much of their summed duration overlapped another env launch.

usage: python tools/trace_overlap.py <kernel_trace.csv>
"""
import csv
import sys
from collections import Counter

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "env_kernel" in r["Kernel_Name"]]
if rows:
    print("columns:", list(rows[0].keys()))
grid_key = next((k for k in (rows[0].keys() if rows else []) if k.startswith("Grid_Size")), None)
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", r.get("Stream_Id", "?")),
             int(r[grid_key]) if grid_key else 0) for r in rows)
print(len(iv), "env launches; queues:", Counter(q for _, _, q, _ in iv).most_common(), "grids:", Counter(g for *_, g in iv))
tot = sum(e - s for s, e, *_ in iv)
# time covered by at least one env launch vs summed durations
cover, cur_s, cur_e = 0, None, None
for s, e, *_ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            cover += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
cover += cur_e - cur_s
print(f"summed env-launch time {tot / 1e6:.2f} ms, covered {cover / 1e6:.2f} ms -> mean concurrency {tot / cover:.2f}")
other = [r for r in csv.DictReader(open(sys.argv[1])) if "mlp_infer" in r["Kernel_Name"]]
print(len(other), "inference launches, mean", sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in other) / max(1, len(other)) / 1e3, "us",
      "queues:", Counter(r.get("Queue_Id", "?") for r in other).most_common())
