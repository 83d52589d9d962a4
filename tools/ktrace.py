"""Per (kernel, grid) average durations from a rocprofv3 kernel-trace CSV."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(list)
for r in rows:
    if pat not in r["Kernel_Name"]:
        continue
    key = (r["Kernel_Name"][:70], r.get("Grid_Size", r.get("Grid_Size_X", "?")))
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (k, g), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"n={len(v):4d} grid={g:>8s} median={v[len(v) // 2]:9.1f}us min={v[0]:9.1f}us  {k}")
