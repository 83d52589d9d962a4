"""Per-kernel mean of every counter in the rocprofv3 --pmc passes under a directory (p*/run_counter_collection.csv)."""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for path in sorted(glob.glob(f"{sys.argv[1]}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0][:48] + f" g{r['Grid_Size']}"
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in sorted(acc.items()):
    print(name)
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
