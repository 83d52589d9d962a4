"""Per-iteration summary of a rocprofv3 --stats kernel CSV (bench: warmup + steps iterations)."""
import csv
import sys

path = sys.argv[1]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
rows = list(csv.DictReader(open(path)))
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs']) / iters / 1e6:8.2f} ms/it {float(r['Percentage']):5.1f}% "
          f"n={int(r['Calls']) // iters:5d}/it avg={float(r['AverageNs']) / 1e3:8.1f}us {r['Name'][:80]}")
