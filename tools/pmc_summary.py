"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (run separately, as
MI355X_MICROARCH.md prescribes) into per-launch HBM bytes for one kernel.

usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <kernel substring> <min grid threads> <out.json> [mesh]
                                  [kernel_stats.csv] [round tag]

The optional kernel-stats CSV (rocprofv3 --kernel-trace --stats of the same bench command) adds the kernel's
average duration (kernel_us_rocprof), so bench.py can report the traffic at the profiler's own kernel time.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide
coalesced streaming reads -> doubled; WRITE_SIZE is taken as is.  Both counters are in KB.
"""
import csv
import json
import sys


def per_launch(path, kernel, min_grid):
    """Mean counter value per launch over the kernel's launches of its most frequent grid size (>= min_grid):
    the collection's step launches (one per arena group and env step), not the set-up launches."""
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"] and int(r["Grid_Size"]) >= min_grid]
    grids = {}
    for r in rows:
        grids[int(r["Grid_Size"])] = grids.get(int(r["Grid_Size"]), 0) + 1
    grid = max(grids, key=grids.get) if grids else 0
    v = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) == grid]
    return len(v), sum(v) / max(len(v), 1), grid


def main():
    fdir, wdir, kernel, min_grid, out = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5]
    mesh = sys.argv[6] if len(sys.argv) > 6 else "synthetic"
    stats = sys.argv[7] if len(sys.argv) > 7 else None
    tag = sys.argv[8] if len(sys.argv) > 8 else None
    nf, fetch_kb, gf = per_launch(f"{fdir}/run_counter_collection.csv", kernel, min_grid)
    nw, write_kb, gw = per_launch(f"{wdir}/run_counter_collection.csv", kernel, min_grid)
    assert gf == gw, (gf, gw)
    res = {"kernel": kernel, "launches": [nf, nw], "grid_threads": gf, "arenas_per_launch": gf // 64 * 4,
           "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
           "hbm_bytes_per_launch": (2 * fetch_kb + write_kb) * 1024,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read half count), WRITE_SIZE x1; KB = 1024 B", "mesh": mesh,
           "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE --output-format csv -- python3 bench.py --steps 1 "
                      f"--warmup 0 --no-cpu-baseline --mesh {mesh} (two separate passes)"}
    if stats:
        for r in csv.DictReader(open(stats)):
            if kernel in r["Name"]:
                res["kernel_us_rocprof"] = float(r["AverageNs"]) / 1e3
                res["kernel_stats_source"] = stats
                break
    if tag:
        res["round"] = tag
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
