"""MFMA utilisation of the training GEMMs from a rocprofv3 --pmc pass (tools/gpu_round.sh's mfma pass).

usage: python tools/mfma_summary.py <mfma dir> <kernel_stats.csv of the same round> <tag> [command line]

Per kernel: dispatches, the per-dispatch means of SQ_INSTS_VALU_MFMA_F16 / SQ_INSTS_VALU_MFMA_MOPS_F16 /
SQ_VALU_MFMA_BUSY_CYCLES (summed over the chip), the busy cycles per SIMD (/ 256 CUs x 4 SIMDs) and the busy
fraction against the kernel's average duration in the kernel trace at 2.4 GHz.
"""
import csv
import glob
import sys
from collections import defaultdict

CLOCK_HZ, SIMDS = 2.4e9, 256 * 4


def main():
    mdir, kstats, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    cmd = sys.argv[4] if len(sys.argv) > 4 else "python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-legs"
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(f"{mdir}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open(kstats))}
    print("# rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F16 SQ_BUSY_CYCLES "
          "SQ_WAVES GRBM_GUI_ACTIVE")
    print(f"#   --kernel-include-regex gemm -- {cmd}  ({tag}; counters summed over the chip)")
    print("# per-dispatch means.  MFMA busy per SIMD = SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs x 4 SIMDs), against the "
          "kernel's average")
    print(f"# duration in the same round's kernel trace ({kstats}) at 2.4 GHz")
    for name, cs in sorted(vals.items(), key=lambda kv: -len(kv[1].get("SQ_VALU_MFMA_BUSY_CYCLES", []))):
        busy = cs.get("SQ_VALU_MFMA_BUSY_CYCLES")
        if not busy:
            continue
        n = len(busy)
        mean = lambda k: sum(cs[k]) / len(cs[k]) if cs.get(k) else float("nan")  # noqa: E731
        b = mean("SQ_VALU_MFMA_BUSY_CYCLES")
        d = dur.get(name)
        frac = f"{b / SIMDS / (d * 1e-9 * CLOCK_HZ):.3f}" if d else "n/a (not in the trace)"
        dtxt = f"{d / 1e3:.1f} us" if d else "n/a"
        print(f"{name.split('(')[0]}: dispatches {n}, MFMA insts {mean('SQ_INSTS_VALU_MFMA_F16'):.4g}, "
              f"MFMA_MOPS_F16 {mean('SQ_INSTS_VALU_MFMA_MOPS_F16'):.4g}, MFMA busy {b:.4g} ({b / SIMDS:.0f} per SIMD), "
              f"avg duration {dtxt}, MFMA busy fraction {frac}")


if __name__ == "__main__":
    main()
