# A/B of two library builds on one box: bench.py alternately with $RLGPU_LIB_A (A) and the in-tree
# library (B), a few rounds each, so box-to-box spread does not enter the comparison.
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for i in 1 2 3; do
  RLGPU_LIB=$RLGPU_LIB_A timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/ab/a$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/ab/b$i.log 2>&1 || exit 1
done
python - <<'PY'
import json
for ab in "ab":
    rows = [json.loads(open(f"gpurun_out/ab/{ab}{i}.log").read().strip().splitlines()[-1]) for i in (1, 2, 3)]
    print(ab, " ".join(f"{r['ms_per_step']:.1f}ms collect={r['phase_s_per_iteration']['collect']*1e3:.1f} learn={r['phase_s_per_iteration']['learn']*1e3:.1f} env={r['roofline']['kernel_ms']*1e3:.0f}us" for r in rows))
PY
