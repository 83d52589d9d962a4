# grouped collection: bench.py with and without the per-launch timing events, groups 1 / 2 / 4
export TMPDIR=/tmp
O=gpurun_out/${TAG:-groups2}
mkdir -p $O
for tm in 0 1; do
for g in 1 2 4; do
  RLGPU_BENCH_ENV_TIMING=$tm RLGPU_BENCH_COLLECT_GROUPS=$g timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > $O/bench_${tm}_$g.json 2> $O/bench_${tm}_$g.err || { tail -20 $O/bench_${tm}_$g.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_${tm}_$g.json').read().strip().splitlines()[-1]); print('timing $tm groups $g', round(d['value']), round(d['ms_per_step'],1), round(d['phase_s_per_iteration']['collect']*1e3,1), d['roofline']['kernel_ms'])"
done
done
