# grouped rollout collection: the learner / distributed / trainer tests, then bench.py with collect groups 1 and 4
export TMPDIR=/tmp
O=gpurun_out/${TAG:-groups}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_learner_gpu.py tests/test_dist_gpu.py tests/test_trainer_facade.py tests/test_configs_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for g in 1 4 1 4; do
  RLGPU_BENCH_COLLECT_GROUPS=$g timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-legs > $O/bench_$g.json 2> $O/bench_$g.err || { tail -20 $O/bench_$g.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$g.json').read().strip().splitlines()[-1]); print('groups $g', round(d['value']), d['ms_per_step'], d['phase_s_per_iteration']['collect'], d['roofline']['kernel_ms'], d['roofline']['units_per_launch'])"
done
