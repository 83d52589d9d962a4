# H3 iteration: PPO parity tests, bench per H3 variant, kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ppo.py -m gpu -x -q --timeout 120 --timeout-method thread -k "h3 or gemm or forward" > gpurun_out/t_ppo.log 2>&1 && \
for v in 0 3; do RLGPU_H3_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_h3v$v.log 2>&1 || exit 1; done && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profcsv -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/profcsv.log 2>&1 && \
python tools/kstats.py gpurun_out/profcsv/run_kernel_stats.csv 4 30 > gpurun_out/kstats.txt
