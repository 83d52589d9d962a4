# Iteration loop on the GPU box: PPO/learner GPU tests, bench, rocprofv3 kernel stats (CSV).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ppo.py tests/test_learner_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_ppo.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profcsv -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/profcsv.log 2>&1
