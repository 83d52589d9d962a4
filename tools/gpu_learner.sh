# Learner / PPO GPU tests and a bench line (no CPU baseline).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_learner_gpu.py tests/test_ppo.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_learner.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
