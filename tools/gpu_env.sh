# Env iteration on the GPU box: env parity tests, per-phase profile, bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_mesh.py tests/test_learner_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_env.log 2>&1 && \
timeout -k 10 120 python tools/env_phase_profile.py 4096 32 > gpurun_out/env_phase.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
