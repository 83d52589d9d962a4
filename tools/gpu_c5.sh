export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ppo.py tests/test_learner_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_c5.log 2>&1
