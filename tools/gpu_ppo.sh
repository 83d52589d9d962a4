# PPO GPU tests only (GEMM arithmetic / minibatch parity).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ppo.py -m gpu -x -v --timeout 120 --timeout-method thread -k "h3 or gemm or forward" > gpurun_out/t_ppo.log 2>&1
