# env kernel built at different optimisation levels: env parity tests + late-game step time
export TMPDIR=/tmp
mkdir -p gpurun_out/envopt
for v in O3 O1 Os; do
  if [ $v = O3 ]; then L=""; else L=$PWD/reinforcement-learning_amd/rlgpu/librlgpu_env$v.so; fi
  RLGPU_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/envopt/t_$v.log 2>&1 || exit 1
  RLGPU_LIB=$L ENV_WARM=200 timeout -k 10 120 python tools/env_scale.py 4096 > gpurun_out/envopt/s_$v.log 2>&1 || exit 1
done
