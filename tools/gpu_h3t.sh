# H3 k-major wgrad staging: parity tests, kernel times, bench
export TMPDIR=/tmp
mkdir -p gpurun_out/h3t
timeout -k 10 400 python -u -m pytest tests/test_ppo.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/h3t/t_ppo.log 2>&1 || exit 1
for v in ${H3VARS:-0}; do
  RLGPU_H3_VARIANT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/h3t/k$v -o run -- python tools/gemm_bench.py 2 > gpurun_out/h3t/k$v.log 2>&1 || exit 1
  RLGPU_H3_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/h3t/bench$v.log 2>&1 || exit 1
done
