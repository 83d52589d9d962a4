# x6 GEMM pipeline variants: parity tests per variant, GEMM microbench, bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1 2; do
  export RLGPU_X6_VARIANT=$v
  timeout -k 10 300 python -u -m pytest tests/test_ppo.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ppo_v$v.log 2>&1 || exit 1
  timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/gemm_v$v.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_v$v.log 2>&1 || exit 1
done
