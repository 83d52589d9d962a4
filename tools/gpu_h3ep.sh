# H3 epilogue change: parity tests, kernel times, bench
export TMPDIR=/tmp
mkdir -p gpurun_out/h3e
timeout -k 10 400 python -u -m pytest tests/test_ppo.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/h3e/t_ppo.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/h3e/k -o run -- python tools/gemm_bench.py 2 > gpurun_out/h3e/k.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/h3e/bench.log 2>&1
