# Full GPU check: every -m gpu test, smoke(), bench (with CPU baseline), rocprofv3 kernel stats (CSV).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profcsv -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/profcsv.log 2>&1
