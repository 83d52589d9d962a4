export TMPDIR=/tmp
mkdir -p gpurun_out/r03a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03a/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r03a/bench.log 2>&1
