# GPU test run: every -m gpu test (or the pytest selection given as arguments), then smoke().
export TMPDIR=/tmp
mkdir -p gpurun_out/t
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t/smoke.log 2>&1
