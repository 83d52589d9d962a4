#!/bin/bash
# procedural SOCCAR mesh: parity test, then the bench on both meshes (no CPU baseline)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03b
timeout -k 10 300 python -u -m pytest tests/test_env_gpu.py -k "procedural_soccar" -x -v --timeout 280 --timeout-method thread > gpurun_out/r03b/test.log 2>&1
tail -n 2 gpurun_out/r03b/test.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03b/bench_proc.json 2> gpurun_out/r03b/bench_proc.err
cat gpurun_out/r03b/bench_proc.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline --mesh synthetic > gpurun_out/r03b/bench_syn.json 2> gpurun_out/r03b/bench_syn.err
cat gpurun_out/r03b/bench_syn.json
