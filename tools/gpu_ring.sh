#!/bin/bash
# ring GEMM (gemm_h3r) check + timing on the GPU box: bit-identity vs the staged kernel, then the
# microbenchmark under each RLGPU_H3_RING setting
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ring
timeout -k 10 400 python -u -m pytest tests/test_gemm_ring.py -x -v --timeout 380 --timeout-method thread > gpurun_out/ring/test.log 2>&1
for r in 0 1 2 3; do
  RLGPU_H3_RING=$r timeout -k 10 120 python -u tools/gemm_bench.py 2 0,2,3,4 > gpurun_out/ring/bench_$r.log 2>&1
done
tail -n 3 gpurun_out/ring/test.log
grep -h "" gpurun_out/ring/bench_*.log
