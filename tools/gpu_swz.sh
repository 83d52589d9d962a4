#!/bin/bash
# swizzled H3 GEMM: bit-identity vs the ring kernel (test_gemm_ring), microbench, learn bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tools/gpu_ring.sh > /dev/null 2>&1 || { tail -30 gpurun_out/ring/test.log; exit 1; }
tail -3 gpurun_out/ring/test.log
grep -h "" gpurun_out/ring/bench_0.log gpurun_out/ring/bench_1.log
timeout -k 10 120 python -u tools/learn_bench.py 24 2>&1 | grep -v amdgpu.ids
