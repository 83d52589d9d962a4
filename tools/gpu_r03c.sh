#!/bin/bash
# env parity with the internal-edge adjustment (all meshes), swizzled H3 GEMM bit-identity, learn bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03c
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_configs_gpu.py tests/test_plugins.py tests/test_mesh.py -k "not two_rank and not c4 and not c5" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03c/env_tests.log 2>&1
rc=$?
tail -n 15 gpurun_out/r03c/env_tests.log
[ $rc -eq 0 ] || exit $rc
tools/gpu_swz.sh
