#!/bin/bash
# box-triangle GJK / EPA: device vs oracle bit for bit, then the env parity tests that run the mesh path
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/gjk
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gjk.py tests/test_boxbox.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/gjk_test.log 2>&1
rc=$?; tail -n 12 $O/gjk_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_configs_gpu.py tests/test_mesh.py -m gpu -k "not two_rank and not c5" -x -v --timeout 300 --timeout-method thread > $O/env_tests.log 2>&1
rc=$?; tail -n 25 $O/env_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/env_phase_profile.py 4096 16 64 procedural > $O/phase.txt 2>&1; head -n 3 $O/phase.txt
