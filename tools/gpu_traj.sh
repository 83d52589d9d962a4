#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/final
timeout -k 10 300 python -u -m pytest tests/test_trajectories.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/final/traj.log 2>&1
rc=$?; tail -n 5 gpurun_out/final/traj.log; exit $rc
