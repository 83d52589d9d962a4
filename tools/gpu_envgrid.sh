#!/bin/bash
# env parity (custom / procedural / synthetic meshes, C2 size) + phase profiles on both meshes
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/eg
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_configs_gpu.py -k "not two_rank and not c4 and not c5" -x -q --timeout 300 --timeout-method thread > gpurun_out/eg/test.log 2>&1
tail -n 3 gpurun_out/eg/test.log
timeout -k 10 200 python -u tools/env_phase_profile.py 4096 24 64 procedural > gpurun_out/eg/procedural.txt 2>&1
timeout -k 10 200 python -u tools/env_phase_profile.py 4096 24 64 synthetic > gpurun_out/eg/synthetic.txt 2>&1
head -n 8 gpurun_out/eg/procedural.txt; grep -A4 slowest gpurun_out/eg/procedural.txt
head -n 8 gpurun_out/eg/synthetic.txt; grep -A4 slowest gpurun_out/eg/synthetic.txt
