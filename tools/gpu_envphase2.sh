#!/bin/bash
# env kernel phase profile at C2 size on both meshes
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ep
timeout -k 10 200 python -u tools/env_phase_profile.py 4096 24 64 procedural > gpurun_out/ep/procedural.txt 2>&1
timeout -k 10 200 python -u tools/env_phase_profile.py 4096 24 64 synthetic > gpurun_out/ep/synthetic.txt 2>&1
cat gpurun_out/ep/procedural.txt gpurun_out/ep/synthetic.txt
