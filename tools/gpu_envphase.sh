# Env per-phase cycles early (8 warm steps) and late (600 warm steps) in the episodes
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/env_phase_profile.py 4096 32 8 > gpurun_out/env_phase_w8.log 2>&1 && \
timeout -k 10 200 python tools/env_phase_profile.py 4096 32 600 > gpurun_out/env_phase_w600.log 2>&1
