# Env kernel per-phase cycles at several arena counts (1, 4 waves per SIMD): issue- vs latency-bound.
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 1024 4096 8192; do
  timeout -k 10 120 python tools/env_phase_profile.py $n 32 > gpurun_out/env_phase_$n.log 2>&1 || exit 1
done
