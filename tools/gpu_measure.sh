# Measurement pass on the GPU box: GEMM microbench, env per-phase profile, rocprofv3 kernel stats (CSV).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 && \
timeout -k 10 120 python tools/env_phase_profile.py > gpurun_out/env_phase.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profcsv -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/profcsv.log 2>&1
