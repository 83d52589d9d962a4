# Round checkpoint on the GPU box: every -m gpu test, smoke(), bench (with CPU baseline), rocprofv3
# kernel stats (CSV) of the bench, env-kernel FETCH_SIZE / WRITE_SIZE passes.
export TMPDIR=/tmp
mkdir -p gpurun_out/round
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/round/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/round/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/round/prof -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/round/prof.log 2>&1 && \
python tools/kstats.py gpurun_out/round/prof/run_kernel_stats.csv 4 40 > gpurun_out/round/kstats.txt && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex env_kernel --output-format csv -d gpurun_out/round/fetch -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/round/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex env_kernel --output-format csv -d gpurun_out/round/write -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/round/write.log 2>&1 && \
timeout -k 10 200 python tools/infer_trace.py > gpurun_out/round/infer_trace.txt 2>&1 && \
timeout -k 10 200 python tools/env_phase_profile.py 4096 32 600 > gpurun_out/round/env_phase_w600.txt 2>&1 && \
timeout -k 10 120 python tools/env_phase_profile.py 4096 32 8 > gpurun_out/round/env_phase_w8.txt 2>&1
