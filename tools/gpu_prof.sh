# bench line + rocprofv3 kernel stats of the bench (CSV + summary)
export TMPDIR=/tmp
mkdir -p gpurun_out/p
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/p/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p/prof -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/p/prof.log 2>&1 && \
python tools/kstats.py gpurun_out/p/prof/run_kernel_stats.csv 4 40 > gpurun_out/p/kstats.txt
