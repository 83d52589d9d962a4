# bench per training GEMM arithmetic + kernel stats of the default (h3)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --train-gemm x6 > gpurun_out/bench_x6.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --train-gemm h3 > gpurun_out/bench_h3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profcsv -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/profcsv.log 2>&1 && \
python tools/kstats.py gpurun_out/profcsv/run_kernel_stats.csv 4 30 > gpurun_out/kstats.txt
