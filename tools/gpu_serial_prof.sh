# Kernel stats of the bench with the minibatch's two model passes serialised (isolated kernel times).
export TMPDIR=/tmp
mkdir -p gpurun_out
export RLGPU_SERIAL_MINIBATCH=1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_serial.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profser -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/profser.log 2>&1
