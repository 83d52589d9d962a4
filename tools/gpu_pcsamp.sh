# PC sampling (beta) of the env kernel: instruction-level hotspots
export TMPDIR=/tmp
mkdir -p gpurun_out/pcs
timeout -k 10 60 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 --output-format csv -d gpurun_out/pcs/s -o run -- python tools/env_scale.py 4096 > gpurun_out/pcs/s.log 2>&1 || \
timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 100 --output-format csv -d gpurun_out/pcs/h -o run -- python tools/env_scale.py 4096 > gpurun_out/pcs/h.log 2>&1
ls -la gpurun_out/pcs/* > gpurun_out/pcs/ls.txt 2>&1
