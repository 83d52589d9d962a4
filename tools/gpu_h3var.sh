# H3 GEMM variants: kernel times (microbench under rocprofv3) + bench per variant
export TMPDIR=/tmp
mkdir -p gpurun_out/h3var
for v in ${H3VARS:-0 4}; do
  RLGPU_H3_VARIANT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/h3var/k$v -o run -- python tools/gemm_bench.py 2 > gpurun_out/h3var/k$v.log 2>&1 || exit 1
  python tools/kstats.py gpurun_out/h3var/k$v/run_kernel_stats.csv 1 12 > gpurun_out/h3var/kstats$v.txt
  RLGPU_H3_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/h3var/bench$v.log 2>&1 || exit 1
done
