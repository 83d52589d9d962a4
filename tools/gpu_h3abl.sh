# H3 GEMM ablation timings (microbench only, shape 0 = 50000x512x512 pre-split, shape 8 = 8192^3)
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for v in ${ABL:-0 7 8 9}; do
  RLGPU_H3_VARIANT=$v timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abl/k$v -o run -- python tools/gemm_bench.py 2 0,8 > gpurun_out/abl/k$v.log 2>&1 || exit 1
done
