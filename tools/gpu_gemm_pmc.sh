# GEMM microbench (kernel stats) + SQ PMC passes over the H3 GEMM kernel on the main PPO shapes.
export TMPDIR=/tmp
mkdir -p gpurun_out/gpmc
timeout -k 10 120 python tools/gemm_bench.py 0,2 > gpurun_out/gpmc/gemm_bench.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gpmc/ks -o run -- python tools/gemm_bench.py 2 0,5 > gpurun_out/gpmc/ks.log 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex gemm_x6 --output-format csv -d gpurun_out/gpmc/p$i -o run -- python tools/gemm_bench.py 2 0,5 > gpurun_out/gpmc/p$i.log 2>&1 || exit 1
done
