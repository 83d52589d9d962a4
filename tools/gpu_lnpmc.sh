#!/bin/bash
# LayerNorm row kernels of the learn phase: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and
# SQ counters over tools/learn_bench.py (RLGPU_H3_RING=0)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/lnpmc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "ln_act|gemm_x6|gather_rows|policy_loss|reduce" --output-format csv -d gpurun_out/lnpmc/p$i -o run -- python tools/learn_bench.py 4 > gpurun_out/lnpmc/p$i.log 2>&1
done
python tools/pmc_table.py gpurun_out/lnpmc > gpurun_out/lnpmc/table.txt
cat gpurun_out/lnpmc/table.txt
