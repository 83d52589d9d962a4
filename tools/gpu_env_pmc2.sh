# SQ PMC passes over the env kernel only (instruction mix, wait breakdown, instruction fetch).
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc2/avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_IFETCH"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex env_kernel --output-format csv -d gpurun_out/pmc2/p$i -o run -- python tools/env_scale.py 4096 > gpurun_out/pmc2/p$i.log 2>&1 || exit 1
done
