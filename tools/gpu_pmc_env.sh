# PMC passes (one counter group per run) over the env kernel only.
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex env_kernel --output-format csv -d gpurun_out/pmc/p$i -o run -- python tools/env_phase_profile.py 4096 8 > gpurun_out/pmc/p$i.log 2>&1 || exit 1
done
