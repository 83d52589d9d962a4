#!/bin/bash
# Env kernel at HEAD: per-phase cycles (profiled launches, tools/env_phase_profile.py) and the instruction mix /
# wait counters of the bench's env launches (one rocprofv3 --pmc pass of 8 SQ counters, MI355X_MICROARCH.md).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-envmix}
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
timeout -k 10 300 python -u tools/env_phase_profile.py 4096 24 64 procedural 0 > $O/phase.txt 2>&1 || { tail -20 $O/phase.txt; exit 1; }
echo "phase profile done"
C=""
for c in SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU; do
  grep -q "\b$c\b" $O/avail.txt && C="$C $c"
done
echo "counters:$C"
timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex env_kernel --output-format csv -d $O/mix -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-legs > $O/mix.log 2>&1 || { tail -5 $O/mix.log; exit 1; }
echo "mix pass done"
C2=""
for c in SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH; do
  grep -q "\b$c\b" $O/avail.txt && C2="$C2 $c"
done
echo "counters2:$C2"
timeout -s KILL 90 rocprofv3 --pmc $C2 --kernel-include-regex env_kernel --output-format csv -d $O/mix2 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-legs > $O/mix2.log 2>&1 || { tail -5 $O/mix2.log; exit 1; }
echo "mix2 pass done"
