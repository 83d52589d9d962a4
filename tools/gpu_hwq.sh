#!/bin/bash
# Grouped collection against the HIP runtime's hardware-queue count: bench lines (3 iterations) for collect groups 1 / 2 / 4
# with GPU_MAX_HW_QUEUES at the box default (4) and 8 / 16.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-hwq}
mkdir -p $O
B="--steps 3 --warmup 1 --no-cpu-baseline --no-legs"
for q in 4 8 16; do
  for g in 1 2 4; do
    GPU_MAX_HW_QUEUES=$q RLGPU_BENCH_COLLECT_GROUPS=$g timeout -k 10 240 python -u bench.py $B > $O/b.tmp 2>&1 || { tail -20 $O/b.tmp; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/b.tmp').read().strip().splitlines()[-1]); p={k: round(v*1e3,1) for k,v in d['phase_s_per_iteration'].items()}
print('hwq $q groups $g', round(d['value']), d['ms_per_step'], json.dumps(p)[:200])" | tee -a $O/summary.txt
  done
done
