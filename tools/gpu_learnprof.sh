#!/bin/bash
# learn-phase microbenchmark (tools/learn_bench.py) under rocprofv3 kernel stats, per RLGPU_H3_RING setting
# usage: tools/gpu_learnprof.sh "0 1 4"
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/lp
for r in ${1:-0 1}; do
  RLGPU_H3_RING=$r timeout -k 10 120 python -u tools/learn_bench.py 24 > gpurun_out/lp/wall_$r.log 2>&1
  [ "$2" = "noprof" ] && { cat gpurun_out/lp/wall_$r.log; continue; }
  RLGPU_H3_RING=$r timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lp/prof_$r -o run -- python tools/learn_bench.py 12 > gpurun_out/lp/prof_$r.log 2>&1
  python tools/kstats.py gpurun_out/lp/prof_$r/run_kernel_stats.csv 1 14 > gpurun_out/lp/kstats_$r.txt
  grep learn_bench gpurun_out/lp/wall_$r.log
  cat gpurun_out/lp/kstats_$r.txt
done
