#!/bin/bash
# 256 x 256 H3 tiles (RLGPU_H3_QUAD=1) against the default: bit-identity test first, then the learn-phase
# microbenchmark alternating the two (C2, and C5 with C5=1), then a kernel trace of each.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-quad}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ppo.py -m gpu -x -v -k "h3_quad" --timeout 280 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for r in 1 2; do
  for v in 0 1; do
    RLGPU_H3_QUAD=$v timeout -k 10 200 python -u tools/learn_bench.py 24 >> $O/learn_$v.txt 2>&1 || { tail -20 $O/learn_$v.txt; exit 1; }
  done
done
grep -H "learn_bench:" $O/learn_*.txt
if [ "${C5:-0}" = 1 ]; then
  for v in 0 1; do
    RLGPU_H3_QUAD=$v timeout -k 10 300 python -u tools/learn_bench.py 4 h3 2048 4 >> $O/c5_$v.txt 2>&1 || { tail -20 $O/c5_$v.txt; exit 1; }
  done
  grep -H "learn_bench:" $O/c5_*.txt
fi
for v in 0 1; do
  RLGPU_H3_QUAD=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python -u tools/learn_bench.py 8 > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  find $O/prof_$v -type f ! -name '*kernel_stats.csv' -delete
  python tools/kstats.py $O/prof_$v/run_kernel_stats.csv 1 12 > $O/kstats_$v.txt 2>&1 || true
done
