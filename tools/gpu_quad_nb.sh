#!/bin/bash
# gemm_h3q LDS buffers: NB=1 (64 KB, room for the other stream's kernels) vs NB=2 (128 KB), in the C2 / C5
# learn-phase microbenchmark, after the bit-identity test with NB=1; then isolated launches of each (kernel trace of
# tools/blaslt_probe.py with the quad kernel forced on).
export TMPDIR=/tmp
O=gpurun_out/${TAG:-quadnb}
mkdir -p $O
RLGPU_H3_QUAD_NB=1 timeout -k 10 300 python -u -m pytest tests/test_ppo.py -m gpu -x -q -k "h3_quad" --timeout 280 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for cfg in "0 2" "1 2" "1 1" "0 2" "1 2" "1 1"; do
  set -- $cfg
  RLGPU_H3_QUAD=$1 RLGPU_H3_QUAD_NB=$2 timeout -k 10 200 python -u tools/learn_bench.py 24 > $O/c2.tmp 2>&1 || { tail -20 $O/c2.tmp; exit 1; }
  echo "c2 quad=$1 nb=$2: $(grep 'learn_bench (' $O/c2.tmp)" | tee -a $O/summary.txt
done
for nb in 2 1; do
  RLGPU_H3_QUAD_NB=$nb timeout -k 10 300 python -u tools/learn_bench.py 6 h3 2048 4 > $O/c5.tmp 2>&1 || { tail -20 $O/c5.tmp; exit 1; }
  echo "c5 default nb=$nb: $(grep 'learn_bench (' $O/c5.tmp)" | tee -a $O/summary.txt
done
for nb in 2 1; do
  RLGPU_H3_QUAD=1 RLGPU_H3_QUAD_NB=$nb timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/iso_$nb -o run -- python3 -u tools/blaslt_probe.py > $O/iso_$nb.log 2>&1 || { tail -5 $O/iso_$nb.log; exit 1; }
  find $O/iso_$nb -type f ! -name '*kernel_stats.csv' -delete
done
