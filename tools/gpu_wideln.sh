# wide-row LayerNorm A/B at the C5 leg's widths (RLGPU_WIDE_LN=0 / 1 / 2), a kernel trace of the default, then
# the PPO gradient tests
export TMPDIR=/tmp
O=gpurun_out/${TAG:-wideln}
mkdir -p $O
for v in ${VARIANTS:-0 1 2}; do
  RLGPU_WIDE_LN=$v timeout -k 10 300 python -u tools/learn_bench.py 8 h3 2048 4 > $O/c5_$v.txt 2>&1 || { tail -20 $O/c5_$v.txt; exit 1; }
done
tail -n 7 $O/c5_*.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u tools/learn_bench.py 4 h3 2048 4 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -type f ! -name '*kernel_stats.csv' -delete
if [ -z "$NOTESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_ppo.py tests/test_shared_head.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
fi
