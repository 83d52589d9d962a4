# row-GEMM A/B: the learn-phase microbenchmark with the full-row kernels off (0) / on (ring variants 1, 2),
# a kernel trace of each, then the PPO numerics tests with the default, then the given test files (if any)
export TMPDIR=/tmp
O=gpurun_out/${TAG:-rowab}
mkdir -p $O
for v in ${VARIANTS:-0 1 2}; do
  RLGPU_ROW_GEMM=$v timeout -k 10 200 python -u tools/learn_bench.py 24 >> $O/learn_$v.txt 2>&1 || { tail -20 $O/learn_$v.txt; exit 1; }
  RLGPU_ROW_GEMM=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python -u tools/learn_bench.py 8 > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  find $O/prof_$v -type f ! -name '*kernel_stats.csv' -delete
done
grep -H "learn_bench:" $O/learn_*.txt
timeout -k 10 600 python -u -m pytest tests/test_ppo.py tests/test_shared_head.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > $O/more_tests.log 2>&1 || { tail -40 $O/more_tests.log; exit 1; }
  tail -3 $O/more_tests.log
fi
