# GAE microbenchmark on one box: HIP-event medians, then a kernel trace of the same calls
export TMPDIR=/tmp
O=gpurun_out/${TAG:-gae}
mkdir -p $O
timeout -k 10 200 python -u tools/gae_bench.py 24 50 > $O/gae24.txt 2>&1 || { tail -20 $O/gae24.txt; exit 1; }
timeout -k 10 200 python -u tools/gae_bench.py 21 50 > $O/gae21.txt 2>&1 || { tail -20 $O/gae21.txt; exit 1; }
cat $O/gae24.txt $O/gae21.txt | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u tools/gae_bench.py 24 20 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -type f ! -name '*kernel_stats.csv' -delete
python tools/kstats.py $O/prof/run_kernel_stats.csv 1 12
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gae.py tests/test_trajectories.py ${MORE_TESTS} -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
