# row-GEMM A/B: learn-phase microbenchmark with the full-row kernel off / on, then the PPO numerics tests
export TMPDIR=/tmp
O=gpurun_out/${TAG:-rowab}
mkdir -p $O
for v in 0 1 0 1; do
  RLGPU_ROW_GEMM=$v timeout -k 10 200 python -u tools/learn_bench.py 24 >> $O/learn_$v.txt 2>&1 || { tail -20 $O/learn_$v.txt; exit 1; }
done
tail -n 12 $O/learn_0.txt $O/learn_1.txt
timeout -k 10 600 python -u -m pytest tests/test_ppo.py tests/test_shared_head.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
