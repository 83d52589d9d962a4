# env collection split into arena groups on separate streams (tools/env_streams.py), then the C5-width PPO tests
export TMPDIR=/tmp
O=gpurun_out/${TAG:-streams}
mkdir -p $O
timeout -k 10 400 python -u tools/env_streams.py 64 4096 > $O/streams.txt 2>&1 || { tail -20 $O/streams.txt; exit 1; }
grep "K=" $O/streams.txt
timeout -k 10 600 python -u -m pytest tests/test_ppo.py -m gpu -x -q -k "c5 or forward_fp32_h3" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
