#!/bin/bash
# round evidence: full -m gpu suite + smoke, the bench line (with CPU baseline), rocprofv3 kernel stats
# of the bench, and the env kernel's HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 4 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -n 3 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
python tools/kstats.py $O/prof/run_kernel_stats.csv 5 30 > $O/kstats.txt; head -n 20 $O/kstats.txt
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex env_kernel --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex env_kernel --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1 || exit 1
python tools/pmc_summary.py $O/fetch $O/write env_kernel 65536 $O/env_pmc.json procedural
