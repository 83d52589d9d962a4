#!/bin/bash
# GPU check: the given pytest selection first (SEL, default: the x86-arithmetic tests), then every -m gpu
# test, smoke() and one bench line (BENCHARGS, default without the CPU baseline).  Output under
# gpurun_out/$TAG.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-check}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${SEL:-tests/test_x86_arith.py} -m gpu -x -v --timeout 400 --timeout-method thread -s > $O/first.log 2>&1
rc=$?; tail -n 8 $O/first.log; [ $rc -eq 0 ] || exit $rc
[ -n "$ONLY" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 4 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 500 python -u bench.py ${BENCHARGS:---no-cpu-baseline} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
