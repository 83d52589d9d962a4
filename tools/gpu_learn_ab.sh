#!/bin/bash
# Learn-phase A/B of library builds (VARIANTS="a t": rlgpu/librlgpu_<v>.so, "t" = the in-tree library): the H3
# GEMM bit-identity and gradient tests on the in-tree library, then tools/learn_bench.py alternating the variants at
# the C5 widths ([2048] x 4) and the C2 widths ([512] x 2).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-learnab}
V=${VARIANTS:-"a t"}
mkdir -p $O
lib() { [ "$1" = t ] && echo "" || echo "$PWD/reinforcement-learning_amd/rlgpu/librlgpu_$1.so"; }
timeout -k 10 600 python -u -m pytest tests/test_ppo.py -m gpu -x -q -k "${TESTS:-h3_quad or minibatch_grads or gemm_modes or c5}" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -n 2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in $V; do
    RLGPU_LIB=$(lib $v) timeout -k 10 300 python -u tools/learn_bench.py 6 h3 2048 4 > $O/c5_$v$i.txt 2>&1 || { tail -5 $O/c5_$v$i.txt; exit 1; }
    echo "c5 $v$i: $(grep 'learn_bench (' $O/c5_$v$i.txt | head -1)"
  done
done
for i in 1 2; do
  for v in $V; do
    RLGPU_LIB=$(lib $v) timeout -k 10 300 python -u tools/learn_bench.py 24 > $O/c2_$v$i.txt 2>&1 || { tail -5 $O/c2_$v$i.txt; exit 1; }
    echo "c2 $v$i: $(grep 'learn_bench (' $O/c2_$v$i.txt | head -1)"
  done
done
