#!/bin/bash
# LayerNorm row-shape variants in the learn microbenchmark (kernel timing per class)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/lnv
for v in 0 1 2 3; do
  RLGPU_LNF_VARIANT=$v RLGPU_LNB_VARIANT=$v timeout -k 10 120 python -u tools/learn_bench.py 24 > gpurun_out/lnv/v$v.log 2>&1
  echo "== variant $v"; grep -v amdgpu.ids gpurun_out/lnv/v$v.log
done
