#!/bin/bash
# env kernel arenas-per-workgroup / tick-inlining variants: parity of the in-tree build (2 arenas per
# workgroup), then env step time of each variant library (procedural SOCCAR mesh, late-ish states)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/apw
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_configs_gpu.py -k "not two_rank and not c5" -m gpu -x -q --timeout 300 --timeout-method thread > $O/env_tests.log 2>&1
rc=$?; tail -n 3 $O/env_tests.log; [ $rc -eq 0 ] || exit $rc
for v in apw4_inline apw4 apw2 apw1; do
  apw=${v#apw}; apw=${apw%_inline}
  RLGPU_ENV_APW=$apw RLGPU_LIB=build_ab/librlgpu_$v.so timeout -k 10 120 python tools/env_phase_profile.py 4096 16 64 procedural > $O/phase_$v.txt 2>&1 || exit 1
  head -n 1 $O/phase_$v.txt | sed "s/^/$v: /"
done
