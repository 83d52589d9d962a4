#!/bin/bash
# parity of the arithmetic-specialised env kernels, then their bench lines and the MSVC phase profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export O=gpurun_out/${TAG:-envspec}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gjk.py tests/test_env_gpu.py tests/test_x86_arith.py tests/test_wheel_rays.py ${EXTRA_TESTS} -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -n 3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-legs --steps 4"
timeout -k 10 300 python -u bench.py $B > $O/bench_msvc.json 2> $O/bench_msvc.err || exit 1
[ -n "$SCALAR" ] && { timeout -k 10 300 python -u bench.py $B --arith scalar > $O/bench_scalar.json 2> $O/bench_scalar.err || exit 1; }
timeout -k 10 200 python -u tools/gjk_bench.py > $O/gjk_bench.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/env_phase_profile.py 4096 24 64 procedural 0 > $O/phase_msvc.txt 2>&1 || exit 1
python - <<'PY'
import json, os
O = os.environ["O"]
for n in ("bench_msvc", "bench_scalar"):
    if not os.path.exists(f"{O}/{n}.json"):
        continue
    d = json.loads(open(f"{O}/{n}.json").read().strip().splitlines()[-1])
    print(n, round(d["value"]), "env-steps/s", "kernel_ms", round(d["roofline"]["kernel_ms"], 4), d["phase_s_per_iteration"])
PY
grep -E 'penetration|n=    1' $O/gjk_bench.txt
tail -12 $O/phase_msvc.txt
