#!/bin/bash
# env kernel A/B/...: the env parity tests on the in-tree library, then bench.py alternating the variants
# (VARIANTS="a b ..." -> reinforcement-learning_amd/rlgpu/librlgpu_<v>.so; "t" = the in-tree library),
# each variant's phase profile and its env-kernel HBM writes (WRITE_SIZE)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-envab}
V=${VARIANTS:-"a t"}
mkdir -p $O
lib() { [ "$1" = t ] && echo "" || echo "$PWD/reinforcement-learning_amd/rlgpu/librlgpu_$1.so"; }
timeout -k 10 600 python -u -m pytest tests/test_gjk.py tests/test_env_gpu.py tests/test_x86_arith.py tests/test_wheel_rays.py ${EXTRA_TESTS} -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -n 3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-legs --steps 4"
for i in 1 2; do
  for v in $V; do
    RLGPU_LIB=$(lib $v) timeout -k 10 300 python -u bench.py $B > $O/$v$i.json 2> $O/$v$i.err || exit 1
  done
done
for v in $V; do
  RLGPU_LIB=$(lib $v) timeout -k 10 200 python -u tools/env_phase_profile.py 4096 24 64 procedural 0 > $O/phase_$v.txt 2>&1 || exit 1
done
P="--steps 1 --warmup 0 --no-cpu-baseline --no-legs"
for v in $V; do
  RLGPU_LIB=$(lib $v) timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w$v -- python3 bench.py $P > $O/w$v.log 2>&1 || exit 1
done
O=$O V="$V" python - <<'PY'
import json, glob, csv, os
O = os.environ["O"]
for v in os.environ["V"].split():
    rows = [json.loads(open(f"{O}/{v}{i}.json").read().strip().splitlines()[-1]) for i in (1, 2)]
    tot, n = 0.0, 0
    for f in glob.glob(f"{O}/w{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "env_kernel" in r["Kernel_Name"] and int(r["Grid_Size"]) >= 65536:
                tot += float(r["Counter_Value"]); n += 1
    print(v, " ".join(f"{r['value']:.0f} env-steps/s env={r['roofline']['kernel_ms']*1e3:.0f}us" for r in rows),
          f"| WRITE_SIZE per env launch {tot / max(n, 1) * 1024 / 1e6:.1f} MB ({n} launches)")
PY
for v in $V; do echo "== $v"; grep -E "slowest workgroup per step|T5 narrowphase  |T5 deferred" $O/phase_$v.txt | head -4; done
