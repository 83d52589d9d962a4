#!/bin/bash
# Timing-only A/B of library builds (VARIANTS="b t": rlgpu/librlgpu_<v>.so, "t" = the in-tree library): bench.py
# alternating the variants (no legs, no CPU baseline), then each variant's env phase profile.  For experiments
# whose bits are wrong on purpose (an ablation): no parity tests run here.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-timingab}
V=${VARIANTS:-"b t"}
mkdir -p $O
lib() { [ "$1" = t ] && echo "" || echo "$PWD/reinforcement-learning_amd/rlgpu/librlgpu_$1.so"; }
B="--no-cpu-baseline --no-legs --steps 4"
for i in 1 2; do
  for v in $V; do
    RLGPU_LIB=$(lib $v) timeout -k 10 300 python -u bench.py $B > $O/$v$i.json 2> $O/$v$i.err || exit 1
  done
done
for v in $V; do
  RLGPU_LIB=$(lib $v) timeout -k 10 200 python -u tools/env_phase_profile.py 4096 24 64 procedural 0 > $O/phase_$v.txt 2>&1 || exit 1
done
O=$O V="$V" python - <<'PY'
import json, os
O = os.environ["O"]
for v in os.environ["V"].split():
    rows = [json.loads(open(f"{O}/{v}{i}.json").read().strip().splitlines()[-1]) for i in (1, 2)]
    print(v, " ".join(f"{r['value']:.0f} env-steps/s env={r['roofline']['kernel_ms']*1e3:.0f}us "
                      f"collect={r['phase_s_per_iteration']['collect']*1e3:.1f}ms learn={r['phase_s_per_iteration']['learn']*1e3:.1f}ms" for r in rows))
PY
for v in $V; do echo "== $v"; grep -E "mean workgroup|T1 wheels|T2 car|T5 narrow pairs|T6 solve" $O/phase_$v.txt | head -8; done
