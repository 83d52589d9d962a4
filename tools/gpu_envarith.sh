#!/bin/bash
# env kernel cost of the reference build's arithmetic on one box: this host's rsqrtss table (for offline
# analysis), bench lines with the MSVC x64 arithmetic and in the scalar mode, then the phase profile of the first
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export O=gpurun_out/${TAG:-envarith}
mkdir -p $O
python - <<'PY'
import os, sys
import numpy as np
sys.path.insert(0, "reinforcement-learning_amd")
from rlgpu import arith
t, b = arith.rsqrt_table()
np.save(os.environ["O"] + "/rsqrt_table.npy", t)
print("rsqrt table bits", b, "formula bits", arith.formula_bits(), open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0])
PY
B="--no-cpu-baseline --no-legs --steps 4"
timeout -k 10 300 python -u bench.py $B > $O/bench_msvc.json 2> $O/bench_msvc.err || exit 1
timeout -k 10 300 python -u bench.py $B --arith scalar > $O/bench_scalar.json 2> $O/bench_scalar.err || exit 1
timeout -k 10 200 python -u tools/env_phase_profile.py 4096 24 64 procedural 0 > $O/phase_msvc.txt 2>&1 || exit 1
python - <<'PY'
import json, os
O = os.environ["O"]
for n in ("bench_msvc", "bench_scalar"):
    d = json.loads(open(f"{O}/{n}.json").read().strip().splitlines()[-1])
    print(n, round(d["value"]), "env-steps/s", "kernel_ms", round(d["roofline"]["kernel_ms"], 4), d["phase_s_per_iteration"])
PY
tail -32 $O/phase_msvc.txt
