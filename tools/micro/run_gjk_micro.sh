#!/bin/bash
# builds gjk_micro.hip with several flag sets (here, on the CPU side: call with "build"), runs them (GPU box)
cd "$(dirname "$0")"
if [ "$1" = build ]; then
  H=/opt/rocm/bin/hipcc
  B="--offload-arch=gfx950 -std=c++17 -ffp-contract=off -Wno-unused-variable"
  $H $B -O3 gjk_micro.hip -o gjk_O3 &
  wait
  exit 0
fi
for v in gjk_O3; do echo "== $v"; timeout -k 5 60 ./$v || exit 1; done
