#!/bin/bash
# builds gjk_micro.hip with several flag sets (here, on the CPU side: call with "build"), runs them (GPU box)
cd "$(dirname "$0")"
if [ "$1" = build ]; then
  H=/opt/rocm/bin/hipcc
  B="--offload-arch=gfx950 -std=c++17 -ffp-contract=off -Wno-unused-variable"
  $H $B -O3 gjk_micro.hip -o gjk_O3 &
  $H $B -O3 -fno-hip-fp32-correctly-rounded-divide-sqrt gjk_micro.hip -o gjk_fastdiv &
  $H $B -O1 gjk_micro.hip -o gjk_O1 &
  wait
  exit 0
fi
for v in gjk_O3 gjk_fastdiv gjk_O1; do echo "== $v"; timeout -k 5 60 ./$v || exit 1; done
