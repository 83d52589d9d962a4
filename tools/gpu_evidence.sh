#!/bin/bash
# Round evidence on one box: the bench under rocprofv3 kernel trace + stats, the env kernel's HBM traffic
# (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md), and MFMA counters over the training
# GEMMs.  Each rocprofv3 run is a step of its own under a time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export O=gpurun_out/${TAG:-evidence}
mkdir -p $O
B1="--steps 1 --warmup 0 --no-cpu-baseline --no-legs"
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
echo "counters listed: $(grep -c . $O/avail.txt)"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > $O/ks.log 2>&1 || { tail -5 $O/ks.log; exit 1; }
echo "kernel trace done"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex env_kernel --output-format csv -d $O/fetch -o run -- python3 bench.py $B1 > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
echo "fetch pass done"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex env_kernel --output-format csv -d $O/write -o run -- python3 bench.py $B1 > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
echo "write pass done"
MF=""
for c in SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F16 SQ_BUSY_CYCLES SQ_WAVES; do
  grep -q "\b$c\b" $O/avail.txt && MF="$MF $c"
done
echo "mfma counters:$MF"
if [ -n "$MF" ]; then
  timeout -s KILL 240 rocprofv3 --pmc $MF GRBM_GUI_ACTIVE --kernel-include-regex gemm --output-format csv -d $O/mfma -o run -- python3 bench.py $B1 > $O/mfma.log 2>&1 || { tail -5 $O/mfma.log; exit 1; }
  echo "mfma pass done"
fi
ls -R $O | head -40
