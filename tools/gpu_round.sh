#!/bin/bash
# Round checkpoint on one GPU box (TAG names the output folder and the profile files):
#   every -m gpu test, smoke(), the default bench line (with CPU baseline and legs), the bench under
#   rocprofv3 --kernel-trace --stats, the env kernel's FETCH_SIZE / WRITE_SIZE passes (separate runs,
#   MI355X_MICROARCH.md) summarised with the trace's kernel duration, and the training GEMMs' MFMA counters.
# Every GPU step runs under its own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-round}
O=gpurun_out/$TAG
mkdir -p $O
SKIP_TESTS=${SKIP_TESTS:-0}
if [ "$SKIP_TESTS" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  echo "smoke ok"
fi
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench_line.json
echo "bench done"
B1="--steps 1 --warmup 0 --no-cpu-baseline --no-legs"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs > $O/ks.log 2>&1 || { tail -5 $O/ks.log; exit 1; }
python tools/kstats.py $O/ks/run_kernel_stats.csv 4 40 > $O/kstats.txt
echo "kernel trace done"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex env_kernel --output-format csv -d $O/fetch -o run -- python3 bench.py $B1 > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex env_kernel --output-format csv -d $O/write -o run -- python3 bench.py $B1 > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
python tools/pmc_summary.py $O/fetch $O/write env_kernel 4096 $O/env_pmc.json procedural $O/ks/run_kernel_stats.csv $TAG
echo "pmc passes done"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F16 SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex gemm --output-format csv -d $O/mfma -o run -- python3 bench.py $B1 > $O/mfma.log 2>&1 || { tail -5 $O/mfma.log; exit 1; }
python tools/mfma_summary.py $O/mfma $O/ks/run_kernel_stats.csv $TAG > $O/gemm_mfma_pmc.txt
echo "mfma pass done"
