# kernel trace of one grouped-collection iteration: do the groups' env launches overlap?
export TMPDIR=/tmp
O=gpurun_out/${TAG:-groups3}
mkdir -p $O
for g in 4 1; do
RLGPU_BENCH_COLLECT_GROUPS=$g timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t$g -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-legs > $O/t$g.log 2>&1 || { tail -20 $O/t$g.log; exit 1; }
python tools/trace_overlap.py $O/t$g/run_kernel_trace.csv || exit 1
rm -f $O/t$g/run_kernel_trace.csv
done
