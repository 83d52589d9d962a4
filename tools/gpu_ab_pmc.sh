# A/B of two library builds: bench.py (3 alternating runs each) plus each build's env-kernel WRITE_SIZE
export TMPDIR=/tmp
bash tools/gpu_ab.sh || exit 1
for v in a b; do
  if [ $v = a ]; then L=$RLGPU_LIB_A; else L=""; fi
  RLGPU_LIB=$L timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex env_kernel --output-format csv -d gpurun_out/ab/w$v -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ab/w$v.log 2>&1 || exit 1
  python3 -c "
import csv,glob
rows=[r for f in glob.glob('gpurun_out/ab/w$v/**/*counter_collection.csv',recursive=True) for r in csv.DictReader(open(f))]
v=[float(r['Counter_Value']) for r in rows if r['Counter_Name']=='WRITE_SIZE']
print('$v WRITE_SIZE KB per launch', sum(v)/max(len(v),1), len(v))"
done
