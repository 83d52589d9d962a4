# 128 x 256-tile H3 GEMM (RLGPU_H3_WIDE=1, gemm_h3w) against the default 128 x 128 gemm_x6 at C2 and C5 widths
export TMPDIR=/tmp
O=gpurun_out/${TAG:-wide}
mkdir -p $O
for v in 0 1; do
  RLGPU_H3_WIDE=$v timeout -k 10 300 python -u tools/learn_bench.py 8 h3 2048 4 > $O/c5_$v.txt 2>&1 || { tail -20 $O/c5_$v.txt; exit 1; }
  RLGPU_H3_WIDE=$v timeout -k 10 300 python -u tools/learn_bench.py 24 h3 > $O/c2_$v.txt 2>&1 || { tail -20 $O/c2_$v.txt; exit 1; }
done
grep -H "learn_bench\|forward / input\|weight-gradient" $O/*.txt
