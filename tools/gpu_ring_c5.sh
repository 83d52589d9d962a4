# H3 forward-GEMM kernel A/B at the C5 leg's widths: the register-staged gemm_x6 (RLGPU_H3_RING=0) against the
# LDS-DMA ring variants 1..4 (csrc/ppo.hip h3_ring), tools/learn_bench.py 8 h3 2048 4
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ringc5}
mkdir -p $O
for v in ${VARIANTS:-0 1 2 3 4}; do
  RLGPU_H3_RING=$v timeout -k 10 300 python -u tools/learn_bench.py 8 h3 ${WIDTH:-2048} ${DEPTH:-4} > $O/ring_$v.txt 2>&1 || { tail -20 $O/ring_$v.txt; exit 1; }
done
grep -H "learn_bench\|forward / input" $O/ring_*.txt
