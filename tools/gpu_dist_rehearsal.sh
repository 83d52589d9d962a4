# Two ranks of bench.py sharing the one GPU of the box over gloo: exercises the C++ Learner's
# collective callbacks (gradient all-reduce, advantage moments, return samples) end to end.
export TMPDIR=/tmp
mkdir -p gpurun_out
RLGPU_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --arenas 1024 > gpurun_out/dist2.log 2>&1
