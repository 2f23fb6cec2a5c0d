#!/bin/bash
# bench defaults at N=1 and a 2-rank gloo rehearsal of the N>1 defaults (replica + sharded line)
set -e
export TMPDIR=/tmp
O=gpurun_out/r02k
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quality > $O/bench.log 2>&1
JXG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_gloo2.log 2>&1
