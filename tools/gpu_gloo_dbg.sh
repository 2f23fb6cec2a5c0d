#!/bin/bash
# 2-rank gloo sharded bench on one GPU, product and a variant library
set -e
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
JXG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-quality --mode shard --alt-coder 0 --alt-thesis 0 > $O/prod.log 2>&1 || true
JXG_LIB_PATH=$PWD/tools/var/libjxg_e20k.so JXG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-quality --mode shard --alt-coder 0 --alt-thesis 0 > $O/e20k.log 2>&1 || true
