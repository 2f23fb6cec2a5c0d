#!/bin/bash
set -e
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
JXG_LIB_PATH=$PWD/tools/var/libjxg_sdbg.so JXG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-quality > $O/dflt.log 2>&1 || true
