#!/bin/bash
set -e
export TMPDIR=/tmp
O=gpurun_out/r02e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
JXG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_gloo2_strong.log 2>&1
JXG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 5 --warmup 2 --config 4 > $O/bench_gloo4_16k.log 2>&1
JXG_LIB_PATH=$PWD/tools/var/libjxg_mprof.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --alt-ans-streams 0 --alt-thesis 0 --no-quality > $O/bench_mprof.log 2>&1
