#!/bin/bash
# full GPU suite, default bench, gloo 2-rank default (shard) bench, native probe
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03v}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
JXG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 60 --warmup 2 > $O/bench_gloo2.log 2>&1
