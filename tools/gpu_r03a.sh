#!/bin/bash
# Round 3, first GPU pass: the new sharding tests, the whole GPU suite, a
# short default bench and a 2-rank gloo rehearsal of the streamed-shard bench.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03a}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 240 --timeout-method thread > $O/gpu_shard.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread --deselect tests/test_gpu_shard.py > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1
JXG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 2 > $O/bench_gloo2.log 2>&1
