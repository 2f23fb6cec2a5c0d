#!/bin/bash
# pipelined completion thread: shard tests, probes, gloo 2-rank benches (both stream modes)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03t}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -x -q --timeout 240 --timeout-method thread > $O/shard_tests.log 2>&1
for H in 544 1088 4320; do for M in host native; do
  JXG_SS_PROFILE=1 timeout -k 10 120 python -u tools/stream_probe.py --mode $M --world 1 --h $H --frames 300 --warmup 30 2>&1 | grep "mode\|rank" >> $O/probe.log
done; done
for M in shard shard-py; do
  JXG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 60 --warmup 2 --mode $M --alt-replica 0 > $O/bench_gloo2_$M.log 2>&1
done
