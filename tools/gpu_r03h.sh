#!/bin/bash
# Round 3: the native shard stream (jxg_shard_stream_*): its GPU tests, the
# 2-process streamed-frames test, then the gloo 2-rank bench in both stream
# modes (native completion thread vs the Python protocol).
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03h}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 240 --timeout-method thread -k "native or stream" --deselect tests/test_gpu_shard.py::test_multiprocess_streamed_frames > $O/stream_tests.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py::test_multiprocess_streamed_frames -x -v -s --timeout 280 --timeout-method thread > $O/mp_stream_test.log 2>&1
for M in shard shard-py; do
  JXG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 40 --warmup 2 --mode $M --alt-replica 0 > $O/bench_gloo2_$M.log 2>&1
done
