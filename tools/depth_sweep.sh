#!/bin/bash
# 1080p stream throughput vs pipeline depth (lanes = GPU_MAX_HW_QUEUES - 1,
# capped at 12): latency-bound if ms/frame falls as 1/lanes.
O=gpurun_out/$1; mkdir -p $O
for q in 5 7 9 11 13; do
  JXG_BENCH_HW_QUEUES=$q timeout -k 10 120 python tools/stream_probe.py --mode plain --world 1 --w 1920 --h 1080 --frames 256 --warmup 32 >> $O/depth_1080p.log 2>&1 || exit $?
  JXG_BENCH_HW_QUEUES=$q timeout -k 10 120 python tools/stream_probe.py --mode host --world 1 --h 544 --frames 256 --warmup 32 >> $O/depth_slice8.log 2>&1 || exit $?
done
