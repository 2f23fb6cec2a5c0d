#!/bin/bash
# native shard stream: depth / lag sweep at a 1/8 slice
export TMPDIR=/tmp
O=gpurun_out/${1:-r03s}
mkdir -p $O
for DL in "12 3" "8 3" "6 3" "12 1" "12 6" "10 2"; do set -- $DL
  JXG_SS_DEPTH=$1 JXG_SS_LAG=$2 JXG_SS_PROFILE=1 timeout -k 10 120 python -u tools/stream_probe.py --mode native --world 1 --h 544 --frames 300 --warmup 30 2>&1 | grep "mode\|rank" | sed "s/^/d$1 l$2 /" >> $O/probe.log || exit 1
done
timeout -k 10 120 python -u tools/stream_probe.py --mode host --world 1 --h 544 --frames 300 --warmup 30 2>&1 | grep "mode" >> $O/probe.log
