#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r03m}
mkdir -p $O
for H in 544 4320; do
  JXG_SS_PROFILE=1 timeout -k 10 120 python -u tools/stream_probe.py --mode native --world 1 --h $H --frames 200 --warmup 30 >> $O/probe.log 2>&1 || exit 1
done
JXG_SS_PROFILE=1 timeout -k 10 120 python -u tools/stream_probe.py --mode native --world 2 --h 1088 --frames 200 --warmup 30 >> $O/probe.log 2>&1
