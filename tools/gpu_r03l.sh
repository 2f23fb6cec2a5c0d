#!/bin/bash
# per-rank load emulation: a 1/8 and 1/4 slice of the 8K frame on one context
export TMPDIR=/tmp
O=gpurun_out/${1:-r03l}
mkdir -p $O
for H in 544 1088 4320; do for M in host native; do
  timeout -k 10 120 python -u tools/stream_probe.py --mode $M --world 1 --h $H --frames 200 --warmup 30 2>&1 | grep mode >> $O/probe.log || exit 1
done; done
