#!/bin/bash
# where a 1/8-frame shard spends GPU time (kernel + copy traces), both stream modes
export TMPDIR=/tmp
O=gpurun_out/${1:-r03o}
R=$GRAFT_REPO_ROOT
mkdir -p $O
cd /tmp
for M in host native; do
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/prof_$M -o run --output-format csv -- python3 $R/tools/stream_probe.py --mode $M --world 1 --h 544 --frames 100 --warmup 30 > $R/$O/prof_$M.log 2>&1 || exit 1
done
