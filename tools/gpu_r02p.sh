#!/bin/bash
set -e
export TMPDIR=/tmp
O=gpurun_out/r02p
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --config 3 --steps 2 --warmup 1"
for s in 1 2 3 4; do
  timeout -k 10 200 $B --streams $s > $O/batch_s$s.log 2>&1
done
timeout -k 10 200 $B --coder prefix > $O/batch_prefix_s1.log 2>&1
timeout -k 10 200 $B --coder prefix --streams 3 > $O/batch_prefix_s3.log 2>&1
