#!/bin/bash
# Other BASELINE configs at N=1 (4K, 64 x 1080p batch at d0.5/1/2, 16384^2 P+F)
# and a gloo-rehearsed 2-rank sharded line.  Usage: bash tools/gpu_configs.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-cfg}
O=gpurun_out/$TAG
mkdir -p $O
B="python bench.py --no-cpu-baseline --alt-ans-streams 0 --alt-thesis 0"
timeout -k 10 200 $B --config 1 > $O/cfg_4k.log 2>&1
for d in 0.5 1.0 2.0; do
  timeout -k 10 200 $B --config 3 --steps 2 --warmup 1 --streams 3 --distance $d > $O/cfg_batch_d$d.log 2>&1
done
timeout -k 10 300 $B --config 4 --proposals 3 --steps 5 --warmup 1 > $O/cfg_16k_pf.log 2>&1
