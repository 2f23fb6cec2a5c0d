#!/bin/bash
# Other BASELINE configs at N=1 (4K, 64 x 1080p batch at d0.5/1/2, 16384^2 P+F), the
# bench defaults (ANS through the streaming pipeline; prefix as the alt line).  Usage: bash tools/gpu_configs.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-cfg}
O=gpurun_out/$TAG
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-quality --no-single --alt-thesis 0"
timeout -k 10 200 $B --config 1 > $O/cfg_4k.log 2>&1
for d in 0.5 1.0 2.0; do
  timeout -k 10 200 $B --config 3 --steps 6 --warmup 3 --distance $d --alt-coder 0 > $O/cfg_batch_d$d.log 2>&1
done
timeout -k 10 300 $B --config 4 --proposals 3 --steps 4 --warmup 1 --alt-coder 0 > $O/cfg_16k_pf.log 2>&1
