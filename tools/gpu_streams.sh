#!/bin/bash
set -e
mkdir -p gpurun_out/streams
for C in prefix ans; do for S in 1 2 3 4; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --coder $C --streams $S --steps 12 > gpurun_out/streams/${C}_s$S.log 2>&1
done; done
