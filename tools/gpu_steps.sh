#!/bin/bash
# bench value vs the number of timed steps (pipeline fill / drain amortisation)
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for k in 20 60 120; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --steps $k > $O/steps_$k.log 2>&1
done
