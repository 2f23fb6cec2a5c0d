#!/bin/bash
set -e
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
for round in 1 2 3; do
  for q in 16 24 32; do
    JXG_BENCH_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --steps 100 > $O/q${q}_$round.log 2>&1
  done
done
JXG_BENCH_HW_QUEUES=32 timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --config 3 --steps 6 --warmup 3 > $O/b_q32.log 2>&1
JXG_BENCH_HW_QUEUES=16 timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --config 3 --steps 6 --warmup 3 > $O/b_q16.log 2>&1
