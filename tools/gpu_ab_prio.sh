#!/bin/bash
set -e
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
for round in 1 2; do
  for spec in base:16 plo:16 phi:16 plo:32 base:32; do
    n=${spec%%:*}; q=${spec#*:}
    JXG_BENCH_HW_QUEUES=$q JXG_LIB_PATH=$PWD/tools/var/libjxg_$n.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --steps 100 > $O/${n}_q${q}_$round.log 2>&1
  done
done
