#!/bin/bash
# HBM traffic passes (FETCH_SIZE, WRITE_SIZE) for the front kernel, one pass each.
set -e
export TMPDIR=/tmp
R=$PWD
OUT=gpurun_out/pmc_front2
mkdir -p $OUT
for P in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -k 10 120 rocprofv3 --pmc $P --kernel-include-regex front_kernel -d $R/$OUT/$P -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/$OUT/$P.log 2>&1
  cd $R
done
timeout -k 10 200 python bench.py --coder ans --no-cpu-baseline > gpurun_out/bench_ans2.log 2>&1
