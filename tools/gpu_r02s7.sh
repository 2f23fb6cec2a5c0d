#!/bin/bash
# merge chunk 32 / 64 / 128 and the write kernel at 2 waves per SIMD (no
# spills): GPU tests on wwpe2, kernel stats of one-at-a-time 8K encodes, two rounds
set -e
export TMPDIR=/tmp
O=gpurun_out/r02s7
R=$PWD
mkdir -p $O
JXG_LIB_PATH=$R/tools/var/libjxg_wwpe2.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_wwpe2.log 2>&1
for round in 1 2; do
  for n in ch64 ch32 ch128 wwpe2; do
    cd /tmp && JXG_LIB_PATH=$R/tools/var/libjxg_$n.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/${n}_$round -o run --output-format csv -- python3 $R/tools/ans_run.py 6 > $R/$O/${n}_$round.log 2>&1
    cd $R
  done
done
