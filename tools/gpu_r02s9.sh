#!/bin/bash
# small-frame pipeline: lag 3 / 12 lanes (default) vs lag 4 vs lag 4 + 16
# lanes, 64 x 1080p and 4K, two rounds on one box; stream tests on l4m16
set -e
export TMPDIR=/tmp
O=gpurun_out/r02s9
R=$PWD
mkdir -p $O
JXG_LIB_PATH=$R/tools/var/libjxg_l4m16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_l4m16.log 2>&1
B="python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0"
for r in 1 2; do
  for n in base l4 l4m16; do
    JXG_LIB_PATH=$R/tools/var/libjxg_$n.so timeout -k 10 200 $B --config 3 --steps 6 --warmup 3 > $O/b1080_${n}_$r.log 2>&1
    JXG_LIB_PATH=$R/tools/var/libjxg_$n.so timeout -k 10 200 $B --config 1 > $O/b4k_${n}_$r.log 2>&1
  done
done
