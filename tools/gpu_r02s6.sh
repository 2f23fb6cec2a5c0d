#!/bin/bash
# early assembly in the streaming pipeline: GPU tests on the candidate, then
# same-box benches (8K default, 4K, 64 x 1080p) of ch64 (without) and early
# (with), twice, and the host profile of the candidate at 1080p
set -e
export TMPDIR=/tmp
O=gpurun_out/r02s6
R=$PWD
mkdir -p $O
JXG_LIB_PATH=$R/tools/var/libjxg_early.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_early.log 2>&1
B="python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0"
for r in 1; do
  for n in ch64 early; do
    JXG_LIB_PATH=$R/tools/var/libjxg_$n.so timeout -k 10 200 $B --config 3 --steps 6 --warmup 3 > $O/b1080_${n}_$r.log 2>&1
    JXG_LIB_PATH=$R/tools/var/libjxg_$n.so timeout -k 10 200 $B --config 1 > $O/b4k_${n}_$r.log 2>&1
    JXG_LIB_PATH=$R/tools/var/libjxg_$n.so timeout -k 10 200 $B > $O/b8k_${n}_$r.log 2>&1
  done
done
JXG_LIB_PATH=$R/tools/var/libjxg_pprofe.so timeout -k 10 120 python tools/stream_timing.py 1920 1080 96 ans > $O/pprof_1080p.log 2>&1
