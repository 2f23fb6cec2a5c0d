#!/bin/bash
# host profile of pipeline builds at 1080p ANS: bash tools/gpu_pprof2.sh TAG lib...
set -e
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
for r in 1 2; do
for L in "$@"; do
  n=$(basename $L .so)
  JXG_LIB_PATH=$PWD/$L timeout -k 10 120 python tools/stream_timing.py 1920 1080 96 ans > $O/${n}_$r.log 2>&1
done
done
