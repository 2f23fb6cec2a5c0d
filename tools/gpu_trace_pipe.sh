#!/bin/bash
# Kernel timeline of the streaming bench (8K ANS) for library builds:
# bash tools/gpu_trace_pipe.sh TAG lib1 lib2 ...   -> gpurun_out/TAG/<lib>/run_kernel_trace.csv
set -e
export TMPDIR=/tmp
TAG=$1; shift
R=$PWD
mkdir -p gpurun_out/$TAG
for L in "$@"; do
  n=$(basename $L .so)
  cd /tmp && JXG_LIB_PATH=$R/$L timeout -k 10 180 rocprofv3 --kernel-trace -d $R/gpurun_out/$TAG/$n -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --steps 20 --warmup 3 > $R/gpurun_out/$TAG/$n.log 2>&1
  cd $R
done
