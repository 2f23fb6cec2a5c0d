#!/bin/bash
# Per-kernel durations of one-at-a-time 8K encodes (tools/front_phase_probe.py)
# under rocprofv3 --kernel-trace --stats, for the product library and variant
# builds (tools/ab/libjxg_NAME.so).  Usage: bash tools/ktrace_ab.sh TAG NAME...
set -e
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/$1; shift
mkdir -p $O
for n in base "$@"; do
  L=$R/jpeg-xl-lossy-image-compression-thesis_amd/jxg/libjxg.so
  [ $n != base ] && L=$R/tools/ab/libjxg_$n.so
  cd /tmp
  JXG_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$n -o run --output-format csv -- python3 $R/tools/front_phase_probe.py 7 cjxl 10 > $O/$n.log 2>&1
  cd $R
done
