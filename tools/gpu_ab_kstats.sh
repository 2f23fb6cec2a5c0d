#!/bin/bash
# per-kernel durations of library builds, one-at-a-time 8K encodes (no pipeline):
# bash tools/gpu_ab_kstats.sh TAG lib1 lib2 ...  -> gpurun_out/TAG/<lib>_<round>/run_kernel_stats.csv
set -e
export TMPDIR=/tmp
TAG=$1; shift
R=$PWD
mkdir -p gpurun_out/$TAG
for round in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    cd /tmp && JXG_LIB_PATH=$R/$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/${n}_$round -o run --output-format csv -- python3 $R/tools/ans_run.py 6 > $R/gpurun_out/$TAG/${n}_$round.log 2>&1
    cd $R
  done
done
