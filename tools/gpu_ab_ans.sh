#!/bin/bash
# same-box A/B of ANS chain builds: bash tools/gpu_ab_ans.sh TAG lib1 lib2 ... (paths)
set -e
export TMPDIR=/tmp
TAG=$1; shift
R=$PWD
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ans or config" > gpurun_out/$TAG/tests.log 2>&1
for round in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    cd /tmp && JXG_LIB_PATH=$R/$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/${n}_$round -o run --output-format csv -- python3 $R/tools/ans_run.py 6 > $R/gpurun_out/$TAG/${n}_$round.log 2>&1
    cd $R
  done
done
