#!/bin/bash
# Same-box A/B of tools/var builds: the GPU test suite on the candidate, then
# per-kernel stats of one-at-a-time 8K encodes, two rounds each.
# Usage: bash tools/gpu_ab_var.sh TAG candidate base [more...]
set -e
export TMPDIR=/tmp
TAG=$1; CAND=$2; shift
R=$PWD
O=gpurun_out/$TAG
mkdir -p $O
JXG_LIB_PATH=$R/tools/var/libjxg_$CAND.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$CAND.log 2>&1
for round in 1 2; do
  for n in "$@"; do
    cd /tmp && JXG_LIB_PATH=$R/tools/var/libjxg_$n.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/${n}_$round -o run --output-format csv -- python3 $R/tools/ans_run.py 6 > $R/$O/${n}_$round.log 2>&1
    cd $R
  done
done
for n in "$@"; do
  JXG_LIB_PATH=$R/tools/var/libjxg_$n.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --alt-coder 0 --alt-thesis 0 > $O/bench_$n.log 2>&1
done
