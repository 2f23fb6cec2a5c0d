#!/bin/bash
# merge_eval pruning: parity, then A/B vs a build without it
set -e
export TMPDIR=/tmp
O=gpurun_out/r03s2k
mkdir -p $O
JXG_LIB_PATH=tools/var/libjxg_mprune.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_filters.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1
B="python bench.py --no-cpu-baseline --no-quality --alt-coder 0"
for r in 1 2; do
  JXG_LIB_PATH=tools/var/libjxg_mprune.so timeout -k 10 200 $B > $O/prune_r$r.log 2>&1
  timeout -k 10 200 $B > $O/mnoprune_r$r.log 2>&1
done
JXG_LIB_PATH=tools/var/libjxg_mprune.so timeout -k 10 200 python tools/merge_probe.py > $O/probe_prune.log 2>&1
timeout -k 10 200 python tools/merge_probe.py > $O/probe_mnoprune.log 2>&1
