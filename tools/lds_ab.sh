#!/bin/bash
# Same-box A/B of the front kernel's LDS layout (tools/ab/libjxg_s67.so: row
# stride 67, no skew) against the product: parity of the variant first, then
# alternating short benches.  Usage: bash tools/lds_ab.sh TAG
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
V=$PWD/tools/ab/libjxg_s67.so
JXG_LIB_PATH=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filters.py tests/test_gpu_aq.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_s67.log 2>&1
B="--steps 40 --no-cpu-baseline --no-quality --no-single --alt-coder 0 --alt-thesis 0 --alt-cjxl 0"
for r in 1 2; do
  timeout -k 10 200 python bench.py $B > $O/bench_base_$r.log 2>&1
  JXG_LIB_PATH=$V timeout -k 10 200 python bench.py $B > $O/bench_s67_$r.log 2>&1
done
# host-CPU A/B: blocking-sync events (JXG_EVENT_BLOCKING=1) on the headline and
# on the 8-rank gloo rehearsal
JXG_EVENT_BLOCKING=1 timeout -k 10 200 python bench.py $B > $O/bench_evblock.log 2>&1
JXG_EVENT_BLOCKING=1 JXG_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 8 --steps 20 --warmup 3 > $O/bench_gloo8_evblock.log 2>&1
