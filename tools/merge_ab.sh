#!/bin/bash
# Merge-stage iteration on the GPU box: parity subset, a short bench.
# Usage: bash tools/merge_ab.sh TAG
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bigvb.py tests/test_gpu_configs.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python bench.py --steps 40 --no-cpu-baseline --no-quality --no-single --alt-coder 0 --alt-thesis 0 --alt-cjxl 0 > $O/bench.log 2>&1
