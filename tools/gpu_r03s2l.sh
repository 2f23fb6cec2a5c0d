#!/bin/bash
set -e
export TMPDIR=/tmp
O=gpurun_out/r03s2l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_filters.py -x -v --timeout 200 --timeout-method thread > $O/gpu_filters.log 2>&1
