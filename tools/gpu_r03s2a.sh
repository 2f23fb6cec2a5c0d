#!/bin/bash
# restoration filters: GPU parity + the whole GPU suite, filter cost probe, default bench
set -e
export TMPDIR=/tmp
O=gpurun_out/r03s2a
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_filters.py -x -v --timeout 120 --timeout-method thread > $O/gpu_filters.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -u tools/filters_probe.py > $O/filters_probe.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
