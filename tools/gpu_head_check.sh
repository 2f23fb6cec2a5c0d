#!/bin/bash
# the committed tree as the round-end driver runs it: GPU tests, smoke, default bench
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-head_check}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
