#!/bin/bash
# Front-kernel iteration on the GPU box: parity subset, phase profile
# (tools/ab/libjxg_fprof.so), a short bench (headline + roofline + e4).
# Usage: bash tools/front_ab.sh TAG
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_filters.py tests/test_gpu_aq.py tests/test_gpu_bigvb.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
JXG_LIB_PATH=$PWD/tools/ab/libjxg_fprof.so timeout -k 10 120 python tools/front_phase_probe.py 7 cjxl 5 > $O/phases.log 2>&1
JXG_LIB_PATH=$PWD/tools/ab/libjxg_fprof.so timeout -k 10 120 python tools/front_phase_probe.py 4 cjxl 5 >> $O/phases.log 2>&1
timeout -k 10 300 python bench.py --steps 40 --no-cpu-baseline --no-quality --no-single --alt-coder 0 --alt-thesis 0 --alt-cjxl 0 > $O/bench.log 2>&1
