#!/bin/bash
# ac_hist iteration: parity subset, kernel trace A/B against tools/ab/libjxg_prev.so,
# phase clock (tools/ab/libjxg_fprof.so).  Usage: bash tools/hist_ab.sh TAG
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bigvb.py tests/test_gpu_shard.py tests/test_gpu_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
bash tools/ktrace_ab.sh $1 prev
JXG_LIB_PATH=$PWD/tools/ab/libjxg_fprof.so timeout -k 10 120 python tools/front_phase_probe.py 7 cjxl 5 > $O/phases.log 2>&1
