#!/bin/bash
# host time per streaming submit (JXG_PIPE_PROFILE build): bash tools/gpu_pprof.sh TAG LIB
set -e
export TMPDIR=/tmp
O=gpurun_out/$1; L=$2
mkdir -p $O
JXG_LIB_PATH=$PWD/$L timeout -k 10 120 python tools/stream_timing.py 1920 1080 64 ans > $O/pprof_1080p_ans.log 2>&1
JXG_LIB_PATH=$PWD/$L timeout -k 10 120 python tools/stream_timing.py 1920 1080 64 prefix > $O/pprof_1080p_prefix.log 2>&1
JXG_LIB_PATH=$PWD/$L timeout -k 10 120 python tools/stream_timing.py 7680 4320 24 ans > $O/pprof_8k_ans.log 2>&1
