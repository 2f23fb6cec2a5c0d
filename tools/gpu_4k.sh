#!/bin/bash
# 4K streaming investigation: host time per submit (JXG_PIPE_PROFILE build)
# and the kernel timeline of the 4K bench (config 1)
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
R=$PWD
mkdir -p $O
JXG_LIB_PATH=$R/tools/var/libjxg_pprof.so timeout -k 10 120 python tools/stream_timing.py 3840 2160 100 ans > $O/pprof_4k_ans.log 2>&1
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace -d $R/$O/trace4k -o run --output-format csv -- python3 $R/bench.py --config 1 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --steps 60 --warmup 16 > $R/$O/bench4k_trace.log 2>&1
cd $R && timeout -k 10 180 python3 bench.py --config 1 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/bench4k.log 2>&1
