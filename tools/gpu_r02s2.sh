#!/bin/bash
# Bench + kernel stats on the restored tree, and the per-phase merge_eval
# cycle profile (JXG_MERGE_PROFILE build in tools/var).
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r02s2}
R=$PWD
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
JXG_LIB_PATH=$R/tools/var/libjxg_mprof.so timeout -k 10 120 python tools/mprof_run.py 4 > $O/mprof.log 2>&1
cd /tmp && GPU_MAX_HW_QUEUES=16 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/tools/ans_run.py 6 > $R/$O/kstats.log 2>&1
