#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r03u}
mkdir -p $O
JXG_SS_PROFILE=1 timeout -k 10 120 python -u tools/stream_probe.py --mode native --world 1 --h 544 --frames 300 --warmup 30 2>&1 | grep "mode\|rank" >> $O/probe.log
JXG_LIB_PATH=$PWD/tools/var/libjxg_pprof.so timeout -k 10 120 python -u tools/stream_probe.py --mode host --world 1 --h 544 --frames 300 --warmup 30 2>&1 | grep "mode\|profile" >> $O/probe.log
