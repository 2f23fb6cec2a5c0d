#!/bin/bash
# merge_eval chunk 64 vs 256 (kernel stats + pipelined bench), and the host
# profile of the 1080p ANS pipeline (JXG_PIPE_PROFILE build)
set -e
export TMPDIR=/tmp
O=gpurun_out/r02s5
R=$PWD
mkdir -p $O
for round in 1 2; do
  for n in ch64 ch256; do
    cd /tmp && JXG_LIB_PATH=$R/tools/var/libjxg_$n.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/${n}_$round -o run --output-format csv -- python3 $R/tools/ans_run.py 6 > $R/$O/${n}_$round.log 2>&1
    cd $R
  done
done
for n in ch64 ch256; do
  JXG_LIB_PATH=$R/tools/var/libjxg_$n.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --alt-coder 0 --alt-thesis 0 > $O/bench_$n.log 2>&1
done
JXG_LIB_PATH=$R/tools/var/libjxg_pprof.so timeout -k 10 120 python tools/stream_timing.py 1920 1080 96 ans > $O/pprof_1080p.log 2>&1
JXG_LIB_PATH=$R/tools/var/libjxg_pprof.so timeout -k 10 120 python tools/stream_timing.py 7680 4320 40 ans > $O/pprof_8k.log 2>&1
