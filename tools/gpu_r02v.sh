#!/bin/bash
# stream tests + host profile + 64 x 1080p / 4K / 8K benches: bash tools/gpu_r02v.sh TAG
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 120 --timeout-method thread > $O/stream_tests.log 2>&1
JXG_LIB_PATH=$PWD/tools/var/libjxg_pprof.so timeout -k 10 120 python tools/stream_timing.py 1920 1080 96 ans > $O/pprof_1080p_ans.log 2>&1
B="python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0"
timeout -k 10 200 $B --config 3 --steps 6 --warmup 3 > $O/cfg_batch_d1.0.log 2>&1
timeout -k 10 200 $B --config 1 > $O/cfg_4k.log 2>&1
timeout -k 10 200 $B > $O/bench_8k.log 2>&1
