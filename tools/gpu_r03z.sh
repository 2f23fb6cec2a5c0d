#!/bin/bash
# early assembly in the streaming pipeline: stream tests, config 3, 8K
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03z}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --config 3 --steps 6 --warmup 1 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/cfg3.log 2>&1
JXG_LIB_PATH=$PWD/tools/var/libjxg_pprof.so timeout -k 10 300 python -u bench.py --config 3 --steps 4 --warmup 1 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/cfg3_pprof.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-quality --alt-thesis 0 > $O/bench8k.log 2>&1
