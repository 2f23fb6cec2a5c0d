#!/bin/bash
# stream tests, host profile of the lag-2 pipeline, 64 x 1080p bench: bash tools/gpu_r02t.sh TAG
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_configs.py -x -v --timeout 120 --timeout-method thread > $O/stream_tests.log 2>&1
bash tools/gpu_pprof.sh $1 tools/var/libjxg_pprof.so
timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --config 3 --steps 6 --warmup 3 > $O/cfg_batch_d1.0.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/bench_8k.log 2>&1
