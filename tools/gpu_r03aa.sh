#!/bin/bash
# chain batches: stream / config / shard tests, config 3, 8K, 1/8 slice, A/B vs JXG_CHAIN_BATCH=0
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03aa}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_configs.py tests/test_gpu_shard.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
for B in 1 0; do
  JXG_CHAIN_BATCH=$B JXG_CHAIN_PROFILE=1 timeout -k 10 300 python -u bench.py --config 3 --steps 6 --warmup 1 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/cfg3_b$B.log 2>&1
  JXG_CHAIN_BATCH=$B JXG_CHAIN_PROFILE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/bench8k_b$B.log 2>&1
  JXG_CHAIN_BATCH=$B JXG_CHAIN_PROFILE=1 timeout -k 10 120 python -u tools/stream_probe.py --mode host --world 1 --h 544 --frames 300 --warmup 30 2>&1 | grep "mode\|chain" | sed "s/^/b$B /" >> $O/probe.log
done
