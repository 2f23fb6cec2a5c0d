#!/bin/bash
# consolidated copies: GPU suite, stream probes, default bench
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03r}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
for H in 544 4320; do for M in host native; do
  timeout -k 10 120 python -u tools/stream_probe.py --mode $M --world 1 --h $H --frames 200 --warmup 30 2>&1 | grep mode >> $O/probe.log
done; done
timeout -k 10 300 python -u bench.py --warmup 3 --no-cpu-baseline --no-quality > $O/bench.log 2>&1
