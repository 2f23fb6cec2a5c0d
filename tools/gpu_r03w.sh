#!/bin/bash
# configs after the round-3 changes: 64x1080p (d1), 4K, 16384^2 P+F; 8-context
# sharded emulation of 8K over 8 (one process) vs the unsharded pipeline
export TMPDIR=/tmp
O=gpurun_out/${1:-r03w}
mkdir -p $O
timeout -k 10 300 python -u bench.py --config 3 --steps 6 --warmup 1 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/cfg3.log 2>&1
timeout -k 10 300 python -u bench.py --config 1 --warmup 3 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/cfg1.log 2>&1
timeout -k 10 300 python -u bench.py --config 4 --steps 4 --warmup 1 --proposals 3 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/cfg4.log 2>&1
for W in 2 4 8; do
  timeout -k 10 200 python -u tools/stream_probe.py --mode host --world $W --frames 60 --warmup 16 2>&1 | grep mode >> $O/emul.log
done
