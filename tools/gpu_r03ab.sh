#!/bin/bash
# chain batches with deeper pipelines (lanes sharing hardware queues)
export TMPDIR=/tmp
O=gpurun_out/${1:-r03ab}
mkdir -p $O
for B in 0 1; do for L in 12 20 28; do
  JXG_CHAIN_BATCH=$B JXG_PIPE_MAX_LANES=$L JXG_PIPE_QUEUE_CAP=0 timeout -k 10 120 python -u tools/stream_probe.py --mode host --world 1 --h 544 --frames 300 --warmup 40 2>&1 | grep "mode" | sed "s/^/b$B L$L /" >> $O/probe.log
done; done
for B in 0 1; do for L in 12 24; do
  JXG_CHAIN_BATCH=$B JXG_PIPE_MAX_LANES=$L JXG_PIPE_QUEUE_CAP=0 timeout -k 10 300 python -u bench.py --config 3 --steps 6 --warmup 1 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/cfg3_b${B}_L$L.log 2>&1
  python3 -c "import json; d=json.loads([l for l in open('$O/cfg3_b${B}_L$L.log') if l.startswith('{')][-1]); print('cfg3 b$B L$L', d['value'])" >> $O/probe.log
done; done
