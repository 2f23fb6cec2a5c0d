#!/bin/bash
# config 3 (64 x 1080p d1): several streaming pipelines per GPU (host threads)
export TMPDIR=/tmp
O=gpurun_out/${1:-r03x}
mkdir -p $O
for S in 1 2 3 4; do for Q in 16 32; do
  JXG_BENCH_HW_QUEUES=$Q timeout -k 10 300 python -u bench.py --config 3 --steps 6 --warmup 1 --streams $S --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/cfg3_s${S}_q$Q.log 2>&1
  python3 -c "import json; d=json.loads([l for l in open('$O/cfg3_s${S}_q$Q.log') if l.startswith('{')][-1]); print('streams $S queues $Q', d['value'])" >> $O/sum.log
done; done
