#!/bin/bash
# rANS chain variants: parity (ANS configs) and the one-at-a-time emit stage time
export TMPDIR=/tmp
O=gpurun_out/${1:-r03p}; shift
mkdir -p $O
for V in "$@"; do
  JXG_LIB_PATH=$PWD/tools/var/libjxg_$V.so timeout -k 10 200 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 150 --timeout-method thread -k ans > $O/tests_$V.log 2>&1 || { echo "$V tests failed" >> $O/sum.log; continue; }
  JXG_LIB_PATH=$PWD/tools/var/libjxg_$V.so timeout -k 10 120 python -u bench.py --no-pipeline --steps 8 --warmup 2 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/iso_$V.log 2>&1
  JXG_LIB_PATH=$PWD/tools/var/libjxg_$V.so timeout -k 10 150 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/pipe_$V.log 2>&1
  python3 -c "
import json
d=json.loads([l for l in open('$O/iso_$V.log') if l.startswith('{')][-1])
p=json.loads([l for l in open('$O/pipe_$V.log') if l.startswith('{')][-1])
print('$V', 'ms_emit', d['stages_ms']['ms_emit'], 'latency', d['ms_latency'], 'pipelined', p['value'], p.get('ans_chain'))" >> $O/sum.log
done
