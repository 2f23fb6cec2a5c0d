#!/bin/bash
# the 8K-over-8 native stream test alone, chain priority on / off
export TMPDIR=/tmp
O=gpurun_out/${1:-r03k}
mkdir -p $O
T=tests/test_gpu_shard.py
JXG_ANS_PRIO=1 timeout -k 10 200 python -u -m pytest $T -x -v --timeout 150 --timeout-method thread -k "native_stream_8k or sharded_8k_ans" > $O/prio1.log 2>&1; echo "prio1 rc $?" >> $O/rc.log
JXG_ANS_PRIO=0 timeout -k 10 200 python -u -m pytest $T -x -v --timeout 150 --timeout-method thread -k "native_stream_8k or sharded_8k_ans" > $O/prio0.log 2>&1; echo "prio0 rc $?" >> $O/rc.log
