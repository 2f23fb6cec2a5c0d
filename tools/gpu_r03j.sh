#!/bin/bash
# rANS chains on a high-priority stream: parity, then the one-process stream
# probe with and without it
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03j}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_shard.py -x -v --timeout 240 --timeout-method thread -k "ans or native or stream or config" --deselect tests/test_gpu_shard.py::test_multiprocess_streamed_frames > $O/tests.log 2>&1
for P in 1 0; do for W in 1 2; do for M in host native; do
  JXG_ANS_PRIO=$P timeout -k 10 120 python -u tools/stream_probe.py --mode $M --world $W --frames 60 2>&1 | grep mode | sed "s/^/prio $P /" >> $O/probe.log
done; done; done
