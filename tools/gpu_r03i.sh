#!/bin/bash
# streamed shards in one process: native vs Python protocol, then kernel traces
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03i}
mkdir -p $O
for W in 1 2; do for M in host native; do
  timeout -k 10 120 python -u tools/stream_probe.py --mode $M --world $W --frames 40 >> $O/probe.log 2>&1
done; done
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_native -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/stream_probe.py --mode native --world 2 --frames 30 > $GRAFT_REPO_ROOT/$O/prof_native.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_host -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/stream_probe.py --mode host --world 2 --frames 30 > $GRAFT_REPO_ROOT/$O/prof_host.log 2>&1
