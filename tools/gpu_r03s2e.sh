#!/bin/bash
# is 64 x 1080p bound per process (HIP runtime / host) or per GPU (command processor)?
# one bench alone, then two concurrent bench processes on the same GPU
set -e
export TMPDIR=/tmp
O=gpurun_out/r03s2e
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 --config 3 --steps 16 --warmup 3"
JXG_PIPE_BATCH=1 timeout -k 10 200 $B > $O/one.log 2>&1
JXG_PIPE_BATCH=1 timeout -k 10 200 $B > $O/two_a.log 2>&1 &
A=$!
JXG_PIPE_BATCH=1 timeout -k 10 200 $B > $O/two_b.log 2>&1 &
Bp=$!
wait $A
wait $Bp
JXG_PIPE_BATCH=4 timeout -k 10 200 $B > $O/two_k4_a.log 2>&1 &
A=$!
JXG_PIPE_BATCH=4 timeout -k 10 200 $B > $O/two_k4_b.log 2>&1 &
Bp=$!
wait $A
wait $Bp
